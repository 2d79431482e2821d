#!/usr/bin/env bash
# > 4 Gbase database parity test alone, with a heartbeat
# under gpurun_out/ while the oracle builds its 4.4 Gbase index.
set -euo pipefail
TAG=${1:-x}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
(while true; do date >> gpurun_out/hb_${TAG}.txt; sleep 30; done) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread \
    -k wide_database --durations=0 > gpurun_out/pytest_wide_${TAG}.log 2>&1
