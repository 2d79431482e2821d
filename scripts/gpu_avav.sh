#!/usr/bin/env bash
# GPU-box pass for the all-vs-all path: GPU tests, then the C4 job benchmark
# (no text at full size; with text at a reduced size).
#   gpurun -- bash scripts/gpu_avav.sh <tag>
set -euo pipefail
TAG=${1:-x}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
echo "tests ok" >> gpurun_out/steps_${TAG}.txt
timeout -k 10 600 python -u scripts/bench_avav.py > gpurun_out/avav_${TAG}.json 2> gpurun_out/avav_${TAG}.err
echo "avav ok" >> gpurun_out/steps_${TAG}.txt
timeout -k 10 600 python -u scripts/bench_avav.py --reads 200000 --text > gpurun_out/avav_text_${TAG}.json 2> gpurun_out/avav_text_${TAG}.err
echo "avav text ok" >> gpurun_out/steps_${TAG}.txt
