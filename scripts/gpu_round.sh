#!/usr/bin/env bash
# One GPU-box pass: VALU micro, GPU test suite, smoke, bench + kernel-trace stats.
#   gpurun -- bash scripts/gpu_round.sh <tag> [micro] [tests] [bench] [prof]
set -euo pipefail
TAG=${1:-x}; shift || true
STEPS=${*:-"micro tests bench prof"}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    micro) timeout -k 10 120 ./scripts/micro/valu_rate > gpurun_out/micro_${TAG}.txt 2>&1 ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 ;;
    diag) IMSAME_DEBUG_ROUNDS=1 timeout -k 10 300 python -u scripts/round_diag.py > gpurun_out/diag_${TAG}.log 2>&1 ;;
    newtests) timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c3_ or c5_" > gpurun_out/pytest_new_${TAG}.log 2>&1 ;;
    c3) timeout -k 10 600 python -u bench.py --config c3 --steps 2 > gpurun_out/bench_c3_${TAG}.json 2> gpurun_out/bench_c3_${TAG}.err ;;
    c5s) timeout -k 10 600 python -u bench.py --config c5 --reads 4000 --steps 1 --warmup 0 > gpurun_out/bench_c5s_${TAG}.json 2> gpurun_out/bench_c5s_${TAG}.err ;;
    c5) timeout -k 10 900 python -u bench.py --config c5 --steps 1 --warmup 0 > gpurun_out/bench_c5_${TAG}.json 2> gpurun_out/bench_c5_${TAG}.err ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 ;;
    bench) timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err ;;
    benchq) timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_${TAG} -o kt --output-format csv \
            -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err ;;
  esac
  echo "$s ok" >> gpurun_out/steps_${TAG}.txt
done
