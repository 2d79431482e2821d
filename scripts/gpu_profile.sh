#!/usr/bin/env bash
# Benchmark + rocprofv3 passes on the GPU box (run through gpurun).
#   1. bench.py (default config)                       -> gpurun_out/bench_<tag>.json
#   2. kernel trace + stats of a 2-step bench          -> gpurun_out/prof_<tag>/
#   3. PMC FETCH_SIZE pass, 4. PMC WRITE_SIZE pass      -> gpurun_out/pmc_{fetch,write}_<tag>/
# Stops at the first failing step (set -e); every GPU step has its own limit.
set -euo pipefail
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
echo "bench ok" >> gpurun_out/steps_${TAG}.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_${TAG} -o kt --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err
echo "prof ok" >> gpurun_out/steps_${TAG}.txt
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -d gpurun_out/pmc_fetch_${TAG} -o pmc --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_pmc1_${TAG}.json 2> gpurun_out/bench_pmc1_${TAG}.err
echo "pmc fetch ok" >> gpurun_out/steps_${TAG}.txt
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -d gpurun_out/pmc_write_${TAG} -o pmc --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_pmc2_${TAG}.json 2> gpurun_out/bench_pmc2_${TAG}.err
echo "pmc write ok" >> gpurun_out/steps_${TAG}.txt
