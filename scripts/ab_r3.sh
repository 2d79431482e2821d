#!/usr/bin/env bash
# A/B of NW launch forms on one box: gpurun -- bash scripts/ab_r3.sh TAG
# (each run under its own time limit; stops at the first failure)
set -uo pipefail
TAG=${1:-ab}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name, env..., -- bench args
    local name=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 300 python -u bench.py --cpu-sample 0 --e2e off "$@" \
        > gpurun_out/ab_${TAG}_${name}.json 2> gpurun_out/ab_${TAG}_${name}.err
    local rc=$?
    echo "$name rc=$rc" >> gpurun_out/ab_${TAG}_steps.txt
    [ $rc -eq 0 ] || exit $rc
}
HEAD="IMSAME_NW_PERSIST=1 IMSAME_NW_K=10 IMSAME_ROUND1B=0"
for rep in 1 2; do
  run sh8_head_$rep $HEAD -- --shard 0/8 --steps 20 --warmup 2
  run sh8_np10r1b_$rep IMSAME_NW_K=10 -- --shard 0/8 --steps 20 --warmup 2
  run sh8_def_$rep X=1 -- --shard 0/8 --steps 20 --warmup 2
  run sh8_np10_$rep IMSAME_NW_K=10 IMSAME_ROUND1B=0 -- --shard 0/8 --steps 20 --warmup 2
done
for rep in 1 2; do
  run c2_head_$rep $HEAD -- --steps 8 --warmup 2
  run c2_np10r1b_$rep IMSAME_NW_K=10 -- --steps 8 --warmup 2
  run c2_def_$rep X=1 -- --steps 8 --warmup 2
done
