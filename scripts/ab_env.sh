#!/usr/bin/env bash
# A/B of environment settings on one box, alternating:
#   gpurun -- bash scripts/ab_env.sh TAG "nameA:VAR=1,VAR2=2 nameB:VAR=0" [bench args]
set -uo pipefail
TAG=${1:-ab}; SETS=$2; shift 2
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2; do
  for ns in $SETS; do
    n=${ns%%:*}; e=${ns#*:}
    env ${e//,/ } timeout -k 10 300 python -u bench.py --cpu-sample 0 --e2e off "$@" > gpurun_out/abenv_${TAG}_${n}_$rep.json \
        2> gpurun_out/abenv_${TAG}_${n}_$rep.err
    rc=$?; echo "$n $rep rc=$rc" >> gpurun_out/abenv_${TAG}_steps.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
