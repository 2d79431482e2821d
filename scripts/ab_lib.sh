#!/usr/bin/env bash
# A/B of builds of libimsame_dev.so on one box, alternating:
#   gpurun -- bash scripts/ab_lib.sh TAG "name=path name2=path2 ..." [bench args]
# ("cur" = the tree's own imsame_amd/lib/libimsame_dev.so is always run first)
set -uo pipefail
TAG=${1:-ab}; LIBS=$2; shift 2
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2; do
  for nv in cur= $LIBS; do
    n=${nv%%=*}; v=${nv#*=}
    if [ -n "$v" ]; then export IMSAME_LIB_DEV=$PWD/$v; else unset IMSAME_LIB_DEV; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --e2e off "$@" > gpurun_out/ablib_${TAG}_${n}_$rep.json \
        2> gpurun_out/ablib_${TAG}_${n}_$rep.err
    rc=$?; echo "$n $rep rc=$rc" >> gpurun_out/ablib_${TAG}_steps.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
