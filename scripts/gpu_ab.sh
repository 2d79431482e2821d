#!/usr/bin/env bash
# A/B benches on one GPU box:
#   gpurun -- bash scripts/gpu_ab.sh TAG name:VAR=v,VAR=v name2: name3@0/8:VAR=v ...
# each variant = bench.py --cpu-sample 0 --e2e off --steps 5 under its env
# (name@R/N: the shard R of N, one rank's work of an N-GPU run); stops at the
# first failing run (no GPU work after a fault).
set -uo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  shard=""
  case $name in *@*) shard="--shard ${name#*@}"; name=${name%@*}_$(echo ${shard#--shard } | tr / _) ;; esac
  case $name in sync*) shard="$shard --upload sync" ;; esac
  IFS=',' read -ra kv <<< "$envs"
  env "${kv[@]}" timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 5 $shard \
      > gpurun_out/ab_${TAG}_${name}.json 2> gpurun_out/ab_${TAG}_${name}.err
  rc=$?; echo "$name rc=$rc" >> gpurun_out/ab_${TAG}.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
