#!/usr/bin/env bash
# A/B of device-library variants built into imsame_amd/lib/var/ (one bench each)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/var
for v in "$@"; do
  IMSAME_LIB_DEV=$PWD/imsame_amd/lib/var/libimsame_dev_$v.so timeout -k 10 240 python bench.py --cpu-sample 0 --steps 3 > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err
  echo "$v ok" >> gpurun_out/var/steps.txt
done
