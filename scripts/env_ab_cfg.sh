#!/usr/bin/env bash
# A/B of runtime knobs on one bench config: env_ab_cfg.sh <config> "<VAR=v ...>" ...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
CFG=$1; shift
mkdir -p gpurun_out/envab_${CFG}
i=0
for spec in "$@"; do
  i=$((i+1))
  env $spec timeout -k 10 300 python bench.py --config ${CFG} --cpu-sample 0 --steps 2 --warmup 1 \
      > gpurun_out/envab_${CFG}/$i.json 2> gpurun_out/envab_${CFG}/$i.err
  echo "$i $spec" >> gpurun_out/envab_${CFG}/index.txt
done
