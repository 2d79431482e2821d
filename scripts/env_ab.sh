#!/usr/bin/env bash
# A/B of runtime knobs (environment variables) on the default bench, one line each
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/envab
i=0
for spec in "$@"; do
  i=$((i+1))
  env $spec timeout -k 10 240 python bench.py --cpu-sample 0 --steps 3 > gpurun_out/envab/$i.json 2> gpurun_out/envab/$i.err
  echo "$i $spec" >> gpurun_out/envab/index.txt
done
