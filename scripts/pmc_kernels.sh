#!/usr/bin/env bash
# PMC passes (one counter group per run) over one bench step, seed + NW kernels only.
set -euo pipefail
TAG=${1:-pmc}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex 'seed_kernel|nw16_kernel' -T -d gpurun_out/${TAG}_p$i -o pmc --output-format csv \
      -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/${TAG}_p$i.json 2> gpurun_out/${TAG}_p$i.err
  echo "pass $i ok" >> gpurun_out/${TAG}_steps.txt
done
