#!/usr/bin/env bash
# SQ instruction/cycle counters of one bench step (one counter group per pass).
set -euo pipefail
TAG=${1:-sq}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_WAVES" "SQ_INSTS_LDS SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -T -d gpurun_out/${TAG}_p$i -o pmc --output-format csv \
      -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/${TAG}_p$i.json 2> gpurun_out/${TAG}_p$i.err
  echo "pass $i ok" >> gpurun_out/${TAG}_steps.txt
done
