set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
O=gpurun_out/small_ops_r6l.txt
for envs in "X=1" "HSA_ENABLE_SDMA=1" "GPU_FORCE_BLIT_COPY_SIZE=0" "HSA_FORCE_SDMA_SIZE=1" "HSA_ENABLE_SDMA_COPY_SIZE_OVERRIDE=1"; do
  echo "$envs $(env $envs timeout -k 10 120 ./scripts/micro/small_ops 2000000)" >> $O || exit 1
done
