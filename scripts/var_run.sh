set -euo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/var
for w in 3 5; do
  IMSAME_LIB_DEV=$PWD/imsame_amd/lib/var/libimsame_dev_w$w.so timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/var/w$w.json 2> gpurun_out/var/w$w.err
done
timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/var/w4.json 2> gpurun_out/var/w4.err
IMSAME_SPEC=8 timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/var/w4s8.json 2> gpurun_out/var/w4s8.err
IMSAME_SPEC=2 timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/var/w4s2.json 2> gpurun_out/var/w4s2.err
