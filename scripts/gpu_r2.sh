#!/usr/bin/env bash
# One GPU-box pass for round 2:  gpurun -- bash scripts/gpu_r2.sh <tag> [steps...]
# steps: tests newtests smoke bench prof pmc ; a step that fails with anything
# but pytest's "tests failed" (1) ends the script (no GPU work after a fault).
set -uo pipefail
TAG=${1:-x}; shift || true
STEPS=${*:-"tests smoke bench prof"}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {   # $1 = exit status, $2 = step
  echo "$2 rc=$1" >> gpurun_out/steps_${TAG}.txt
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2 (rc $1)"; exit "$1"; fi
}
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
             > gpurun_out/pytest_gpu_${TAG}.log 2>&1; ok_or_stop $? tests ;;
    newtests) timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 300 --timeout-method thread \
             -k "query_shards or path_arena or cli_devices or multi_device or full_c2 or lanes or c2_shape or e2e" \
             > gpurun_out/pytest_new_${TAG}.log 2>&1; ok_or_stop $? newtests ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
           ok_or_stop $? smoke ;;
    bench) timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
           ok_or_stop $? bench ;;
    e2e) timeout -k 10 900 python -u bench.py --cpu-sample 0 --steps 1 > gpurun_out/bench_e2e_${TAG}.json \
           2> gpurun_out/bench_e2e_${TAG}.err; ok_or_stop $? e2e ;;
    e2eb*) BR=${s#e2eb}; IMSAME_E2E_ARGS="${BR:+-batch_reads $BR}" timeout -k 10 900 python -u bench.py --cpu-sample 0 --steps 1 \
           --warmup 0 --e2e on > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    benchq) timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
           ok_or_stop $? benchq ;;
    seedl*) L=${s#seedl}; IMSAME_SEED_L1=$L timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off \
           > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    bud*) B=${s#bud}; IMSAME_SEED_BUDGET=$B timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off \
           > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    c3) timeout -k 10 600 python -u bench.py --config c3 --steps 2 --cpu-sample 0 --e2e off > gpurun_out/bench_c3_${TAG}.json \
           2> gpurun_out/bench_c3_${TAG}.err; ok_or_stop $? c3 ;;
    shard*) SH=${s#shard}; timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --shard ${SH/_//} --steps 5 \
           > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    ranks4) timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
             --master-port 29519 bench.py --gpus 4 --dist-backend gloo --device 0 --cpu-sample 0 --e2e off \
             > gpurun_out/bench_ranks4_${TAG}.json 2> gpurun_out/bench_ranks4_${TAG}.err; ok_or_stop $? ranks4 ;;
    ranks2) timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
             --master-port 29517 bench.py --gpus 2 --dist-backend gloo --device 0 --cpu-sample 0 --e2e off \
             > gpurun_out/bench_ranks2_${TAG}.json 2> gpurun_out/bench_ranks2_${TAG}.err; ok_or_stop $? ranks2 ;;
    lanes*) LN=${s#lanes}; LN=${LN%%_*}; SH=${s#lanes${LN}}; SH=${SH#_}
           IMSAME_LANES=$LN timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 5 ${SH:+--shard ${SH/_//}} \
           > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    nowin) IMSAME_NW_WINDOW=0 timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 5 \
           > gpurun_out/bench_nowin_${TAG}.json 2> gpurun_out/bench_nowin_${TAG}.err; ok_or_stop $? nowin ;;
    syncup) timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 5 --upload sync \
           > gpurun_out/bench_syncup_${TAG}.json 2> gpurun_out/bench_syncup_${TAG}.err; ok_or_stop $? syncup ;;
    bench5) timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 5 \
           > gpurun_out/bench5_${TAG}.json 2> gpurun_out/bench5_${TAG}.err; ok_or_stop $? bench5 ;;
    onepass) IMSAME_NW_ONEPASS=1 timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 5 \
           > gpurun_out/bench_onepass_${TAG}.json 2> gpurun_out/bench_onepass_${TAG}.err; ok_or_stop $? onepass ;;
    band*) BW=${s#band}; IMSAME_NW_BAND=$BW timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 5 \
           > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    nwprof) IMSAME_NW_PROF=1 IMSAME_LANES=1 timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off --steps 1 --warmup 1 \
           > gpurun_out/bench_nwprof_${TAG}.json 2> gpurun_out/bench_nwprof_${TAG}.err; ok_or_stop $? nwprof ;;
    nwprof1) IMSAME_NW_ONEPASS=1 IMSAME_NW_PROF=1 IMSAME_LANES=1 timeout -k 10 600 python -u bench.py --cpu-sample 0 --e2e off \
           --steps 1 --warmup 1 > gpurun_out/bench_nwprof1_${TAG}.json 2> gpurun_out/bench_nwprof1_${TAG}.err; ok_or_stop $? nwprof1 ;;
    pmcsq) timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
             --kernel-include-regex 'nw16_kernel|seed_' -T -d gpurun_out/pmc_${TAG}_p1 -o pmc --output-format csv \
             -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --e2e off > gpurun_out/pmc_${TAG}_p1.json \
             2> gpurun_out/pmc_${TAG}_p1.err; ok_or_stop $? pmcsq ;;
    w5) IMSAME_LIB_DEV=$PWD/imsame_amd/lib/alt/libimsame_dev_w5.so timeout -k 10 600 python -u bench.py --cpu-sample 0 \
           --e2e off --steps 5 > gpurun_out/bench_w5_${TAG}.json 2> gpurun_out/bench_w5_${TAG}.err; ok_or_stop $? w5 ;;
    clitests) timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_avav.py -m gpu -v --timeout 300 --timeout-method thread \
             -k "cli or driver or multi_device" > gpurun_out/pytest_cli_${TAG}.log 2>&1; ok_or_stop $? clitests ;;
    nwtests) timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 300 --timeout-method thread \
             -k "two_pass or nw_pairs or nw_packed or c2_shape or e2e or lanes or path_arena or async_query or shards" \
             > gpurun_out/pytest_nw_${TAG}.log 2>&1; ok_or_stop $? nwtests ;;
    c5) timeout -k 10 600 python -u bench.py --config c5 --steps 1 --warmup 0 > gpurun_out/bench_c5_${TAG}.json \
           2> gpurun_out/bench_c5_${TAG}.err; ok_or_stop $? c5 ;;
    c5wprof) timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_c5w_${TAG} -o kt --output-format csv \
            -- python3 bench.py --config c5w --steps 1 --warmup 0 > gpurun_out/bench_c5wprof_${TAG}.json \
            2> gpurun_out/bench_c5wprof_${TAG}.err; ok_or_stop $? c5wprof ;;
    c5w) timeout -k 10 900 python -u bench.py --config c5w --steps 1 --warmup 0 > gpurun_out/bench_c5w_${TAG}.json \
           2> gpurun_out/bench_c5w_${TAG}.err; ok_or_stop $? c5w ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_${TAG} -o kt --output-format csv \
            -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --e2e off > gpurun_out/bench_prof_${TAG}.json \
            2> gpurun_out/bench_prof_${TAG}.err; ok_or_stop $? prof ;;
    pmc) i=0
         for grp in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
                    "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE"; do
           i=$((i+1))
           timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex 'nw16_kernel|seed_' -T \
             -d gpurun_out/pmc_${TAG}_p$i -o pmc --output-format csv \
             -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --e2e off > gpurun_out/pmc_${TAG}_p$i.json \
             2> gpurun_out/pmc_${TAG}_p$i.err
           ok_or_stop $? pmc$i
         done ;;
  esac
done
