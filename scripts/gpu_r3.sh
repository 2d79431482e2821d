#!/usr/bin/env bash
# One GPU-box pass for round 3:  gpurun -- bash scripts/gpu_r3.sh <tag> [steps...]
# Every GPU step runs under its own time limit; a step that fails with anything
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
PYT="python -u -m pytest -v --timeout 600 --timeout-method thread"
BQ="--cpu-sample 0 --e2e off"
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 1500 $PYT tests -m gpu > gpurun_out/pytest_gpu_${TAG}.log 2>&1; ok_or_stop $? tests ;;
    # the GPU suite once with every reused device arena poisoned (IMSAME_DEBUG_POISON)
    poison) IMSAME_DEBUG_POISON=1 timeout -k 10 1500 $PYT tests -m gpu > gpurun_out/pytest_poison_${TAG}.log 2>&1
            ok_or_stop $? poison ;;
    t:*) K=${s#t:}; timeout -k 10 900 $PYT tests -m gpu -k "$K" > gpurun_out/pytest_sel_${TAG}.log 2>&1
         ok_or_stop $? "$s" ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
           ok_or_stop $? smoke ;;
    bench) timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
           ok_or_stop $? bench ;;
    bench20) timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20_${TAG}.json \
           2> gpurun_out/bench20_${TAG}.err; ok_or_stop $? bench20 ;;
    benchq) timeout -k 10 600 python -u bench.py $BQ --steps 5 > gpurun_out/benchq_${TAG}.json 2> gpurun_out/benchq_${TAG}.err
           ok_or_stop $? benchq ;;
    e2e) timeout -k 10 900 python -u bench.py --cpu-sample 0 --steps 1 --e2e on > gpurun_out/bench_e2e_${TAG}.json \
           2> gpurun_out/bench_e2e_${TAG}.err; ok_or_stop $? e2e ;;
    c3) timeout -k 10 900 python -u bench.py --config c3 --steps 2 --cpu-sample 0 --e2e off > gpurun_out/bench_c3_${TAG}.json \
           2> gpurun_out/bench_c3_${TAG}.err; ok_or_stop $? c3 ;;
    c5w) timeout -k 10 900 python -u bench.py --config c5w --steps 1 --warmup 0 > gpurun_out/bench_c5w_${TAG}.json \
           2> gpurun_out/bench_c5w_${TAG}.err; ok_or_stop $? c5w ;;
    shard*) SH=${s#shard}; timeout -k 10 600 python -u bench.py $BQ --shard ${SH/_//} --steps 5 \
           > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    lanes*) LN=${s#lanes}; LN=${LN%%_*}; SH=${s#lanes${LN}}; SH=${SH#_}
           IMSAME_LANES=$LN timeout -k 10 600 python -u bench.py $BQ --steps 5 ${SH:+--shard ${SH/_//}} \
           > gpurun_out/bench_${s}_${TAG}.json 2> gpurun_out/bench_${s}_${TAG}.err; ok_or_stop $? $s ;;
    avav) timeout -k 10 900 python -u scripts/bench_avav.py --reads 2000000 --text > gpurun_out/avav_${TAG}.json \
           2> gpurun_out/avav_${TAG}.err; ok_or_stop $? avav ;;
    nwprof) IMSAME_NW_PROF=1 IMSAME_LANES=1 timeout -k 10 600 python -u bench.py $BQ --steps 1 --warmup 1 \
           > gpurun_out/bench_nwprof_${TAG}.json 2> gpurun_out/bench_nwprof_${TAG}.err; ok_or_stop $? nwprof ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_${TAG} -o kt --output-format csv \
            -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --e2e off > gpurun_out/bench_prof_${TAG}.json \
            2> gpurun_out/bench_prof_${TAG}.err; ok_or_stop $? prof ;;
    profc3) timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_c3_${TAG} -o kt --output-format csv \
            -- python3 bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --e2e off > gpurun_out/bench_profc3_${TAG}.json \
            2> gpurun_out/bench_profc3_${TAG}.err; ok_or_stop $? profc3 ;;
    profc5w) timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_c5w_${TAG} -o kt --output-format csv \
            -- python3 bench.py --config c5w --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_profc5w_${TAG}.json \
            2> gpurun_out/bench_profc5w_${TAG}.err; ok_or_stop $? profc5w ;;
    # PMC passes, one counter group per run, the program directly after `--`
    pmc*) CFG=${s#pmc}; CFG=${CFG:-c2}; i=0
         for grp in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
                    "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE"; do
           i=$((i+1))
           timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-include-regex 'nw16_kernel|nw_kernel|seed_' -T \
             -d gpurun_out/pmc_${CFG}_${TAG}_p$i -o pmc --output-format csv \
             -- python3 bench.py --config $CFG --steps 1 --warmup 0 --cpu-sample 0 --e2e off \
             > gpurun_out/pmc_${CFG}_${TAG}_p$i.json 2> gpurun_out/pmc_${CFG}_${TAG}_p$i.err
           ok_or_stop $? pmc${CFG}$i
         done ;;
  esac
done
