#!/usr/bin/env bash
# One GPU-box pass for round 6:  gpurun -- bash scripts/gpu_r6.sh <tag> [steps...]
# A step "e:VAR=VAL,VAR2=VAL2:step" runs `step` with those variables set (its
# outputs get a suffix from them); "t:a+b" runs the GPU tests matching -k "a or b".  Every GPU step runs under its own time
# limit; a step that fails with anything but pytest's "tests failed" (1) ends
# the script (no GPU work after a fault).
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
run_step() {   # $1 = step, $2 = output suffix
  local s=$1 X=$2 O=gpurun_out
  # VARIANT=name: the device library built by `make -C imsame_amd/csrc variant NAME=name`
  if [ -n "${VARIANT:-}" ]; then export IMSAME_LIB_DEV=imsame_amd/lib/variants/libimsame_dev_${VARIANT}.so; fi
  case $s in
    tests) timeout -k 10 1500 $PYT tests -m gpu > $O/pytest_gpu_${TAG}$X.log 2>&1; ok_or_stop $? tests$X ;;
    # the GPU suite once with every reused device arena poisoned (IMSAME_DEBUG_POISON)
    poison) IMSAME_DEBUG_POISON=1 timeout -k 10 1500 $PYT tests -m gpu > $O/pytest_poison_${TAG}$X.log 2>&1
            ok_or_stop $? poison$X ;;
    t:*) K=${s#t:}; K=${K//+/ or }; timeout -k 10 900 $PYT tests -m gpu -k "$K" > $O/pytest_sel_${TAG}$X.log 2>&1; ok_or_stop $? "$s$X" ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_${TAG}$X.log 2>&1
           ok_or_stop $? smoke$X ;;
    bench) timeout -k 10 900 python -u bench.py > $O/bench_${TAG}$X.json 2> $O/bench_${TAG}$X.err; ok_or_stop $? bench$X ;;
    bench20) timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench20_${TAG}$X.json \
           2> $O/bench20_${TAG}$X.err; ok_or_stop $? bench20$X ;;
    benchq) timeout -k 10 600 python -u bench.py $BQ --steps 5 > $O/benchq_${TAG}$X.json 2> $O/benchq_${TAG}$X.err
           ok_or_stop $? benchq$X ;;
    e2e) timeout -k 10 900 python -u bench.py --cpu-sample 0 --steps 1 --e2e on > $O/bench_e2e_${TAG}$X.json \
           2> $O/bench_e2e_${TAG}$X.err; ok_or_stop $? e2e$X ;;
    # e2e with CLI flags: e2ef:-batch_reads+250000 (+ stands for a space)
    e2ef:*) F=${s#e2ef:}; F=${F//+/ }; FS=$(echo "$F" | tr -c 'a-z0-9\n' '_')
           IMSAME_E2E_ARGS="$F" timeout -k 10 900 python -u bench.py --cpu-sample 0 --steps 1 --e2e on \
           > $O/bench_e2e${FS}_${TAG}$X.json 2> $O/bench_e2e${FS}_${TAG}$X.err; ok_or_stop $? "e2e$FS$X" ;;
    c3) timeout -k 10 900 python -u bench.py --config c3 --steps 2 $BQ > $O/bench_c3_${TAG}$X.json \
           2> $O/bench_c3_${TAG}$X.err; ok_or_stop $? c3$X ;;
    # C3 with the oracle as the checker on 3 windows (parity + NW accounting) and the port as CPU baseline
    c3p) timeout -k 10 1100 python -u bench.py --config c3 --steps 2 --e2e off --cpu-kind port > $O/bench_c3p_${TAG}$X.json \
           2> $O/bench_c3p_${TAG}$X.err; ok_or_stop $? c3p$X ;;
    c5) timeout -k 10 900 python -u bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5_${TAG}$X.json \
           2> $O/bench_c5_${TAG}$X.err; ok_or_stop $? c5$X ;;
    c5w) timeout -k 10 900 python -u bench.py --config c5w --steps 1 --warmup 0 > $O/bench_c5w_${TAG}$X.json \
           2> $O/bench_c5w_${TAG}$X.err; ok_or_stop $? c5w$X ;;
    shard*) SH=${s#shard}; timeout -k 10 600 ${PINCMD:-} python -u bench.py $BQ --shard ${SH/_//} --steps 10 --warmup 2 \
           > $O/bench_${s}_${TAG}$X.json 2> $O/bench_${s}_${TAG}$X.err; ok_or_stop $? $s$X ;;
    avav) timeout -k 10 900 python -u scripts/bench_avav.py --reads 2000000 --text > $O/avav_${TAG}$X.json \
           2> $O/avav_${TAG}$X.err; ok_or_stop $? avav$X ;;
    nwprof) IMSAME_NW_PROF=1 IMSAME_LANES=1 timeout -k 10 600 python -u bench.py $BQ --steps 1 --warmup 1 \
           > $O/bench_nwprof_${TAG}$X.json 2> $O/bench_nwprof_${TAG}$X.err; ok_or_stop $? nwprof$X ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_${TAG}$X -o kt --output-format csv \
            -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --e2e off > $O/bench_prof_${TAG}$X.json \
            2> $O/bench_prof_${TAG}$X.err; ok_or_stop $? prof$X ;;
    profsh*) SH=${s#profsh}; timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_${s}_${TAG}$X -o kt \
            --output-format csv -- python3 bench.py --shard ${SH/_//} --steps 5 --warmup 1 --cpu-sample 0 --e2e off \
            > $O/bench_${s}_${TAG}$X.json 2> $O/bench_${s}_${TAG}$X.err; ok_or_stop $? $s$X ;;
    profc3) timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d $O/prof_c3_${TAG}$X -o kt --output-format csv \
            -- python3 bench.py --config c3 --steps 2 --warmup 1 --cpu-sample 0 --e2e off > $O/bench_profc3_${TAG}$X.json \
            2> $O/bench_profc3_${TAG}$X.err; ok_or_stop $? profc3$X ;;
    profc5w) timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d $O/prof_c5w_${TAG}$X -o kt --output-format csv \
            -- python3 bench.py --config c5w --steps 1 --warmup 0 --cpu-sample 0 > $O/bench_profc5w_${TAG}$X.json \
            2> $O/bench_profc5w_${TAG}$X.err; ok_or_stop $? profc5w$X ;;
    # PMC passes, one counter group per run, the program directly after `--`
    # (sqpmc<cfg>: the SQ group only)
    pmc*|sqpmc*) CFG=${s#sqpmc}; CFG=${CFG#pmc}; CFG=${CFG:-c2}; i=0
         GRPS=("SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
               "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE")
         [[ $s == sqpmc* ]] && GRPS=("${GRPS[0]}" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY")
         for grp in "${GRPS[@]}"; do
           i=$((i+1))
           timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-include-regex 'nw16_kernel|nw_kernel|nwl_kernel|nwp_kernel|seed_' -T \
             -d $O/pmc_${CFG}_${TAG}${X}_p$i -o pmc --output-format csv \
             -- python3 bench.py --config $CFG --steps 1 --warmup 0 --cpu-sample 0 --e2e off \
             > $O/pmc_${CFG}_${TAG}${X}_p$i.json 2> $O/pmc_${CFG}_${TAG}${X}_p$i.err
           ok_or_stop $? pmc${CFG}$i$X
         done ;;
    # nw16 first-sweep loop ceiling (scripts/micro/nw16_loop.py); MICRO_VALU / MICRO_WPS from the env
    micro) timeout -k 10 600 python -u scripts/micro/nw16_loop.py --valu ${MICRO_VALU:-351} \
             ${MICRO_WPS:+--waves-per-simd $MICRO_WPS} --out $O/micro_${TAG}$X.json > $O/micro_${TAG}$X.log 2>&1
           ok_or_stop $? micro$X ;;
    # small NW launches per form (scripts/micro/nw_small.py)
    nwsmall) IMSAME_NW_PROF=1 timeout -k 10 600 python -u scripts/micro/nw_small.py ${NWS_ARGS:-} --out $O/nwsmall_${TAG}$X.json \
             > $O/nwsmall_${TAG}$X.log 2>&1; ok_or_stop $? nwsmall$X ;;
    benchab) local Y=$X k=1; while [ -e $O/benchab_${TAG}$Y.json ]; do k=$((k+1)); Y=${X}_$k; done
           timeout -k 10 600 python -u bench.py $BQ --steps 10 --warmup 2 > $O/benchab_${TAG}$Y.json \
           2> $O/benchab_${TAG}$Y.err; ok_or_stop $? benchab$Y ;;
    # single-file write rates of this box's TMPDIR (scripts/micro/write_rate.c; host only)
    wrate) gcc -O2 -pthread -o /tmp/write_rate scripts/micro/write_rate.c && \
           timeout -k 10 300 /tmp/write_rate ${TMPDIR:-/tmp} 3 > $O/wrate_${TAG}$X.txt 2>&1; ok_or_stop $? wrate$X ;;
    *) echo "unknown step $s" >> $O/steps_${TAG}.txt ;;
  esac
}
dispatch() {   # $1 = step (maybe with e: / pN: prefixes), $2 = suffix so far
  local s=$1 X=$2
  if [[ $s == p[0-9]*:* ]]; then
    # pN:step -- the step pinned to the first N CPUs this process may use (the
    # host-thread budget one rank of an N-GPU run gets); suffix _pN
    local np=${s%%:*}; np=${np#p}; local inner=${s#*:}
    local cpus=$(python3 -c "import os;print(','.join(map(str,sorted(os.sched_getaffinity(0))[:$np])))")
    ( export PINCMD="taskset -c $cpus" IMSAME_HOST_THREADS=$np; dispatch "$inner" "${X}_p$np" ) || exit $?
  elif [[ $s == e:* ]]; then
    local spec=${s#e:}; local envs=${spec%%:*}; local inner=${spec#*:}
    local sfx="${X}_$(echo "$envs" | tr '=,' '__')"
    ( export ${envs//,/ }; dispatch "$inner" "$sfx" ) || exit $?
  else
    run_step "$s" "$X"
  fi
}
for s in $STEPS; do
  dispatch "$s" "" || exit $?
done
