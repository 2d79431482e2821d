#!/usr/bin/env bash
# Host-side sanitizer runs (CPU only -- GPU sanitizers are
# not available on the pool).  Logs go to $1 (default profiles/r4_sanitize/).
#
#  1. ThreadSanitizer and Address+UndefinedBehavior builds of the CLI's host
#     side (imsame_host.c, imsame_pipe.c) driven by tests/san/pipe_race.c
#     against a CPU stand-in for the device (tests/san/fake_dev.c: lanes on
#     their own threads handing over 3 pieces each, as the library does):
#     parallel FASTA parse vs serial, the threaded align/render/write pipeline
#     (per-thread pwrite at computed offsets into fallocate'd ranges) vs one
#     thread, pipe_render_range with 5 threads, a write that fails part-way;
#     each build with IMSAME_ONE_WRITER off and on, and one piece per lane.
#  2. Address+UndefinedBehavior builds of the oracle (lib + CLI binary), the
#     wave emulator and libimsame_host.so, loaded by the whole CPU test suite
#     (IMSAME_ORACLE_LIB / IMSAME_ORACLE_BIN / IMSAME_EMU_LIB / IMSAME_LIB_HOST;
#     the sanitizer runtimes preloaded into the test processes).
#
#   bash scripts/sanitize.sh [OUTDIR] [pytest -k expression]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-profiles/r5_sanitize}
KEXPR=${2:-}
B=/tmp/imsame_san
mkdir -p "$OUT" "$B"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
HOST="imsame_amd/csrc/host/imsame_pipe.c imsame_amd/csrc/host/imsame_host.c"

echo "== 1. host pipeline: tsan, asan+ubsan" | tee "$OUT/pipe_race.log"
gcc -O1 -g -fno-omit-frame-pointer -fsanitize=thread -D_FILE_OFFSET_BITS=64 -Wall -o $B/pipe_race_tsan \
    tests/san/pipe_race.c tests/san/fake_dev.c $HOST -lpthread -lm
gcc -O1 $SAN -D_FILE_OFFSET_BITS=64 -Wall -o $B/pipe_race_asan tests/san/pipe_race.c tests/san/fake_dev.c $HOST \
    -lpthread -lm
# and with 4 KiB render pieces: ~1500 hand-offs to each part's writer thread
gcc -O1 -g -fno-omit-frame-pointer -fsanitize=thread -DRW_PIECE=4096 -D_FILE_OFFSET_BITS=64 -Wall \
    -o $B/pipe_race_tsan_small tests/san/pipe_race.c tests/san/fake_dev.c $HOST -lpthread -lm
for ow in 0 1; do
  for lp in 3 1; do
    echo "-- IMSAME_ONE_WRITER=$ow IMSAME_LANE_PARTS=$lp" | tee -a "$OUT/pipe_race.log"
    IMSAME_ONE_WRITER=$ow IMSAME_LANE_PARTS=$lp TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
        $B/pipe_race_tsan $B 2>&1 | tee -a "$OUT/pipe_race.log"
    IMSAME_ONE_WRITER=$ow IMSAME_LANE_PARTS=$lp TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
        $B/pipe_race_tsan_small $B 2>&1 | tee -a "$OUT/pipe_race.log"
    IMSAME_ONE_WRITER=$ow IMSAME_LANE_PARTS=$lp ASAN_OPTIONS="detect_leaks=1" UBSAN_OPTIONS="print_stacktrace=1" \
        $B/pipe_race_asan $B 2>&1 | tee -a "$OUT/pipe_race.log"
  done
done

echo "== 2. CPU suite with asan+ubsan oracle, emulator, host library" | tee "$OUT/cpu_suite_asan.log"
gcc -O2 $SAN -D_FILE_OFFSET_BITS=64 -D_LARGEFILE64_SOURCE -Wall -fPIC -shared -o $B/liboracle.so \
    oracle/imsame_oracle.c -lpthread -lm
gcc -O2 $SAN -D_FILE_OFFSET_BITS=64 -D_LARGEFILE64_SOURCE -Wall -DORACLE_MAIN -o $B/imsame_oracle \
    oracle/imsame_oracle.c -lpthread -lm
g++ -std=c++20 -O2 $SAN -fPIC -shared -pthread -Wall -Wno-unused-function -Wno-unknown-pragmas -x c++ \
    -o $B/libwave_emu.so tests/emu/wave_emu.cpp
gcc -O2 $SAN -Wall -fPIC -D_FILE_OFFSET_BITS=64 -shared -o $B/libimsame_host.so imsame_amd/csrc/host/imsame_host.c \
    -lpthread
export IMSAME_ORACLE_LIB=$B/liboracle.so IMSAME_ORACLE_BIN=$B/imsame_oracle IMSAME_EMU_LIB=$B/libwave_emu.so \
       IMSAME_LIB_HOST=$B/libimsame_host.so
# the uninstrumented python loads instrumented libraries: the runtimes go first
# (leak checking off: the interpreter's own allocations are not ours)
RT="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
set +e
rm -f "$OUT"/report.*
# reports go to files (a test process that aborts loses pytest's captured stderr)
env LD_PRELOAD="$RT" ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0:log_path=$PWD/$OUT/report" \
    UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:log_path=$PWD/$OUT/report" \
    python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider ${KEXPR:+-k "$KEXPR"} 2>&1 | tee -a "$OUT/cpu_suite_asan.log"
rc=${PIPESTATUS[0]}
set -e
(ls "$OUT"/report.* 2>/dev/null || true) | wc -l > "$OUT/sanitizer_reports.txt"
echo "pytest rc=$rc, sanitizer reports: $(cat "$OUT/sanitizer_reports.txt")" | tee -a "$OUT/cpu_suite_asan.log"
exit $rc
