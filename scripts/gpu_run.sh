#!/bin/bash
# One parameterised GPU pass (replaces the round-3 gpu_r3*.sh one-offs). Steps are chosen by STEPS
# (space-separated, run in order, the first failure ends the call):
#   test       the -m gpu parity suite (pytest, per-test timeout)
#   smoke      __graft_entry__.smoke()
#   ab         dec_time.py over WLS x LIBS, ROUNDS alternating rounds (one process per run)
#   modes      diagnostic variants of the wave kernel (libhpk_diag.so, HPK_DEBUG_MODE in MODES, default 0 1 2) on WLS
#   pmc        FETCH_SIZE / WRITE_SIZE / SQ passes of dec_time.py on WLS (separate rocprofv3 runs; with
#              HPK_COMPACT=1 the compacted form, summaries named pmc_compact_*)
#   lds        LDS bank-conflict attribution: SQ counters of libhpk_diag.so modes 0 8 9 10 on config 5
#   trace      rocprofv3 --kernel-trace --stats of a short bench run
#   bench      bench.py (reads the pmc summaries of this OUT when present; BENCH_ARGS after, so
#              BENCH_ARGS="--pmc-dir profiles" reads the committed ones)
# Output under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}; mkdir -p $OUT
WLS=${WLS:-config5}
LIBS=${LIBS:-libhpk.so}
kernel_of() { echo ${DECODE_KERNEL_NAME:-hpk_decode_wave}; }  # (round 6: the wave kernel decodes every batch)
lits_of() { case $1 in config5) echo 32000000;; c2_4m) echo 4000000;; *) echo 1000000;; esac; }
for step in ${STEPS:-test}; do
  case $step in
  test)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
    tail -3 $OUT/pytest_gpu.log ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
    tail -2 $OUT/smoke.log ;;
  ab)
    for wl in $WLS; do for r in $(seq ${ROUNDS:-2}); do for lib in $LIBS; do
      HPK_LIB=loona_amd/$lib timeout -k 10 180 python scripts/dec_time.py $wl ${REPS:-20} >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl $lib failed"; tail -20 $OUT/dec_time.err; exit 1; }
    done; done; done
    python3 -c "
import json
for l in open('$OUT/dec_time.jsonl'):
    d = json.loads(l); print(d['workload'], d['lib'], d['debug_mode'], d['decode_us'], d['checked'])" ;;
  modes)
    for wl in $WLS; do for r in $(seq ${ROUNDS:-2}); do for m in ${MODES:-0 1 2}; do
      HPK_LIB=loona_amd/libhpk_diag.so HPK_DEBUG_MODE=$m timeout -k 10 180 python scripts/dec_time.py $wl ${REPS:-20} >> $OUT/modes.jsonl 2>>$OUT/modes.err || { echo "modes $wl $m failed"; tail -20 $OUT/modes.err; exit 1; }
    done; done; done
    cat $OUT/modes.jsonl ;;
  pmc)
    SQ=${SQ:-"SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"}
    for wl in $WLS; do
      k=$(kernel_of $wl); n=$(lits_of $wl)
      for lib in $LIBS; do
        sfx=${lib#libhpk}; sfx=${sfx%.so}; pre=${HPK_COMPACT:+compact_}; d=$OUT/pmc_${pre}${wl}${sfx}
        HPK_LIB=loona_amd/$lib timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- python3 scripts/dec_time.py $wl 10 > $d.log 2>&1 &&
        HPK_LIB=loona_amd/$lib timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- python3 scripts/dec_time.py $wl 10 >> $d.log 2>&1 &&
        HPK_LIB=loona_amd/$lib timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc_sq_${pre}${wl}${sfx} -o run -- python3 scripts/dec_time.py $wl 10 >> $d.log 2>&1 || { echo "pmc $wl $lib failed"; tail $d.log; exit 1; }
        python3 scripts/pmc_traffic.py $d $n $wl ${KERNEL:-$k} > $d.json &&
        python3 scripts/pmc_sq.py $OUT/pmc_sq_${pre}${wl}${sfx} $n $wl ${KERNEL:-$k} > $OUT/pmc_sq_${pre}${wl}${sfx}.json || { echo "pmc summary $wl failed"; exit 1; }
        cat $d.json $OUT/pmc_sq_${pre}${wl}${sfx}.json
      done
    done ;;
  lds)
    # LDS bank-conflict attribution (libhpk_diag.so modes 8/9/10: the table reads / the window read / the
    # byte stores of the body step issued twice) against the product's counters (mode 0), config 5
    SQ=${SQ:-"SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"}
    for m in ${MODES:-0 8 9 10}; do
      HPK_LIB=loona_amd/libhpk_diag.so HPK_DEBUG_MODE=$m timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/lds_m$m -o run -- python3 scripts/dec_time.py config5 10 > $OUT/lds_m$m.log 2>&1 || { echo "lds mode $m failed"; tail $OUT/lds_m$m.log; exit 1; }
      python3 scripts/pmc_sq.py $OUT/lds_m$m 32000000 config5 hpk_decode_wave > $OUT/lds_m$m.json || exit 1
      echo "mode $m"; cat $OUT/lds_m$m.json
    done ;;
  trace)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_trace.log 2>&1 || { echo "trace failed"; tail $OUT/bench_trace.log; exit 1; }
    tail -1 $OUT/bench_trace.log ;;
  bench)
    timeout -k 10 600 python3 bench.py --pmc-dir $OUT ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
    cat $OUT/bench.json ;;
  *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "exit 0"
