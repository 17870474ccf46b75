#!/bin/bash
# Encode measurements on the GPU box (config 3 unless WLS says otherwise), output under gpurun_out/$TAG:
#   time   enc_time.py over LIBS, ROUNDS alternating rounds (one process per run)
#   prof   per-phase cycles of hpk_encode2 (libhpk_diag.so, HPK_ENCODE_CFG=9; scripts/enc_prof.py)
#   pmc    FETCH_SIZE / WRITE_SIZE / SQ passes of enc_time.py for hpk_encode2 (separate rocprofv3 runs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-enc}; mkdir -p $OUT
WLS=${WLS:-config3}
LIBS=${LIBS:-libhpk.so}
for step in ${STEPS:-time}; do
  case $step in
  time)
    for wl in $WLS; do for r in $(seq ${ROUNDS:-3}); do for lib in $LIBS; do
      HPK_LIB=loona_amd/$lib timeout -k 10 180 python scripts/enc_time.py $wl ${REPS:-20} >> $OUT/enc_time.jsonl 2>>$OUT/enc_time.err || { echo "enc_time $wl $lib failed"; tail -20 $OUT/enc_time.err; exit 1; }
    done; done; done
    cat $OUT/enc_time.jsonl ;;
  prof)
    for wl in $WLS; do
      timeout -k 10 180 python scripts/enc_prof.py $wl >> $OUT/enc_prof.jsonl 2>>$OUT/enc_prof.err || { echo "enc_prof $wl failed"; tail -20 $OUT/enc_prof.err; exit 1; }
    done
    cat $OUT/enc_prof.jsonl ;;
  pmc)
    SQ=${SQ:-"SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"}
    for wl in $WLS; do for lib in $LIBS; do
      sfx=${lib#libhpk}; sfx=${sfx%.so}; d=$OUT/pmc_enc_${wl}${sfx}
      HPK_LIB=loona_amd/$lib timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- python3 scripts/enc_time.py $wl 10 > $d.log 2>&1 &&
      HPK_LIB=loona_amd/$lib timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- python3 scripts/enc_time.py $wl 10 >> $d.log 2>&1 &&
      HPK_LIB=loona_amd/$lib timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d ${d}_sq -o run -- python3 scripts/enc_time.py $wl 10 >> $d.log 2>&1 || { echo "pmc $wl $lib failed"; tail $d.log; exit 1; }
      python3 scripts/pmc_traffic.py $d 1000000 $wl hpk_encode2 > $d.json &&
      python3 scripts/pmc_sq.py ${d}_sq 1000000 $wl hpk_encode2 > ${d}_sq.json || { echo "pmc summary $wl failed"; exit 1; }
      cat $d.json ${d}_sq.json
    done; done ;;
  *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "exit 0"
