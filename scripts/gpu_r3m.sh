#!/bin/bash
# Round 3 full pass on the product library: GPU parity suite, PMC traffic (FETCH_SIZE / WRITE_SIZE,
# separate passes) and SQ issue counters of the config-5 (wave) and config-2 (fill) decode launches,
# a rocprofv3 kernel-trace summary of the bench, then the bench line reading those summaries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3m}; mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
fi
SQ="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
for wl in config5 config2; do
  if [ $wl = config5 ]; then k=hpk_decode_wave; n=32000000; else k=hpk_decode12; n=1000000; fi
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$wl/fetch -o run -- python3 scripts/dec_time.py $wl 10 > $OUT/pmc_$wl.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$wl/write -o run -- python3 scripts/dec_time.py $wl 10 >> $OUT/pmc_$wl.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc_sq_$wl -o run -- python3 scripts/dec_time.py $wl 10 >> $OUT/pmc_$wl.log 2>&1 || { echo "pmc $wl failed"; tail $OUT/pmc_$wl.log; exit 1; }
  python3 scripts/pmc_traffic.py $OUT/pmc_$wl $n $wl $k > $OUT/pmc_$wl.json &&
  python3 scripts/pmc_sq.py $OUT/pmc_sq_$wl $n $wl $k > $OUT/pmc_sq_$wl.json || { echo "pmc summary $wl failed"; exit 1; }
  cat $OUT/pmc_$wl.json $OUT/pmc_sq_$wl.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_trace.log 2>&1 || { echo "trace failed"; tail $OUT/bench_trace.log; exit 1; }
timeout -k 10 600 python3 bench.py --pmc-dir $OUT > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "exit 0"
