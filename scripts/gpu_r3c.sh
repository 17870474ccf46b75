#!/bin/bash
# Round 3: first runs of the v25 wave-fill decode kernel: correctness on config 5 / config 2 / config 3
# (every byte checked against the generated strings) and its time against the v24 kernel, then the
# GPU parity suite (every case under both kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3c; mkdir -p $OUT
for wl in config5 config2 config3; do
  for k in wave fill; do
    HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=$k timeout -k 10 180 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl $k failed"; tail -20 $OUT/dec_time.err; exit 1; }
  done
done
cat $OUT/dec_time.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "exit 0"
