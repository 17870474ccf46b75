#!/bin/bash
# Round 3: the wave kernel after a change: correctness + time on config 5/2/3 (both kernels), per-wave
# phase stamps on config 5, then the GPU parity suite (every case under both kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3e}; mkdir -p $OUT
for wl in config5 config2 config3; do
  for k in wave fill; do
    HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=$k timeout -k 10 180 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl $k failed"; tail -20 $OUT/dec_time.err; exit 1; }
  done
done
for wl in config5 config2; do
  HPK_WAVE_ALT=1 HPK_LIB=loona_amd/libhpk_diag.so HPK_DECODE_KERNEL=wave timeout -k 10 180 python scripts/dec_time.py $wl 20 | sed 's/"kernel": "wave"/"kernel": "wave_alt"/' >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl alt failed"; tail -20 $OUT/dec_time.err; exit 1; }
done
cat $OUT/dec_time.jsonl
timeout -k 10 180 python scripts/wave_stamps.py config5 >> $OUT/stamps.jsonl 2>>$OUT/stamps.err || { echo "stamps failed"; tail -20 $OUT/stamps.err; exit 1; }
HPK_WAVE_ALT=1 timeout -k 10 180 python scripts/wave_stamps.py config5 | sed 's/"kernel": "wave"/"kernel": "wave_alt"/' >> $OUT/stamps.jsonl 2>>$OUT/stamps.err || { echo "stamps alt failed"; tail -20 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.jsonl
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
fi
HPK_HDEC_TIMING=1 timeout -k 10 300 python -c "
import json, torch, bench
from loona_amd import HuffmanCodec
c = HuffmanCodec(0, stream=torch.cuda.current_stream())
print(json.dumps(bench.run_config4(c, 16)))" > $OUT/config4.json 2> $OUT/config4.err || { echo "config4 failed"; tail $OUT/config4.err; exit 1; }
cat $OUT/config4.json; tail -4 $OUT/config4.err
echo "exit 0"
