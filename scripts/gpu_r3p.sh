#!/bin/bash
# Round 3: config 4 (captured HEADERS, one hpk_hdec_decode_blocks call) device vs CPU batch path,
# with the per-pass host times, then the GPU suite's block-decoder tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3p}; mkdir -p $OUT
HPK_HDEC_TIMING=1 timeout -k 10 300 python -c "
import json, torch, bench
from loona_amd import HuffmanCodec
c = HuffmanCodec(0, stream=torch.cuda.current_stream())
print(json.dumps(bench.run_config4(c, 16)))" > $OUT/config4.json 2> $OUT/config4.err || { echo "config4 failed"; tail $OUT/config4.err; exit 1; }
cat $OUT/config4.json; tail -12 $OUT/config4.err
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "block or hdec or hpack or interop" --timeout 200 --timeout-method thread > $OUT/pytest_blocks.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_blocks.log; exit 1; }
tail -3 $OUT/pytest_blocks.log
echo "exit 0"
