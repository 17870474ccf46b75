#!/bin/bash
# Round 3: small-call latency trace (1k / 5k literals, synchronous, device-resident) with the HIP
# API and kernel traces, split into parts; then config 4 (block decoder, device vs CPU batch path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3q}; mkdir -p $OUT
timeout -k 10 120 python scripts/lat_trace.py 200 > $OUT/lat_plain.jsonl 2> $OUT/lat_plain.err || { echo "lat failed"; tail $OUT/lat_plain.err; exit 1; }
cat $OUT/lat_plain.jsonl
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/lat_trace -o run -- python3 scripts/lat_trace.py 200 > $OUT/lat_traced.jsonl 2> $OUT/lat_traced.err || { echo "lat trace failed"; tail $OUT/lat_traced.err; exit 1; }
cat $OUT/lat_traced.jsonl
python3 scripts/lat_split.py $OUT/lat_trace 200 > $OUT/lat_split.jsonl || exit 1
cat $OUT/lat_split.jsonl
rm -rf $OUT/lat_trace/*/*hip_api_trace.csv.gz 2>/dev/null
HPK_HDEC_TIMING=1 timeout -k 10 300 python -c "
import json, torch, bench
from loona_amd import HuffmanCodec
c = HuffmanCodec(0, stream=torch.cuda.current_stream())
print(json.dumps(bench.run_config4(c, 16)))" > $OUT/config4.json 2> $OUT/config4.err || { echo "config4 failed"; tail $OUT/config4.err; exit 1; }
cat $OUT/config4.json; tail -6 $OUT/config4.err
echo "exit 0"
