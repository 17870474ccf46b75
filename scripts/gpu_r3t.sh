#!/bin/bash
# Round 3: host-inclusive rates (1M and 4M config-2 literals, pageable and page-locked) and the
# per-call latency table on the current library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3t}; mkdir -p $OUT
timeout -k 10 300 python scripts/host_rate.py 1000000 10 > $OUT/host_rate.jsonl 2> $OUT/host_rate.err || { echo "host_rate failed"; tail $OUT/host_rate.err; exit 1; }
timeout -k 10 300 python scripts/host_rate.py 4000000 5 >> $OUT/host_rate.jsonl 2>> $OUT/host_rate.err || { echo "host_rate 4M failed"; tail $OUT/host_rate.err; exit 1; }
cat $OUT/host_rate.jsonl
timeout -k 10 400 python scripts/latency.py > $OUT/latency.jsonl 2> $OUT/latency.err || { echo "latency failed"; tail $OUT/latency.err; exit 1; }
cat $OUT/latency.jsonl
echo "exit 0"
