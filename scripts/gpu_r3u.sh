#!/bin/bash
# Round 3: where a host-pointer call's time goes (1M config-2 literals, page-locked): HIP API and
# kernel trace of scripts/host_rate.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3u}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run -- python3 scripts/host_rate.py 1000000 5 > $OUT/host_rate.jsonl 2> $OUT/host_rate.err || { echo "trace failed"; tail $OUT/host_rate.err; exit 1; }
cat $OUT/host_rate.jsonl
ls -la $OUT/trace
echo "exit 0"
