#!/bin/bash
# Round 3 (session 2): GPU parity suite on the product library, per-wave stamps of the config-5
# decode (diagnostic build), then one bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s2}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u scripts/wave_stamps.py config5 > $OUT/stamps.jsonl 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
cat $OUT/stamps.jsonl
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "exit 0"
