#!/bin/bash
# Round 3: product-library decode times (config 3 / 2 / 5), each checked once against the strings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3r}; mkdir -p $OUT
for wl in ${WLS:-config3 config3 config2 config5}; do
  timeout -k 10 180 python scripts/dec_time.py $wl 20 >> $OUT/dec_time.jsonl 2>>$OUT/dec_time.err || { echo "dec_time $wl failed"; tail -20 $OUT/dec_time.err; exit 1; }
done
cat $OUT/dec_time.jsonl
echo "exit 0"
