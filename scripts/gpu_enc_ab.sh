#!/bin/bash
# Encode time of config 3 and config 2 with each variant library (LIBS: names of
# loona_amd/libhpk_NAME.so; "product" = libhpk.so), alternating, plus a kernel trace per library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-enc}
for l in ${LIBS:-product}; do
  if [ "$l" = product ]; then L=loona_amd/libhpk.so; else L=loona_amd/libhpk_$l.so; fi
  for wl in config3 config2; do
    HPK_LIB=$L timeout -k 10 200 python3 scripts/enc_time.py $wl 20 | sed "s/^{/{\"lib\": \"$l\", /" >> $OUT/enc_$TAG.jsonl || exit 1
  done
done
for l in $(echo ${LIBS:-product} | tr ' ' '\n' | sort -u); do
  if [ "$l" = product ]; then L=loona_amd/libhpk.so; else L=loona_amd/libhpk_$l.so; fi
  HPK_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/enc_$TAG/$l -o run -- python3 scripts/enc_time.py config3 20 > $OUT/enc_${TAG}_$l.log 2>&1 || exit 3
done
echo "exit 0"
