#!/bin/bash
# Decode time of config 2 (and config 3 unless NO3) with each variant library (LIBS: names of
# loona_amd/libhpk_NAME.so; "product" = libhpk.so), with a kernel trace per library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-lib}
for l in ${LIBS:-product}; do
  if [ "$l" = product ]; then L=loona_amd/libhpk.so; else L=loona_amd/libhpk_$l.so; fi
  HPK_LIB=$L timeout -k 10 200 python3 scripts/dec_time.py config2 50 | sed "s/^{/{\"lib\": \"$l\", /" >> $OUT/libv_$TAG.jsonl || exit 1
  if [ -z "$NO3" ]; then
    HPK_LIB=$L timeout -k 10 200 python3 scripts/dec_time.py config3 10 | sed "s/^{/{\"lib\": \"$l\", /" >> $OUT/libv_$TAG.jsonl || exit 2
  fi
  HPK_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/libv_$TAG/$l -o run -- python3 scripts/dec_time.py config2 50 > $OUT/libv_${TAG}_$l.log 2>&1 || exit 3
done
echo "exit 0"
