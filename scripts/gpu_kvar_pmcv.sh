#!/bin/bash
# SQ counters of named harness variants (one variant per process and per counter pass), on INPUT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-kpv}
INPUT=${INPUT:-config3}
timeout -k 10 300 python scripts/kinput.py $INPUT /tmp/kpv.bin > $OUT/kpv_$TAG.log 2>&1 || exit 1
for v in ${VARIANTS:-coop1_snake}; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC" \
             "SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_IFETCH SQ_INSTS_VSKIPPED SQ_BUSY_CU_CYCLES"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/kpv_$TAG/${v}_p$i -o run -- ./bench/kvariants /tmp/kpv.bin 3 $v >> $OUT/kpv_$TAG.log 2>&1 || exit 2
  done
  python3 scripts/pmc_summary.py $OUT/kpv_$TAG/${v}_p1 > $OUT/kpv_${TAG}_$v.txt
  for j in 2 3; do python3 scripts/pmc_summary.py $OUT/kpv_$TAG/${v}_p$j | tail -n +2 >> $OUT/kpv_${TAG}_$v.txt; done
done
echo "exit 0"
