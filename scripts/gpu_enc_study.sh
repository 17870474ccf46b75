#!/bin/bash
# Encode study: encode time on config 3 and config 2 (lengths checked), then SQ counter passes of
# hpk_encode2 on config 3 (one rocprofv3 run per pass, kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-es}
timeout -k 10 200 python3 scripts/enc_time.py config3 10 > $OUT/es_$TAG.jsonl 2> $OUT/es_$TAG.err || exit 1
timeout -k 10 200 python3 scripts/enc_time.py config2 20 >> $OUT/es_$TAG.jsonl 2>> $OUT/es_$TAG.err || exit 2
if [ -z "$NO_PMC" ]; then
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS" \
           "SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VSKIPPED SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/es_$TAG/p$i -o run -- python3 scripts/enc_time.py config3 2 >> $OUT/es_$TAG.err 2>&1 || exit 3
done
for j in 1 2 3; do PMC_FILTER=encode python3 scripts/pmc_summary.py $OUT/es_$TAG/p$j >> $OUT/es_${TAG}.txt; done
fi
echo "exit 0"
