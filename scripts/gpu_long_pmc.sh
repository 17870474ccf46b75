#!/bin/bash
# Long-literal kernel study on one workload (WL, default config3): decode time with the product
# library, then SQ counter passes (one rocprofv3 run per pass, kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-lp}
WL=${WL:-config3}
timeout -k 10 200 python3 scripts/dec_time.py $WL 10 > $OUT/lp_$TAG.jsonl 2> $OUT/lp_$TAG.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/lp_$TAG/trace -o run -- python3 scripts/dec_time.py $WL 3 >> $OUT/lp_$TAG.err 2>&1 || exit 2
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS" \
           "SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VSKIPPED SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/lp_$TAG/p$i -o run -- python3 scripts/dec_time.py $WL 2 >> $OUT/lp_$TAG.err 2>&1 || exit 3
done
for j in 1 2 3; do python3 scripts/pmc_summary.py $OUT/lp_$TAG/p$j >> $OUT/lp_${TAG}.txt; done
echo "exit 0"
