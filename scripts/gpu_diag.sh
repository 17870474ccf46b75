#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-diag}
: > $OUT/diag_$TAG.jsonl
for m in 0 1 2 3; do
  HPK_DEBUG_MODE=$m timeout -k 10 300 python scripts/diag_decode.py >> $OUT/diag_$TAG.jsonl 2>> $OUT/diag_$TAG.err || exit $?
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  --output-format csv -d $OUT/pmc_$TAG/a -o run -- python3 scripts/diag_decode.py > $OUT/pmc_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/pmc_$TAG/b -o run -- python3 scripts/diag_decode.py >> $OUT/pmc_$TAG.log 2>&1
echo "exit $?"
