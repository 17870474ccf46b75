#!/bin/bash
# HBM traffic of the bench's decode kernel from PMC counters (MI355X_MICROARCH.md, HBM section):
# FETCH_SIZE and WRITE_SIZE in separate passes (they do not fit one TCC pass), kernel-trace only,
# no runtime/sys trace. Summarised into profiles/pmc_decode.json by scripts/pmc_traffic.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-pmc}
rm -rf $OUT/pmc_$TAG
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG/fetch -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu > $OUT/pmc_$TAG.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$TAG/write -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu >> $OUT/pmc_$TAG.log 2>&1 || { echo "exit $?"; exit 1; }
# raw EA request counters (cross-check only; a missing counter ends the chain, not the summary)
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/pmc_$TAG/rdreq -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu >> $OUT/pmc_$TAG.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_$TAG/wrreq -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu >> $OUT/pmc_$TAG.log 2>&1
rc=$?
python3 scripts/pmc_traffic.py $OUT/pmc_$TAG 1000000 > $OUT/pmc_$TAG.json
echo "exit $rc"
exit $rc
