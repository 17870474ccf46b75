set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=v12 bash scripts/gpu_check.sh > gpurun_out/check_v12.log 2>&1 || { echo "check failed $?"; exit 1; }
bash scripts/gpu_diag4.sh || { echo "diag4 failed"; exit 1; }
TAG=v12 bash scripts/gpu_pmc_traffic.sh > gpurun_out/pmc_v12.out 2>&1
echo "all done $?"
