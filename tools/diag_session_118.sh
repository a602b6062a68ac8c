set -u -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
DIAG_STEP=13 timeout -k 10 300 python tools/diag_parity.py dual_arm 256 100 4 118 > gpurun_out/r03/diag_118_t13.log 2>&1 && \
DIAG_STEP=12 timeout -k 10 300 python tools/diag_parity.py dual_arm 256 100 4 118 > gpurun_out/r03/diag_118_t12.log 2>&1
echo rc=$?
