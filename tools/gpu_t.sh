# run given pytest node ids ($@) on the GPU box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_t.log | head -30
exit $rc
