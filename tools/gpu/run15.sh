# Winograd grad-W 4-wave reduction (round 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r15; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_direct.py tests/test_conv_gemm.py tests/test_ragged_gpu.py tests/test_conv_bnstats_gpu.py -q --timeout 200 --timeout-method thread -m gpu > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; grep -E "^FAILED|AssertionError: |^E  +assert" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
tools/gpu/bench.sh $O "b512|" "b64|--global-batch 64" "b128|--global-batch 128" "b256|--global-batch 256" || exit 1
