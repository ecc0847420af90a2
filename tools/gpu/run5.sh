set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_direct.py tests/test_conv_bnstats_gpu.py tests/test_batchnorm_gpu.py tests/test_slablink_gpu.py -q -s --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1; tail -2 $O/pytest.log; grep -E "rel err" $O/pytest.log | tail -6; grep -E "^FAILED|AssertionError: |^E  +assert" $O/pytest.log | head
tools/gpu/bench.sh $O "b512|" "b256|--global-batch 256" "b64|--global-batch 64" || exit 1
