set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_batchnorm_gpu.py tests/test_slablink_gpu.py tests/test_conv_bnstats_gpu.py tests/test_ragged_gpu.py -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1; tail -1 $O/pytest.log; grep -E "^FAILED|AssertionError: |^E  +assert" $O/pytest.log | head
tools/gpu/bench.sh $O "b64|--global-batch 64" "b128|--global-batch 128" "b512|" || exit 1
tools/gpu/bench.sh gpurun_out/r6 "b64pkw512|NDP_PSGD_PKW=512 --global-batch 64" "b512pkw512|NDP_PSGD_PKW=512" "b512pkw256|NDP_PSGD_PKW=256" || exit 1
