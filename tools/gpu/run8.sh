# BN apply prefetch A/B (round 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_batchnorm_gpu.py tests/test_conv_bnstats_gpu.py tests/test_stem_pool_gpu.py tests/test_slablink_gpu.py tests/test_bn_pair_gpu.py -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; grep -E "^FAILED|AssertionError: |^E  +assert" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
tools/gpu/bench.sh $O "b512|" "b64|--global-batch 64" "b256|--global-batch 256" || exit 1
