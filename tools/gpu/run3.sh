set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_direct.py tests/test_conv_bnstats_gpu.py -q -s --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1; tail -2 $O/pytest.log; grep -E "rel err" $O/pytest.log | head -4; grep -E "^FAILED|AssertionError: |^E  +assert" $O/pytest.log | head
tools/gpu/bench.sh $O "b512|" || exit 1
tools/gpu/pmc.sh $O wino > /dev/null && grep -E "wino" $O/pmc_wino.md
