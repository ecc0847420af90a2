# stem paired-k + float4 weight staging (round 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_conv_direct.py tests/test_conv_bnstats_gpu.py tests/test_stem_pool_gpu.py -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; grep -E "^FAILED|AssertionError: |^E  +assert" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/diag/stem_psplit.py > $O/stem_psplit.jsonl 2> $O/stem_psplit.err || { tail -5 $O/stem_psplit.err; exit 1; }
cat $O/stem_psplit.jsonl
tools/gpu/bench.sh $O "b512|" "b64|--global-batch 64" || exit 1
