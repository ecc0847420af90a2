set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_direct.py tests/test_batchnorm_gpu.py tests/test_conv_gemm.py tests/test_models.py tests/test_ragged_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
tools/gpu/bench.sh $O "b512|" "b64|--global-batch 64" || exit 1
timeout -k 10 120 python tools/toeplitz_bench.py 512 > $O/toep512.md 2>&1 && cat $O/toep512.md
