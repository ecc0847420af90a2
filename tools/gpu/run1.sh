set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_batchnorm_gpu.py tests/test_slablink_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r1/pytest.log 2>&1 || { tail -30 gpurun_out/r1/pytest.log; exit 1; }
tail -2 gpurun_out/r1/pytest.log
tools/gpu/bench.sh gpurun_out/r1 "b512|" "b512s|NDP_FUSION_OFF=bn_vec4" "b64|--global-batch 64" "b64s|NDP_FUSION_OFF=bn_vec4 --global-batch 64" || exit 1
timeout -k 10 120 python tools/toeplitz_bench.py 512 > gpurun_out/r1/toep512.md 2>&1 && timeout -k 10 120 python tools/toeplitz_bench.py 64 > gpurun_out/r1/toep64.md 2>&1
cat gpurun_out/r1/toep512.md gpurun_out/r1/toep64.md
