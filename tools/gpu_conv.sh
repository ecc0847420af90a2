set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_conv_direct.py tests/test_conv_gemm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_conv.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/conv_direct_bench.py > gpurun_out/conv_direct.txt 2>&1; cat gpurun_out/conv_direct.txt
NDP_CONV_VARIANT=1 timeout -k 10 200 python tools/conv_direct_bench.py > gpurun_out/conv_direct_v1.txt 2>&1; cat gpurun_out/conv_direct_v1.txt
