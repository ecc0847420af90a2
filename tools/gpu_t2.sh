set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_conv_gemm.py::test_resnet18_native_convs_vs_fp64"
for cfg in "NDP_BN_SINGLE=1" "NDP_BN_SINGLE_MAX=4" "NDP_BN_SINGLE=0"; do
  env $cfg timeout -k 10 200 python -u -m pytest $T -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; grep "^E .*Assert" gpurun_out/t2.log | head -3; tail -1 gpurun_out/t2.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
