cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/iso; mkdir -p $O
(cd _r2 && timeout -k 10 300 python -u -m pytest tests/test_conv_gemm.py -q --timeout 200 --timeout-method thread > $O/r2.log 2>&1; echo "r2 rc=$?"; tail -2 $O/r2.log)
timeout -k 10 300 python -u -m pytest tests/test_conv_gemm.py -q --timeout 200 --timeout-method thread > $O/r3.log 2>&1; echo "r3 rc=$?"; tail -2 $O/r3.log
