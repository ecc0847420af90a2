set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_linear_gpu.py tests/test_embedding_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lin.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_lin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag_bert_graph_vs_eager.py 10 powersgd > gpurun_out/diag5.log 2>&1; rc=$?; tail -12 gpurun_out/diag5.log; exit $rc
