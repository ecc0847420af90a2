set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_embedding_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_emb.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_emb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag_graph.py --model distilbert --rank 8 --steps 30 > gpurun_out/diag3.log 2>&1; rc=$?
grep -v "^frame\|^  \|^$" gpurun_out/diag3.log | tail -8; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r2_refcfg.sh
