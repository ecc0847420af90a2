set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NDP_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/piecewise_diag.py > gpurun_out/pwdiag.log 2>&1; rc=$?
grep rank gpurun_out/pwdiag.log | grep it; exit $rc
