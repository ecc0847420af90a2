# round-3 baseline on a fresh box: GPU tests, headline bench (b512, b64), RCCL 2-ranks-on-1-GPU probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3base
export TMPDIR=/tmp
O=gpurun_out/r3base
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > $O/b512.json 2> $O/b512.err && cat $O/b512.json || exit 1
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --global-batch 64 > $O/b64.json 2> $O/b64.err && cat $O/b64.json || exit 1
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 tools/probe_rccl_dup.py > $O/dup.log 2>&1
echo "dup rc=$?"; tail -20 $O/dup.log
