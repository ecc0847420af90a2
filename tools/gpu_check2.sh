# full GPU test tier, 2-rank gloo-on-device bench (piecewise-graph path), DistilBERT bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NDP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 5 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err && cat gpurun_out/bench_gloo2.json || { tail -20 gpurun_out/bench_gloo2.err; exit 1; }
timeout -k 10 300 python bench.py --model distilbert --rank 8 --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.err && cat gpurun_out/bench_bert.json
