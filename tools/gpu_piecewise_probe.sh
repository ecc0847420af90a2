# probe: piecewise graph at N=1, and the 2-rank gloo-on-device bench with/without graphs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --graph-mode piecewise > gpurun_out/pw1.json 2> gpurun_out/pw1.err && cat gpurun_out/pw1.json &&
NDP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --graph-mode none > gpurun_out/gloo2_none.json 2> gpurun_out/gloo2_none.err && cat gpurun_out/gloo2_none.json &&
NDP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 3 --reducer dense --graph-mode none > gpurun_out/gloo2_dense.json 2> gpurun_out/gloo2_dense.err && cat gpurun_out/gloo2_dense.json
