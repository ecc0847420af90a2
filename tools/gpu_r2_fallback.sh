# bench.py fallback agreement: 2 gloo ranks sharing the GPU, attempt 0 fails on every rank ->
# both ranks must move to attempt 1 together and report it; plus the plain 2-rank run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NDP_BACKEND=gloo NDP_BENCH_FAIL=0:* timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/fb_inject.json 2> gpurun_out/fb_inject.err || { tail -20 gpurun_out/fb_inject.err; exit 1; }
grep "^{" gpurun_out/fb_inject.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('inject:', d['value'], d['ms_per_step'], d['config']['hip_graph'], d.get('fallback'))"
NDP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/fb_plain.json 2> gpurun_out/fb_plain.err || { tail -20 gpurun_out/fb_plain.err; exit 1; }
grep "^{" gpurun_out/fb_plain.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('plain:', d['value'], d['ms_per_step'], d['config']['hip_graph'], d.get('fallback'), d['config']['global_batch'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/fb_n1.json 2> gpurun_out/fb_n1.err || { tail -10 gpurun_out/fb_n1.err; exit 1; }
python3 tools/jline.py gpurun_out/fb_n1.json
