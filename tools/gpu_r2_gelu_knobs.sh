# Fused GELU-backward + bias sum (DistilBERT FFN): tests + A/B; conv batching knobs A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NDP_FUSED_GELU=1 timeout -k 10 400 python -u -m pytest tests/test_linear_gpu.py tests/test_distilbert_fusions_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gelu_tests.log 2>&1 || { tail -30 gpurun_out/gelu_tests.log; exit 1; }
tail -1 gpurun_out/gelu_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
b bg NDP_FUSED_GELU=1 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bg_off python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bg2 NDP_FUSED_GELU=1 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 || exit 1
bash tools/gpu_r2_knobs.sh
