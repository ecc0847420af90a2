# Fused cross-entropy tests + conv chunk-size variants A/B (b512 / b64).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_loss_gpu.py tests/test_conv_direct.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ce_tests.log 2>&1 || { tail -30 gpurun_out/ce_tests.log; exit 1; }
tail -2 gpurun_out/ce_tests.log
NDP_CONV_VARIANT=2 timeout -k 10 400 python -u -m pytest tests/test_conv_direct.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ce_tests_v2.log 2>&1 || { tail -30 gpurun_out/ce_tests_v2.log; exit 1; }
tail -2 gpurun_out/ce_tests_v2.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 512 64; do
  b ce_$gb python bench.py --global-batch $gb --steps 60 &&
  b noce_$gb NDP_FUSED_CE=0 python bench.py --global-batch $gb --steps 60 &&
  b v2_$gb NDP_CONV_VARIANT=2 python bench.py --global-batch $gb --steps 60 &&
  b v3_$gb NDP_CONV_VARIANT=3 python bench.py --global-batch $gb --steps 60 &&
  b ce2_$gb python bench.py --global-batch $gb --steps 60 || exit 1
done
b bert8 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bert8_noce NDP_FUSED_CE=0 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5
