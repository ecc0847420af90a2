# Slab hand-off + single-launch 8x8 BN: GPU tests, then A/B at the strong-scaling shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_slablink_gpu.py tests/test_loss_gpu.py tests/test_batchnorm_gpu.py tests/test_conv_direct.py tests/test_graph_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/slab_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/slab_tests.log | head -20; }
tail -2 gpurun_out/slab_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 64 128 256 512; do
  b slab_$gb NDP_SLAB_LINKS=1 python bench.py --global-batch $gb --steps 60 &&
  b noslab_$gb NDP_SLAB_LINKS=0 python bench.py --global-batch $gb --steps 60 &&
  b old_$gb NDP_SLAB_LINKS=0 NDP_BN_SINGLE64=0 python bench.py --global-batch $gb --steps 60 || exit 1
done
