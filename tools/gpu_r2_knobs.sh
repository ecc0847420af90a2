# Batching knobs A/B: split-K cap (NDP_CONV_MAXKS) and grad-W slice size (NDP_WGRAD_IMGS_MUL).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NDP_CONV_MAXKS=4 NDP_WGRAD_IMGS_MUL=4 timeout -k 10 300 python -u -m pytest tests/test_conv_direct.py tests/test_slablink_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kn_tests.log 2>&1 || { tail -20 gpurun_out/kn_tests.log; exit 1; }
tail -1 gpurun_out/kn_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 64 128; do
  b k0_$gb python bench.py --global-batch $gb --steps 60 &&
  b ks4_$gb NDP_CONV_MAXKS=4 python bench.py --global-batch $gb --steps 60 &&
  b k0b_$gb python bench.py --global-batch $gb --steps 60 &&
  b ks4b_$gb NDP_CONV_MAXKS=4 python bench.py --global-batch $gb --steps 60 || exit 1
done
for gb in 512 256; do
  b w0_$gb python bench.py --global-batch $gb --steps 60 &&
  b w2_$gb NDP_WGRAD_IMGS_MUL=2 python bench.py --global-batch $gb --steps 60 &&
  b w4_$gb NDP_WGRAD_IMGS_MUL=4 python bench.py --global-batch $gb --steps 60 &&
  b w0b_$gb python bench.py --global-batch $gb --steps 60 || exit 1
done
