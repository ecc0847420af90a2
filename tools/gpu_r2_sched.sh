# Conv MFMA-block scheduling variants (NDP_CONV_VARIANT 5 = iglp_opt(0), 6 = pinned MFMA/LDS
# interleave) for the layer1 / layer2 direct fwd + grad-x kernels: numerics then A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 5 6; do
  NDP_CONV_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_conv_direct.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sched_tests_$v.log 2>&1 || { tail -20 gpurun_out/sched_tests_$v.log; exit 1; }
  tail -1 gpurun_out/sched_tests_$v.log
done
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 512 64; do
  b v0_$gb python bench.py --global-batch $gb --steps 60 &&
  b v5_$gb NDP_CONV_VARIANT=5 python bench.py --global-batch $gb --steps 60 &&
  b v6_$gb NDP_CONV_VARIANT=6 python bench.py --global-batch $gb --steps 60 &&
  b v0b_$gb python bench.py --global-batch $gb --steps 60 &&
  b v6b_$gb NDP_CONV_VARIANT=6 python bench.py --global-batch $gb --steps 60 || exit 1
done
NDP_CONV_VARIANT=6 bash tools/gpu_r2_prof.sh r18_b512_v6 ""
