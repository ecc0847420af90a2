# Deferred conv slabs summed inside the two-kernel BN statistics passes (layer1 8x8 maps).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NDP_BN_STATS_SLABS=1 timeout -k 10 600 python -u -m pytest tests/test_slablink_gpu.py tests/test_batchnorm_gpu.py tests/test_graph_gpu.py tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bnslab_tests.log 2>&1 || { tail -30 gpurun_out/bnslab_tests.log; exit 1; }
tail -1 gpurun_out/bnslab_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 64 128; do
  b on_$gb NDP_BN_STATS_SLABS=1 python bench.py --global-batch $gb --steps 60 &&
  b off_$gb python bench.py --global-batch $gb --steps 60 &&
  b on2_$gb NDP_BN_STATS_SLABS=1 python bench.py --global-batch $gb --steps 60 &&
  b off2_$gb python bench.py --global-batch $gb --steps 60 || exit 1
done
b on_512 NDP_BN_STATS_SLABS=1 python bench.py --steps 60
