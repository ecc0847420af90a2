# Native 3x3 stride-2 grad-x (zero-insert staging): numerics, model tests, A/B vs MIOpen.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_direct.py tests/test_slablink_gpu.py tests/test_graph_gpu.py tests/test_batchnorm_gpu.py tests/test_loss_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dg2_tests.log 2>&1 || { tail -30 gpurun_out/dg2_tests.log; exit 1; }
tail -1 gpurun_out/dg2_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 512 64 256; do
  b dg2_$gb python bench.py --global-batch $gb --steps 60 &&
  b miopen_$gb NDP_CONV_DGRAD2=0 python bench.py --global-batch $gb --steps 60 &&
  b dg2b_$gb python bench.py --global-batch $gb --steps 60 || exit 1
done
