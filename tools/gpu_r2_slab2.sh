# Slab links with the two-kernel 8x8 BN (single64 off), colsum pass-2 change (DistilBERT).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_slablink_gpu.py tests/test_linear_gpu.py tests/test_batchnorm_gpu.py tests/test_loss_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/slab2_tests.log 2>&1 || { tail -30 gpurun_out/slab2_tests.log; exit 1; }
tail -2 gpurun_out/slab2_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 64 128 256 512; do
  b slab_$gb python bench.py --global-batch $gb --steps 60 &&
  b noslab_$gb NDP_SLAB_LINKS=0 python bench.py --global-batch $gb --steps 60 &&
  b slab2_$gb python bench.py --global-batch $gb --steps 60 || exit 1
done
b bert8 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5
