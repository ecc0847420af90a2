# Slab links (two-kernel 8x8 BN), colsum pass 2, fused add+LayerNorm: tests + A/B; then
# 1-rank RCCL rehearsal traces (overlap on) for the profiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_layernorm_gpu.py tests/test_slablink_gpu.py tests/test_linear_gpu.py tests/test_batchnorm_gpu.py tests/test_loss_gpu.py tests/test_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ln_tests.log 2>&1 || { tail -30 gpurun_out/ln_tests.log; exit 1; }
tail -2 gpurun_out/ln_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
b bert8 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bert8_noln NDP_FUSED_LN=0 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 || exit 1
for gb in 64 128 256 512; do
  b slab_$gb python bench.py --global-batch $gb --steps 60 &&
  b noslab_$gb NDP_SLAB_LINKS=0 python bench.py --global-batch $gb --steps 60 || exit 1
done
bash tools/gpu_r2_prof.sh rh_b64 "--global-batch 64 --overlap on" rh_b512 "--overlap on" &&
MARKER=emb_rank_kernel PSTEPS=10 bash tools/gpu_r2_prof.sh bert8 "--model distilbert --rank 8"
