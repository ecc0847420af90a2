# Extend the GEMM solution table with this round's new shapes (packed QKV projection, in-place
# addmm_ GradLink GEMMs): TunableOp tuning runs append to a copy of the shipped table.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp network_distributed_pytorch_amd/tuning/gemm_gfx950.csv gpurun_out/tune_all.csv
t() {  # name, bench args...
  local name=$1; shift
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_all.csv \
    timeout -k 10 500 python bench.py --steps 4 --warmup 2 "$@" > gpurun_out/tt_$name.json 2> gpurun_out/tt_$name.err || { tail -5 gpurun_out/tt_$name.err; return 1; }
  echo "tuned $name: $(grep -vc Validator gpurun_out/tune_all.csv) entries"
}
t bert8 --model distilbert --rank 8 && t r18_512 && t r18_64 --global-batch 64 || exit 1
cp gpurun_out/tune_all.csv network_distributed_pytorch_amd/tuning/gemm_gfx950.csv
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
b bert8_t3 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 &&
b r18_512_t3 python bench.py --steps 60 && b r18_64_t3 python bench.py --global-batch 64 --steps 60
