# Extend the GEMM solution table (ops/gemm_tuning.py) to every bench shape: TunableOp tuning
# runs append to one file seeded with the shipped table; then A/B the table on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp network_distributed_pytorch_amd/tuning/gemm_gfx950.csv gpurun_out/tune_all0.csv
t() {  # name, bench args...
  local name=$1; shift
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_all.csv \
    timeout -k 10 400 python bench.py --steps 4 --warmup 2 "$@" > gpurun_out/tt_$name.json 2> gpurun_out/tt_$name.err || { tail -5 gpurun_out/tt_$name.err; return 1; }
  echo "tuned $name: $(grep -vc Validator gpurun_out/tune_all0.csv) entries"
}
t r18_256 --global-batch 256 && t r18_128 --global-batch 128 &&
t r50_512 --model resnet50 && t r50_64 --model resnet50 --global-batch 64 &&
t r152_512 --model resnet152 && t r152_64 --model resnet152 --global-batch 64 &&
t bert8 --model distilbert --rank 8 || exit 1
cp gpurun_out/tune_all0.csv network_distributed_pytorch_amd/tuning/gemm_gfx950.csv
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for cfg in "r18_512:--steps 60" "r18_256:--global-batch 256 --steps 60" "r18_128:--global-batch 128 --steps 60" "r18_64:--global-batch 64 --steps 60" \
           "r50_512:--model resnet50 --steps 20 --warmup 5" "r152_512:--model resnet152 --steps 20 --warmup 5" "bert8:--model distilbert --rank 8 --steps 20 --warmup 5"; do
  n=${cfg%%:*}; a=${cfg#*:}
  b ${n}_tuned $a && NDP_TUNED_GEMMS=0 b ${n}_default $a || exit 1
done
