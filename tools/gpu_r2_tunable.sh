# hipBLASLt solution tuning (PyTorch TunableOp) for the Toeplitz GEMMs: tune once, then
# time with the tuned table read back (tuning off).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in ${BATCHES:-512 64}; do
  timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > gpurun_out/tu_base_$b.json 2> gpurun_out/tu_base_$b.err || { tail -3 gpurun_out/tu_base_$b.err; exit 1; }
  echo "base b$b $(python3 tools/jline.py gpurun_out/tu_base_$b.json)"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable_b$b.csv \
    timeout -k 10 400 python bench.py --global-batch $b --steps 20 --warmup 5 > gpurun_out/tu_tune_$b.json 2> gpurun_out/tu_tune_$b.err || { tail -5 gpurun_out/tu_tune_$b.err; exit 1; }
  echo "tune-run b$b $(python3 tools/jline.py gpurun_out/tu_tune_$b.json)"
  ls gpurun_out/ | grep tunable || true
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable_b$b.csv \
    timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > gpurun_out/tu_use_$b.json 2> gpurun_out/tu_use_$b.err || { tail -3 gpurun_out/tu_use_$b.err; exit 1; }
  echo "tuned b$b $(python3 tools/jline.py gpurun_out/tu_use_$b.json)"
done
