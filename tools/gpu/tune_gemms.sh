#!/bin/bash
# Re-measure the TunableOp GEMM table for the ResNet-18 bench shapes (per-GPU batch 512/256/128/64):
# every rocBLAS / hipBLASLt solution of every library GEMM the step runs is timed in the eager
# warm-up steps, one fresh results file per batch size.  Merge into the shipped table with
# tools/merge_gemm_tables.py.
#   tools/gpu/tune_gemms.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=$1; mkdir -p $O
export TMPDIR=/tmp
for b in 512 256 128 64; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tune_b$b.csv \
    timeout -k 10 600 python bench.py --no-supervise --steps 3 --warmup 3 --global-batch $b > $O/tune_b$b.out 2>&1 \
    || { echo "tune b$b failed"; tail -5 $O/tune_b$b.out; exit 1; }
  ls $O/tune_b$b* >/dev/null 2>&1 && echo "b$b: $(cat $O/tune_b$b*.csv | grep -vc Validator) shapes"
done
