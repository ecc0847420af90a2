#!/bin/bash
# Two PMC passes (each its own rocprofv3 run, within the per-block counter limits) over an
# eager bench run, merged per kernel by tools/pmc_summary.py: OUT/pmc_TAG.md
#   tools/gpu/pmc.sh OUT TAG [bench args...]
# e.g. tools/gpu/pmc.sh gpurun_out/pmc r18b512
# PROG=tools/sm_bench.py tools/gpu/pmc.sh OUT sm --iters 5   (another python program and its args)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1; TAG=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY"
for pn in p1 p2; do
  if [ $pn = p1 ]; then C=$P1; else C=$P2; fi
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/pmc_${TAG}_$pn" -o run -- \
    python3 ${PROG:-bench.py --no-supervise --graph-mode none --steps 3 --warmup 1} "$@" > "$OUT/pmc_${TAG}_$pn.out" 2>&1 \
    || { echo "PMC $TAG $pn failed"; tail -5 "$OUT/pmc_${TAG}_$pn.out"; exit 1; }
done
c=$(find "$OUT/pmc_${TAG}_p1" "$OUT/pmc_${TAG}_p2" -name '*counter_collection.csv' | tr '\n' ' ')
t=$(find "$OUT/pmc_${TAG}_p1" -name '*kernel_trace.csv' | tr '\n' ' ')
{
  echo "<!-- regenerate: ${PROG:+PROG=$PROG }tools/gpu/pmc.sh OUT $TAG $* -->"
  python3 tools/pmc_summary.py --counters $c --trace $t
} > "$OUT/pmc_$TAG.md"
head -12 "$OUT/pmc_$TAG.md"
rm -rf "$OUT/pmc_${TAG}_p1" "$OUT/pmc_${TAG}_p2"
