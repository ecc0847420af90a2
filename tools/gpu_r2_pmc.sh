# rocprofv3 PMC passes (one counter group per run, --kernel-trace alongside) over the reducer,
# conv and BN kernels: ResNet-18 r=4 b512 and DistilBERT r=8 (eager: one dispatch per kernel call)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY"
run() {  # tag, pass-name, counters, bench args
  local tag=$1 pn=$2 ctrs=$3; shift 3
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d gpurun_out/pmc_${tag}_$pn -o run -- python3 bench.py --graph-mode none "$@" > gpurun_out/pmc_${tag}_$pn.out 2>&1 || { echo "FAIL $tag $pn"; tail -5 gpurun_out/pmc_${tag}_$pn.out; return 1; }
  echo "ok $tag $pn"
}
run r18 p1 "$P1" --steps 3 --warmup 1 &&
run r18 p2 "$P2" --steps 3 --warmup 1 &&
run bert8 p1 "$P1" --model distilbert --rank 8 --steps 2 --warmup 1 &&
run bert8 p2 "$P2" --model distilbert --rank 8 --steps 2 --warmup 1 || exit 1
for tag in r18 bert8; do
  c=$(find gpurun_out/pmc_${tag}_p1 gpurun_out/pmc_${tag}_p2 -name '*counter_collection.csv' | tr '\n' ' ')
  t=$(find gpurun_out/pmc_${tag}_p1 -name '*kernel_trace.csv' | tr '\n' ' ')
  python3 tools/pmc_summary.py --counters $c --trace $t > gpurun_out/pmc_$tag.md && head -40 gpurun_out/pmc_$tag.md
done
rm -rf gpurun_out/pmc_*_p1 gpurun_out/pmc_*_p2
