# PMC passes (see gpu_r2_pmc.sh) — round-3 kernels: ResNet-18 r=4 at batch 512 and 64, ResNet-50 dense, eager so each kernel is one dispatch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3pmc
export TMPDIR=/tmp
P1="FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY"
run() {  # tag, pass-name, counters, bench args
  local tag=$1 pn=$2 ctrs=$3; shift 3
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d gpurun_out/r3pmc/pmc_${tag}_$pn -o run -- python3 bench.py --no-supervise --graph-mode none "$@" > gpurun_out/r3pmc/pmc_${tag}_$pn.out 2>&1 || { echo "FAIL $tag $pn"; tail -5 gpurun_out/r3pmc/pmc_${tag}_$pn.out; return 1; }
  echo "ok $tag $pn"
}
for cfg in "r18b512:" "r18b64:--global-batch 64" "r50b512:--model resnet50 --reducer dense"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  run $tag p1 "$P1" --steps 3 --warmup 1 $args && run $tag p2 "$P2" --steps 3 --warmup 1 $args || exit 1
  c=$(find gpurun_out/r3pmc/pmc_${tag}_p1 gpurun_out/r3pmc/pmc_${tag}_p2 -name '*counter_collection.csv' | tr '\n' ' ')
  t=$(find gpurun_out/r3pmc/pmc_${tag}_p1 -name '*kernel_trace.csv' | tr '\n' ' ')
  python3 tools/pmc_summary.py --counters $c --trace $t > gpurun_out/r3pmc/pmc_$tag.md && head -12 gpurun_out/r3pmc/pmc_$tag.md
  rm -rf gpurun_out/r3pmc/pmc_${tag}_p1 gpurun_out/r3pmc/pmc_${tag}_p2
done
