# tests + benches b512/b64 + LDS-conflict PMC pass (ResNet-18 b512 eager)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_PROF=1 bash tools/gpu_r2_iter.sh || exit 1
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d gpurun_out/pmc_lds -o run -- python3 bench.py --graph-mode none --steps 3 --warmup 1 > gpurun_out/pmc_lds.out 2>&1 || { tail -5 gpurun_out/pmc_lds.out; exit 1; }
python3 tools/pmc_summary.py --counters $(find gpurun_out/pmc_lds -name '*counter_collection.csv') --trace $(find gpurun_out/pmc_lds -name '*kernel_trace.csv') --match conv_ > gpurun_out/pmc_lds.md && cat gpurun_out/pmc_lds.md
rm -rf gpurun_out/pmc_lds
