# conv LDS-layout change: conv numerics, headline benches, PMC passes for ResNet-18 b512
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3lds; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_slablink_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
for b in 512 64; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 10 --global-batch $b > $O/b$b.json 2> $O/b$b.err || { tail -5 $O/b$b.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/b$b.json').read().strip().splitlines()[-1]); print('b$b', r['ms_per_step'], r['value'])"
done
P1="FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY"
for pn in p1 p2; do
  [ $pn = p1 ] && C="$P1" || C="$P2"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/pmc_$pn -o run -- python3 bench.py --no-supervise --graph-mode none --steps 3 --warmup 1 > $O/pmc_$pn.out 2>&1 || { echo "FAIL $pn"; tail -5 $O/pmc_$pn.out; exit 1; }
done
c=$(find $O/pmc_p1 $O/pmc_p2 -name '*counter_collection.csv' | tr '\n' ' ')
t=$(find $O/pmc_p1 -name '*kernel_trace.csv' | tr '\n' ' ')
python3 tools/pmc_summary.py --counters $c --trace $t > $O/pmc_r18b512.md && head -24 $O/pmc_r18b512.md | cut -c1-200
rm -rf $O/pmc_p1 $O/pmc_p2
