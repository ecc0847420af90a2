# PMC passes of single tgemm directions (tools/tg_micro.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tgpmc
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA FETCH_SIZE"
for spec in ${SPECS:-"r50.l1.pw_in:512:fwd"}; do
  IFS=: read shape b d <<< "$spec"
  for pn in p1 p2; do
    [ $pn = p1 ] && ctr="$P1" || ctr="$P2"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $O/${shape}_${b}_${d}_$pn -o run -- python3 tools/tg_micro.py --shape $shape --batch $b --dir $d --iters 10 > $O/${shape}_${b}_${d}_$pn.out 2>&1 || { echo "FAIL $spec $pn"; tail -5 $O/${shape}_${b}_${d}_$pn.out; exit 1; }
  done
  c=$(find $O/${shape}_${b}_${d}_p1 $O/${shape}_${b}_${d}_p2 -name '*counter_collection.csv' | tr '\n' ' ')
  t=$(find $O/${shape}_${b}_${d}_p1 -name '*kernel_trace.csv' | tr '\n' ' ')
  echo "=== $spec"
  python3 tools/pmc_dump.py --counters $c --trace $t --match tgemm
  rm -rf $O/${shape}_${b}_${d}_p1 $O/${shape}_${b}_${d}_p2
done
