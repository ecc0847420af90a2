# tgemm PMC on the micro benchmark (eager, one direction per run): where do the cycles go
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tgpmc
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU"
for sh in r50.l1.pw_in r50.l3.pw_in; do
  for d in fwd dgrad wgrad; do
    for pn in 1 2; do
      [ $pn = 1 ] && C="$P1" || C="$P2"
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/p_${sh}_${d}_$pn -o run -- python3 tools/tg_micro.py --shape $sh --batch 512 --dir $d --iters 10 > $O/p_${sh}_${d}_$pn.out 2>&1 || { echo "FAIL $sh $d $pn"; tail -5 $O/p_${sh}_${d}_$pn.out; exit 1; }
    done
    c=$(find $O/p_${sh}_${d}_1 $O/p_${sh}_${d}_2 -name '*counter_collection.csv' | tr '\n' ' ')
    t=$(find $O/p_${sh}_${d}_1 -name '*kernel_trace.csv' | tr '\n' ' ')
    echo "### $sh $d"; python3 tools/pmc_dump.py --counters $c --trace $t --match tgemm
    rm -rf $O/p_${sh}_${d}_1 $O/p_${sh}_${d}_2
  done
done
