# why are the 64x128 / 128x64 tgemm tiles slow: kernel trace (grid, LDS, VGPR, time) per direction and tile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/wide
mkdir -p $O
export TMPDIR=/tmp
for T in 0 1; do
  for D in fwd dgrad wgrad; do
    NDP_TG_TILE=$T timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/t${T}_$D -o run -- python3 tools/tg_micro.py --shape r50.l1.pw_in --batch 512 --dir $D --iters 5 > $O/t${T}_$D.out 2>&1 || { echo "FAIL $T $D"; tail -5 $O/t${T}_$D.out; exit 1; }
    f=$(find $O/t${T}_$D -name '*kernel_trace.csv' | head -n 1)
    python3 tools/trace_attrs.py "$f" "tile=$T dir=$D"
    rm -rf $O/t${T}_$D
  done
done
