# link-throttled curves at the round-3 defaults (4 PowerSGD groups, overlap on every arm incl. "none")
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3links
mkdir -p $O
export TMPDIR=/tmp
J=$O/link_curves.jsonl
rm -f $J
timeout -k 10 900 python tools/bandwidth_sweep.py --mode emulate --gpus 8 --model distilbert --rank 4 --steps 6 --warmup 3 --jsonl $J > $O/lc_bert8.md 2> $O/lc_bert8.err || { tail -5 $O/lc_bert8.err; exit 1; }
cat $O/lc_bert8.md
for n in 2 4 8; do
  timeout -k 10 600 python tools/bandwidth_sweep.py --mode emulate --gpus $n --model resnet18 --rank 4 --steps 15 --warmup 5 --jsonl $J > $O/lc_r18_$n.md 2> $O/lc_r18_$n.err || { tail -5 $O/lc_r18_$n.err; exit 1; }
  cat $O/lc_r18_$n.md
done
