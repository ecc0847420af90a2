#!/bin/bash
# Link-throttled curves (BASELINE config 5) at HEAD, emulated on one GPU (tools/bandwidth_sweep.py):
# DistilBERT r=4 at N=8 and ResNet-18 r=4 at N=2/4/8, PowerSGD vs dense, links none/100g/10g/1g.
#   tools/gpu/links.sh OUT    -> OUT/link_curves.jsonl + OUT/lc_*.md (tables: tools/link_curves_md.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=$1
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
