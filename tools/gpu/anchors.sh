#!/bin/bash
# Same-box comparison anchors: the reference-semantics eager arm (stock MIOpen /
# ATen model ops + the eager reference reducer loop), stock model ops + the native reducer,
# and the native step, for ResNet-18 r=4 at batch 512 / 64 and DistilBERT r=8; then an
# UNFILTERED DistilBERT r=8 kernel table; then (LINKS=1) the link-throttled curves.
#   tools/gpu/anchors.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-20} WARM=${WARM:-5} tools/gpu/bench.sh "$OUT" \
  "ref512|--stock --reducer powersgd-ref" "stock512|--stock" "native512|" \
  "ref64|--stock --reducer powersgd-ref --global-batch 64" "stock64|--stock --global-batch 64" \
  "native64|--global-batch 64" \
  "bertref|--model distilbert --rank 8 --stock --reducer powersgd-ref" \
  "bertstock|--model distilbert --rank 8 --stock" "bert8|--model distilbert --rank 8" || exit 1
MARKER="psgd_p_wide_kernel" tools/gpu/profile.sh "$OUT" bert8 5 --model distilbert --rank 8 || exit 1
if [ "${LINKS:-0}" = 1 ]; then
  J=$OUT/link_curves.jsonl
  rm -f "$J"
  timeout -k 10 900 python tools/bandwidth_sweep.py --mode emulate --gpus 8 --model distilbert --rank 4 --steps 6 \
    --warmup 3 --jsonl "$J" > "$OUT/lc_bert8.md" 2> "$OUT/lc_bert8.err" || { tail -5 "$OUT/lc_bert8.err"; exit 1; }
  for n in 2 4 8; do
    timeout -k 10 600 python tools/bandwidth_sweep.py --mode emulate --gpus $n --model resnet18 --rank 4 --steps 15 \
      --warmup 5 --jsonl "$J" > "$OUT/lc_r18_$n.md" 2> "$OUT/lc_r18_$n.err" || { tail -5 "$OUT/lc_r18_$n.err"; exit 1; }
  done
  python3 tools/link_curves_md.py "$J" > "$OUT/link_tables.md"
fi
