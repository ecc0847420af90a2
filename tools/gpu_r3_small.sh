# tgemm small-map family (ResNet-18 layer3/4) vs hipBLASLt Toeplitz: split-K cap A/B, micro + steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/small
mkdir -p $O
export TMPDIR=/tmp
for cap in 4 16 64; do
  NDP_TG_SMALL=1 NDP_TG_MAXSPLIT=$cap timeout -k 10 240 python tools/tg_bench.py --iters 30 --batches 64 128 512 \
    --shapes r18.l3.conv r18.l3.entry r18.l3.ds r18.l4.conv r18.l4.entry > $O/tg_c$cap.jsonl 2> $O/tg_c$cap.err || { echo "tg $cap failed"; tail -5 $O/tg_c$cap.err; exit 1; }
  echo "== cap $cap"; python3 -c "
import json
for l in open('$O/tg_c$cap.jsonl'):
    r=json.loads(l); print(r['shape'], r['batch'], r['tgemm_us'], r['previous_us'])"
done
for arm in "base|NDP_TG_SMALL=0" "s16|NDP_TG_SMALL=1,NDP_TG_MAXSPLIT=16" "s64|NDP_TG_SMALL=1,NDP_TG_MAXSPLIT=64"; do
  for cfg in "b64|--global-batch 64" "b128|--global-batch 128"; do
    label=${arm%%|*}; envs=$(echo ${arm#*|} | tr ',' ' '); tag=${cfg%%|*}; args=${cfg#*|}
    env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 10 $args > $O/${tag}_$label.json 2> $O/${tag}_$label.err || { echo "$label $tag failed"; tail -5 $O/${tag}_$label.err; exit 1; }
    echo "${tag}_$label $(python3 tools/jline.py $O/${tag}_$label.json)"
  done
done
