# tgemm variants A/B: per-shape conv timings + ResNet-50 dense / ResNet-152 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tgab
mkdir -p $O
export TMPDIR=/tmp
CFGS=${CFGS:-base: bk64:NDP_TG_BK=64 vec:NDP_TG_VEC=1 bk64vec:NDP_TG_BK=64,NDP_TG_VEC=1}
for cfg in $CFGS; do
  tag=${cfg%%:*}; envs=$(echo ${cfg#*:} | tr ',' ' ')
  env $envs timeout -k 10 200 python tools/tg_bench.py --iters 30 --shapes r50.l1.pw_in r50.l1.pw_out r50.l2.pw_in r50.l3.pw_out r50.l4.pw_out > $O/tg_$tag.jsonl 2> $O/tg_$tag.err || { tail -5 $O/tg_$tag.err; exit 1; }
  python3 -c "
import json
rows=[json.loads(l) for l in open('$O/tg_$tag.jsonl')]
print('$tag', ' '.join(f\"{r['shape'][4:]}/{r['batch']}:{r['tgemm_us']}\" for r in rows))"
done
for cfg in $CFGS; do
  tag=${cfg%%:*}; envs=$(echo ${cfg#*:} | tr ',' ' ')
  for m in "r152:--model resnet152" "r50d:--model resnet50 --reducer dense"; do
    mt=${m%%:*}; args=${m#*:}
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 $args > $O/${mt}_$tag.json 2> $O/${mt}_$tag.err || { echo "bench $mt $tag failed"; tail -5 $O/${mt}_$tag.err; exit 1; }
    echo "$mt $tag $(python3 tools/jline.py $O/${mt}_$tag.json)"
  done
done
