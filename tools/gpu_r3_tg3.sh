# tgemm A/B: 16-B loads (NDP_TG_VEC) x workgroup fill (NDP_TG_FILL), micro + ResNet-50/152 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tg3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 env NDP_TG_VEC=1 python -u -m pytest tests/test_tgconv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest(vec) rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for arm in "v0f256|NDP_TG_VEC=0" "v1f256|NDP_TG_VEC=1" "v1f512|NDP_TG_VEC=1,NDP_TG_FILL=512" "v0f512|NDP_TG_VEC=0,NDP_TG_FILL=512"; do
  label=${arm%%|*}; envs=$(echo ${arm#*|} | tr ',' ' ')
  env $envs NDP_TG_SMALL=1 timeout -k 10 240 python tools/tg_bench.py --iters 30 --batches 64 512 \
    --shapes r18.l3.conv r50.l1.pw_in r50.l1.pw_out r50.l3.pw_in r50.l3.pw_out > $O/tg_$label.jsonl 2> $O/tg_$label.err || { echo "tg $label failed"; tail -5 $O/tg_$label.err; exit 1; }
  echo "== $label"; python3 -c "
import json,sys
for l in open('$O/tg_$label.jsonl'):
    r=json.loads(l); print(r['shape'], r['batch'], r['tgemm_us'])"
done
for arm in "v0f256|NDP_TG_VEC=0" "v1f256|NDP_TG_VEC=1" "v1f512|NDP_TG_VEC=1,NDP_TG_FILL=512"; do
  label=${arm%%|*}; envs=$(echo ${arm#*|} | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model resnet152 > $O/r152_$label.json 2> $O/r152_$label.err || { echo "r152 $label failed"; tail -5 $O/r152_$label.err; exit 1; }
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model resnet50 --reducer dense > $O/r50_$label.json 2> $O/r50_$label.err || { echo "r50 $label failed"; tail -5 $O/r50_$label.err; exit 1; }
  echo "$label r152 $(python3 tools/jline.py $O/r152_$label.json)"; echo "$label r50 $(python3 tools/jline.py $O/r50_$label.json)"
done
# kernel tables at the shipped defaults (b512, b64)
for cfg in "b512:" "b64:--global-batch 64"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$tag -o run -- python3 bench.py --no-supervise --steps 25 --warmup 5 $args > $O/prof_$tag.out 2>&1 || { echo "prof $tag failed"; tail -5 $O/prof_$tag.out; exit 1; }
  f=$(find $O/prof_$tag -name '*kernel_trace.csv' | head -n 1)
  python3 tools/prof_summary.py "$f" --steps 20 --marker 'conv_fwd_kernel<7, 7' --top 60 > $O/kernels_$tag.md && head -30 $O/kernels_$tag.md
  rm -rf $O/prof_$tag
done
