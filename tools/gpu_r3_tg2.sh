# tgemm k-contiguous LDS + pinned loads, wide P pass: tests, tg A/B (depth), benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tg2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tgconv_gpu.py tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -10
[ $rc -eq 0 ] || exit $rc
for D in 2 3; do
  NDP_TG_DEPTH=$D NDP_TG_SMALL=1 timeout -k 10 240 python tools/tg_bench.py --iters 30 --batches 64 512 \
    --shapes r18.l3.conv r18.l4.conv r50.l1.pw_in r50.l3.pw_in r50.l3.pw_out > $O/tg_d$D.jsonl 2> $O/tg_d$D.err || { echo "tg depth $D failed"; tail -5 $O/tg_d$D.err; exit 1; }
  echo "depth $D"; cat $O/tg_d$D.jsonl
done
for spec in "b512||" "b64||--global-batch=64" "r152d2|NDP_TG_DEPTH=2|--model=resnet152" "r152d3|NDP_TG_DEPTH=3|--model=resnet152" "r50d2|NDP_TG_DEPTH=2|--model=resnet50,--reducer=dense" "r50d3|NDP_TG_DEPTH=3|--model=resnet50,--reducer=dense"; do
  label=$(echo "$spec" | cut -d'|' -f1)
  envs=$(echo "$spec" | cut -d'|' -f2 | tr ',' ' ')
  args=$(echo "$spec" | cut -d'|' -f3 | tr ',' ' ' | sed 's/--\([a-z-]*\)=/--\1 /g')
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > $O/$label.json 2> $O/$label.err || { echo "$label failed"; tail -5 $O/$label.err; exit 1; }
  echo "$label [$envs] [$args] $(python3 tools/jline.py $O/$label.json)"
done
