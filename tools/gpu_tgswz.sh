cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tgswz; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tgconv_gpu.py -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "tg pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for z in 0 1; do
  NDP_TG_SWZ=$z timeout -k 10 300 python tools/tg_bench.py --iters 30 --shapes r50.l1.pw_in r50.l1.pw_out r50.l2.pw_in r50.l3.pw_out r50.l4.pw_out > $O/tg_$z.jsonl 2> $O/tg_$z.err || { echo "tg_bench failed"; tail -3 $O/tg_$z.err; exit 1; }
  echo "== NDP_TG_SWZ=$z"; cat $O/tg_$z.jsonl
  NDP_TG_SWZ=$z timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model resnet50 --reducer dense > $O/r50_$z.json 2> $O/r50_$z.err && python -c "import json; r=json.loads(open('$O/r50_$z.json').read().strip().splitlines()[-1]); print('r50 dense', r['ms_per_step'])" || exit 1
  NDP_TG_SWZ=$z timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model resnet152 > $O/r152_$z.json 2> $O/r152_$z.err && python -c "import json; r=json.loads(open('$O/r152_$z.json').read().strip().splitlines()[-1]); print('r152', r['ms_per_step'])" || exit 1
done
