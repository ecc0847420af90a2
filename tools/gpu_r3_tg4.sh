# tgemm tile A/B (NDP_TG_TILE 0: 64x64, 1: 64x128, 2: 128x64, -1: by shape): tests, micro, R50/R152 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tg4
mkdir -p $O
export TMPDIR=/tmp
for T in 0 1 2; do
  timeout -k 10 300 env NDP_TG_TILE=$T NDP_TG_SMALL=1 python -u -m pytest tests/test_tgconv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_t$T.log 2>&1
  rc=$?; echo "pytest tile $T rc=$rc"; tail -2 $O/pytest_t$T.log; [ $rc -eq 0 ] || exit $rc
done
for T in 0 1 2; do
  env NDP_TG_TILE=$T NDP_TG_SMALL=1 timeout -k 10 240 python tools/tg_bench.py --iters 30 --batches 64 512 \
    --shapes r18.l3.conv r18.l4.conv r50.l1.pw_in r50.l1.pw_out r50.l2.pw_in r50.l3.pw_in r50.l3.pw_out r50.l4.pw_out > $O/tg_t$T.jsonl 2> $O/tg_t$T.err || { echo "tg $T failed"; tail -5 $O/tg_t$T.err; exit 1; }
  echo "== tile $T"; python3 -c "
import json
for l in open('$O/tg_t$T.jsonl'):
    r=json.loads(l); print(r['shape'], r['batch'], r['tgemm_us'], r['previous_us'])"
done
for T in 0 1 2 -1; do
  env NDP_TG_TILE=$T timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model resnet152 > $O/r152_t$T.json 2> $O/r152_t$T.err || { echo "r152 $T failed"; tail -5 $O/r152_t$T.err; exit 1; }
  env NDP_TG_TILE=$T timeout -k 10 300 python bench.py --steps 10 --warmup 3 --model resnet50 --reducer dense > $O/r50_t$T.json 2> $O/r50_t$T.err || { echo "r50 $T failed"; tail -5 $O/r50_t$T.err; exit 1; }
  echo "tile $T r152 $(python3 tools/jline.py $O/r152_t$T.json)"; echo "tile $T r50 $(python3 tools/jline.py $O/r50_t$T.json)"
done
