# round 3: tgemm conv family + supervisor checks, then benches (b512, b64, R50 dense, R152 r4)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_tgconv_gpu.py tests/test_bench_gpu.py tests/test_ipc_gpu.py tests/test_gradarena_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" $O/pytest.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "--global-batch 512" "--global-batch 64" "--model resnet50 --reducer dense" "--model resnet152"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $cfg > $O/b_$tag.json 2> $O/b_$tag.err || { echo "bench $cfg failed rc=$?"; tail -5 $O/b_$tag.err; exit 1; }
  python -c "import json,sys; r=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); print('$cfg', r['ms_per_step'], r['value'], r.get('fallback'), r['supervisor']['failed'][:1])"
done
timeout -k 10 300 python tools/tg_bench.py --iters 30 > $O/tg_bench.jsonl 2> $O/tg_bench.err || { echo "tg_bench failed"; tail -5 $O/tg_bench.err; exit 1; }
cat $O/tg_bench.jsonl
