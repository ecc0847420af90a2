# full GPU suite + the headline / reference-config benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3full
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -3; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in ${BENCHES:-"--global-batch=512" "--global-batch=64" "--model=resnet50,--reducer=dense" "--model=resnet152"}; do
  args=$(echo $cfg | tr ',' ' ' | tr '=' ' ')
  tag=$(echo $cfg | tr -d ' -=,')
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > $O/b_$tag.json 2> $O/b_$tag.err || { echo "bench $cfg failed rc=$?"; tail -5 $O/b_$tag.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); print('$cfg', r['ms_per_step'], r['value'], r.get('fallback'), r['supervisor']['failed'][:1])"
done
