# round-3 final verification: full GPU suite, smoke, headline + strong-scaling shapes + reference configs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for spec in "b512||" "b256||--global-batch=256" "b128||--global-batch=128" "b64||--global-batch=64" "dense512||--reducer=dense" "r152||--model=resnet152" "r50d||--model=resnet50,--reducer=dense" "r50p||--model=resnet50" "bert8||--model=distilbert,--rank=8"; do
  label=$(echo "$spec" | cut -d'|' -f1)
  args=$(echo "$spec" | cut -d'|' -f3 | tr ',' ' ' | sed 's/--\([a-z-]*\)=/--\1 /g')
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 $args > $O/$label.json 2> $O/$label.err || { echo "$label failed"; tail -5 $O/$label.err; exit 1; }
  echo "$label $(python3 tools/jline.py $O/$label.json)"
done
cat $O/*.json | grep '^{' > $O/bench_final_round3.jsonl
