# full GPU tier with deferred uploads, then A/B NDP_DEFER_UPLOADS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_full.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  NDP_DEFER_UPLOADS=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/ab_defer$v.json 2> gpurun_out/ab_defer$v.err || exit 1
  echo "DEFER=$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_defer$v.json'));print(d['value'], d['ms_per_step'], d['mean_loss'])")"
done
timeout -k 10 200 python bench.py --model distilbert --rank 8 --steps 10 --warmup 5 > gpurun_out/bert.json 2> gpurun_out/bert.err && cat gpurun_out/bert.json
