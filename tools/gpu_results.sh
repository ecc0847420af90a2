# results refresh: full GPU test tier, headline + comparison arms, DistilBERT, kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_full.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/res_$name.json 2> gpurun_out/res_$name.err || { tail -5 gpurun_out/res_$name.err; return 1; }
  echo "$name $(python3 -c "import json;d=json.load(open('gpurun_out/res_$name.json'));print(d['value'], d['ms_per_step'], d['config']['hip_graph'])")"
}
b headline --steps 50 --warmup 10 &&
b ref --reducer powersgd-ref --steps 10 --warmup 3 &&
b dense --reducer dense --steps 50 --warmup 10 &&
b bert_r8 --model distilbert --rank 8 --steps 10 --warmup 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r18 -o run -- python3 bench.py --steps 25 --warmup 5 > gpurun_out/prof_r18.out 2>&1 &&
f=$(find gpurun_out/prof_r18 -name '*kernel_trace.csv' | head -n 1) && python3 tools/prof_summary.py "$f" --steps 20 --top 80 > gpurun_out/prof_r18.md && head -12 gpurun_out/prof_r18.md
rc=$?; rm -rf gpurun_out/prof_r18; exit $rc
