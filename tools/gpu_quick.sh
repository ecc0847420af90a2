# quick GPU check: selected tests ($TESTS), headline bench, kernel-trace summary
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 30 --warmup 10 ${BENCH_ARGS} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err && cat gpurun_out/bench_quick.json || exit 1
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_q -o run -- python3 bench.py --steps 25 --warmup 5 ${BENCH_ARGS} > gpurun_out/prof_q.out 2>&1 &&
  f=$(find gpurun_out/prof_q -name '*kernel_trace.csv' | head -n 1) && python3 tools/prof_summary.py "$f" --steps 20 --top 80 > gpurun_out/prof_q.md && head -30 gpurun_out/prof_q.md
  rm -rf gpurun_out/prof_q
fi
