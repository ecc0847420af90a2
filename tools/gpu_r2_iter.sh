# one iteration: GPU tests (TESTS, default all), benches b512/b64, kernel profile b64 (+ extra)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for b in 512 64; do
  timeout -k 10 200 python bench.py --global-batch $b --steps 50 --warmup 10 > gpurun_out/it_b$b.json 2> gpurun_out/it_b$b.err || { tail -5 gpurun_out/it_b$b.err; exit 1; }
  echo "b$b $(python3 tools/jline.py gpurun_out/it_b$b.json)"
done
[ "${SKIP_PROF:-0}" = "1" ] || bash tools/gpu_r2_prof.sh b64 "--global-batch 64" ${PROF_EXTRA:-}
