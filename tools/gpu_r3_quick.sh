# quick loop: graph-branch probe, reducer/kernel GPU tests, headline + b64 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3quick
mkdir -p $O
bash tools/gpu_r3_probe_graph.sh || exit 1
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_overlap_gpu.py} -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for gb in 512 64; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --global-batch $gb > $O/b$gb.json 2> $O/b$gb.err || { echo "bench $gb failed"; tail -5 $O/b$gb.err; exit 1; }
  python -c "import json; r=json.loads(open('$O/b$gb.json').read().strip().splitlines()[-1]); print($gb, r['ms_per_step'], r['value'], r.get('fallback'))"
done
