# grid-barrier BN: numerics, A/B benches (NDP_BN_GRID=0/1), kernel tables
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3bn; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_batchnorm_gpu.py tests/test_slablink_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
for gr in 1 0; do
  for b in 512 64; do
    NDP_BN_GRID=$gr timeout -k 10 200 python bench.py --steps 30 --warmup 10 --global-batch $b > $O/b${b}_$gr.json 2> $O/b${b}_$gr.err || { tail -5 $O/b${b}_$gr.err; exit 1; }
    python -c "import json; r=json.loads(open('$O/b${b}_$gr.json').read().strip().splitlines()[-1]); print('grid=$gr b$b', r['ms_per_step'], r['value'], r['replicas_equal'], r['mean_loss'])"
  done
done
PROFS="b512g:--global-batch=512 b64g:--global-batch=64" bash tools/gpu_r3_prof.sh && cp gpurun_out/r3prof/b512g.md gpurun_out/r3prof/b64g.md $O/
[ -n "$FULL" ] && timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_full.log 2>&1
echo "full pytest rc=$?"; tail -3 $O/pytest_full.log
