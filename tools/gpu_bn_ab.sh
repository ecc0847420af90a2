# BN single-launch path: tests, then A/B of column width and of the 3-kernel path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_batchnorm_gpu.py tests/test_pool.py tests/test_models.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_bn.log
[ $rc -eq 0 ] || exit $rc
for v in 4 8 16; do
  NDP_BN_COLW=$v timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/ab_colw$v.json 2> gpurun_out/ab_colw$v.err || exit 1
  echo "COLW=$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_colw$v.json'));print(d['value'], d['ms_per_step'])")"
done
NDP_BN_SINGLE=0 timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/ab_single0.json 2> gpurun_out/ab_single0.err || exit 1
echo "SINGLE=0 $(python3 -c "import json;d=json.load(open('gpurun_out/ab_single0.json'));print(d['value'], d['ms_per_step'])")"
