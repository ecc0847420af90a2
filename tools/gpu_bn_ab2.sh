# single-launch BN for HW 8/16 (NDP_BN_SINGLE_MAX): tests with the path on, then bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_graph_gpu.py::test_resnet18_graph_matches_eager"
timeout -k 10 200 python -u -m pytest $T -q -s --timeout 120 --timeout-method thread 2>&1 | grep -e "eager-vs" -e passed -e failed
NDP_BN_SINGLE_MAX=16 timeout -k 10 300 python -u -m pytest tests/test_batchnorm_gpu.py $T -m gpu -q -s --timeout 120 --timeout-method thread > gpurun_out/pytest_bn2.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep eager-vs gpurun_out/pytest_bn2.log; tail -3 gpurun_out/pytest_bn2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 4 16 4 16; do
  NDP_BN_SINGLE_MAX=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/ab_smax$v.json 2> gpurun_out/ab_smax$v.err || exit 1
  echo "SINGLE_MAX=$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_smax$v.json'));print(d['value'], d['ms_per_step'])")"
done
