# tgemm after address hoisting: kernel tests + A/B, then all round-3 GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tg2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tgconv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tg.log 2>&1
rc=$?; echo "tg pytest rc=$rc"; tail -3 $O/pytest_tg.log
timeout -k 10 300 python tools/tg_bench.py --iters 30 > $O/tg_bench.jsonl 2> $O/tg_bench.err || { echo "tg_bench failed"; tail -5 $O/tg_bench.err; exit 1; }
cat $O/tg_bench.jsonl
timeout -k 10 900 python -u -m pytest tests/test_bench_gpu.py tests/test_ipc_gpu.py tests/test_gradarena_gpu.py -v --timeout 600 --timeout-method thread > $O/pytest_rest.log 2>&1
echo "rest pytest rc=$?"; grep -E "PASSED|FAILED|ERROR" $O/pytest_rest.log | tail -12
