set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_r18.json 2> gpurun_out/bench_r18.err && cat gpurun_out/bench_r18.json &&
timeout -k 10 200 python bench.py --model distilbert --rank 8 --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.err && cat gpurun_out/bench_bert.json &&
timeout -k 10 200 python tools/conv_bench.py > gpurun_out/conv_bench.txt 2>&1 && cat gpurun_out/conv_bench.txt
