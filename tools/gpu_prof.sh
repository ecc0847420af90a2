# rocprofv3 kernel trace of the headline bench (and DistilBERT), summarised per step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r18 -o run -- python3 bench.py --steps 25 --warmup 5 > gpurun_out/prof_r18.out 2>&1 &&
f=$(find gpurun_out/prof_r18 -name '*kernel_trace.csv' | head -n 1) && python3 tools/prof_summary.py "$f" --steps 20 > gpurun_out/prof_r18.md && cat gpurun_out/prof_r18.md &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_bert -o run -- python3 bench.py --model distilbert --rank 8 --steps 12 --warmup 3 > gpurun_out/prof_bert.out 2>&1 &&
f=$(find gpurun_out/prof_bert -name '*kernel_trace.csv' | head -n 1) && python3 tools/prof_summary.py "$f" --steps 10 > gpurun_out/prof_bert.md && cat gpurun_out/prof_bert.md
rm -rf gpurun_out/prof_r18 gpurun_out/prof_bert
