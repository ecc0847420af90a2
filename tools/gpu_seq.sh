# kernel sequence of one headline step (launch order) + summary
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_seq -o run -- python3 bench.py --steps 25 --warmup 5 > gpurun_out/prof_seq.out 2>&1 &&
f=$(find gpurun_out/prof_seq -name '*kernel_trace.csv' | head -n 1) && python3 tools/prof_summary.py "$f" --steps 20 --top 80 --sequence gpurun_out/seq.txt > gpurun_out/prof_seq.md && head -5 gpurun_out/prof_seq.md
rc=$?; rm -rf gpurun_out/prof_seq; exit $rc
