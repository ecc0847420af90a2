# device-flag ordered compute/comm graphs: tests + timelines + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_overlap_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_flags.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_flags.log
[ $rc -eq 0 ] || exit $rc
p() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$name -o run -- python3 bench.py --steps 25 --warmup 5 "$@" > gpurun_out/tl_$name.out 2>&1 || { tail -5 gpurun_out/tl_$name.out; return 1; }
  f=$(find gpurun_out/tl_$name -name '*kernel_trace.csv' | head -n 1)
  python3 tools/prof_timeline.py "$f" --steps 20 --dump gpurun_out/tl_$name.last.txt > gpurun_out/tl_$name.md &&
  python3 tools/prof_summary.py "$f" --steps 20 --marker "conv_fwd_kernel<7, 7" --top 70 > gpurun_out/tl_$name.kern.md &&
  echo "== $name $(python3 tools/jline.py gpurun_out/tl_$name.out)" && sed -n 5,10p gpurun_out/tl_$name.md && grep -n "psgd_p_kernel" gpurun_out/tl_$name.last.txt | head -4
  rm -rf gpurun_out/tl_$name
}
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/fl_$name.json 2> gpurun_out/fl_$name.err || { tail -5 gpurun_out/fl_$name.err; return 1; }
  python3 tools/jline.py gpurun_out/fl_$name.json
}
p b64_ov --global-batch 64 &&
b b64_ov --global-batch 64 --steps 50 --warmup 10 &&
b b64_serial --global-batch 64 --steps 50 --warmup 10 --no-overlap &&
b b512_ov --steps 50 --warmup 10 &&
b b512_serial --steps 50 --warmup 10 --no-overlap &&
p b512_ov
