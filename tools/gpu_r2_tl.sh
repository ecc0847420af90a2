# timeline profiles: overlap vs serial at per-GPU batch 64 and 512
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
p() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$name -o run -- python3 bench.py --steps 25 --warmup 5 "$@" > gpurun_out/tl_$name.out 2>&1 || { tail -5 gpurun_out/tl_$name.out; return 1; }
  f=$(find gpurun_out/tl_$name -name '*kernel_trace.csv' | head -n 1)
  python3 tools/prof_timeline.py "$f" --steps 20 --dump gpurun_out/tl_$name.last.txt > gpurun_out/tl_$name.md &&
  python3 tools/prof_summary.py "$f" --steps 20 --marker "conv_fwd_kernel<7, 7" --top 60 > gpurun_out/tl_$name.kern.md &&
  echo "== $name" && head -14 gpurun_out/tl_$name.md && rm -rf gpurun_out/tl_$name
}
p b64_ov --global-batch 64 &&
p b64_serial --global-batch 64 --no-overlap &&
p b512_ov &&
p b512_serial --no-overlap
