set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
pr() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ps_$name -o run -- python3 bench.py --global-batch 64 --steps 12 --warmup 3 > gpurun_out/ps_$name.out 2>&1 || return 1
  f=$(find gpurun_out/ps_$name -name '*kernel_trace.csv' | head -n 1)
  echo "== $name $(python3 tools/jline.py gpurun_out/ps_$name.out)"
  python3 tools/prof_timeline.py "$f" --steps 8 --dump gpurun_out/ps_$name.last.txt | sed -n 5,9p
  grep -n "psgd_p_kernel" gpurun_out/ps_$name.last.txt | head -4
  rm -rf gpurun_out/ps_$name
}
pr normalprio NDP_SIDE_PRIORITY=normal &&
pr highprio NDP_SIDE_PRIORITY=high &&
pr graphq4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 &&
pr hwq8 GPU_MAX_HW_QUEUES=8
