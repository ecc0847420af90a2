set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pe
export TMPDIR=/tmp
pe() {
  local name=$1; shift
  env timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pe_$name -o run -- python3 tools/probe_events.py "$@" > gpurun_out/pe_$name.out 2>&1 || return 1
  f=$(find gpurun_out/pe_$name -name '*kernel_trace.csv' | head -n 1)
  echo "== $name $(grep ms/step gpurun_out/pe_$name.out)"
  cut -d, -f1-40 "$f" > gpurun_out/pe/$name.csv
  rm -rf gpurun_out/pe_$name
}
pe short_graph 180 5 40,90,170 graph &&
NDP_EVENT_FLAGS=0 pe short_graph_timing 180 5 40,90,170 graph &&
DEBUG_CLR_MAX_BATCH_SIZE=1 pe short_graph_b1 180 5 40,90,170 graph
pr() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ps_$name -o run -- python3 bench.py --global-batch 64 --steps 12 --warmup 3 > gpurun_out/ps_$name.out 2>&1 || return 1
  f=$(find gpurun_out/ps_$name -name '*kernel_trace.csv' | head -n 1)
  echo "== $name $(python3 tools/jline.py gpurun_out/ps_$name.out)"
  python3 tools/prof_timeline.py "$f" --steps 8 --dump gpurun_out/ps_$name.last.txt | sed -n 5,9p
  grep -n "psgd_p_kernel" gpurun_out/ps_$name.last.txt | head -4
  rm -rf gpurun_out/ps_$name
}
pr timing_ev NDP_EVENT_FLAGS=0 &&
pr default_ev NDP_EVENT_FLAGS=2
