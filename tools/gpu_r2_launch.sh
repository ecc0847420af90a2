# host-side graph launch cost vs GPU step time, under HIP runtime graph-launch knobs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label, env assignments..., -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 180 python tools/probe_launch.py "$@" > gpurun_out/pl_$label.json 2> gpurun_out/pl_$label.err || { tail -5 gpurun_out/pl_$label.err; return 1; }
  echo "$label $(tail -n 1 gpurun_out/pl_$label.json)"
}
for b in 64 512; do
  run def_$b X=1 -- --global-batch $b &&
  run bs8_$b DEBUG_HIP_GRAPH_BATCH_SIZE=8 -- --global-batch $b &&
  run bs256_$b DEBUG_HIP_GRAPH_BATCH_SIZE=256 -- --global-batch $b &&
  run pc0_$b DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 -- --global-batch $b &&
  run pc1_$b DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 -- --global-batch $b &&
  run serial_$b X=1 -- --global-batch $b --no-overlap || exit 1
done
