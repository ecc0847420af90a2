# rocprofv3 kernel traces -> per-kernel tables + step timelines (profiles/r2/).
#   bash tools/gpu_r2_prof.sh name "bench args" [name "bench args" ...]
# A name starting with rh_ runs the 1-rank RCCL rehearsal (NDP_FORCE_COLLECTIVES=1, torchrun).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  name=$1; args=$2; shift 2
  case $name in
    rh_*) export NDP_FORCE_COLLECTIVES=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 ;;
    *) unset NDP_FORCE_COLLECTIVES MASTER_ADDR MASTER_PORT RANK LOCAL_RANK WORLD_SIZE ;;
  esac
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$name -o run -- \
    python3 bench.py --steps 25 --warmup 5 $args > gpurun_out/tr_$name.out 2>&1 || { tail -5 gpurun_out/tr_$name.out; exit 1; }
  f=$(find gpurun_out/tr_$name -name '*kernel_trace.csv' | sort | head -n 1)
  python3 tools/prof_timeline.py "$f" --steps ${PSTEPS:-20} --marker "${MARKER:-conv_fwd_kernel<7, 7}" --dump gpurun_out/tr_$name.last.txt > gpurun_out/tr_$name.timeline.md &&
  python3 tools/prof_summary.py "$f" --steps ${PSTEPS:-20} --marker "${MARKER:-conv_fwd_kernel<7, 7}" --top 80 > gpurun_out/tr_$name.kernels.md || exit 1
  echo "== $name: $(python3 tools/jline.py gpurun_out/tr_$name.out)"
  sed -n 5,8p gpurun_out/tr_$name.timeline.md
  rm -rf gpurun_out/tr_$name
done
