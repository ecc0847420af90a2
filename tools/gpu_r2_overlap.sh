# round 2: overlap + native RCCL tests, then A/B benches (overlap vs serial, 1-rank RCCL rehearsal)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_overlap_gpu.py tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_overlap.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_overlap.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/ov_$name.json 2> gpurun_out/ov_$name.err || { tail -5 gpurun_out/ov_$name.err; return 1; }
  python3 tools/jline.py gpurun_out/ov_$name.json
}
rh() {  # 1-rank RCCL rehearsal: name, port, args...
  local name=$1 port=$2; shift 2
  NDP_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py "$@" > gpurun_out/ov_$name.json 2> gpurun_out/ov_$name.err || { tail -8 gpurun_out/ov_$name.err; return 1; }
  python3 tools/jline.py gpurun_out/ov_$name.json
}
b b512_ov --steps 40 --warmup 10 &&
b b512_serial --steps 40 --warmup 10 --no-overlap &&
b b64_ov --global-batch 64 --steps 40 --warmup 10 &&
b b64_serial --global-batch 64 --steps 40 --warmup 10 --no-overlap &&
rh rh512_ov 29561 --steps 40 --warmup 10 &&
rh rh512_serial 29562 --steps 40 --warmup 10 --no-overlap &&
rh rh64_ov 29563 --global-batch 64 --steps 40 --warmup 10 &&
rh rh_dense512 29564 --reducer dense --steps 40 --warmup 10 &&
b dense512 --reducer dense --steps 40 --warmup 10 || exit 1
}
p b64_ov --global-batch 64 &&
p b64_serial --global-batch 64 --no-overlap &&
p b512_ov &&
p b512_serial --no-overlap
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
