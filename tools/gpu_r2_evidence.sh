# round 2 evidence: full GPU test suite, then the headline bench and the strong-scaling
# per-GPU shapes (512/N for N = 1, 2, 4, 8) overlapped vs serial, and the 1-rank RCCL rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/ev_$name.json 2> gpurun_out/ev_$name.err || { tail -5 gpurun_out/ev_$name.err; return 1; }
  python3 tools/jline.py gpurun_out/ev_$name.json
}
rh() {  # 1-rank RCCL rehearsal: name, port, args...
  local name=$1 port=$2; shift 2
  NDP_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py "$@" > gpurun_out/ev_$name.json 2> gpurun_out/ev_$name.err || { tail -8 gpurun_out/ev_$name.err; return 1; }
  python3 tools/jline.py gpurun_out/ev_$name.json
}
b b512 --steps 50 --warmup 10 &&
b b512_serial --steps 50 --warmup 10 --no-overlap &&
b b256 --global-batch 256 --steps 50 --warmup 10 &&
b b128 --global-batch 128 --steps 50 --warmup 10 &&
b b64 --global-batch 64 --steps 50 --warmup 10 &&
b b64_serial --global-batch 64 --steps 50 --warmup 10 --no-overlap &&
b dense512 --reducer dense --steps 50 --warmup 10 &&
b dense64 --reducer dense --global-batch 64 --steps 50 --warmup 10 &&
rh rh512 29561 --steps 50 --warmup 10 &&
rh rh512_serial 29562 --steps 50 --warmup 10 --no-overlap &&
rh rh64 29563 --global-batch 64 --steps 50 --warmup 10 &&
rh rh64_serial 29564 --global-batch 64 --steps 50 --warmup 10 --no-overlap &&
rh rh_dense512 29565 --reducer dense --steps 50 --warmup 10
