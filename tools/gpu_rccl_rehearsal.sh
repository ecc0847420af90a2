# one-GPU rehearsal of the N>1 RCCL path: 1-rank nccl process group with collectives forced on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp NDP_FORCE_COLLECTIVES=1
run() {  # name, port, args...
  local name=$1 port=$2; shift 2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --steps 20 --warmup 5 "$@" > gpurun_out/rh_$name.json 2> gpurun_out/rh_$name.err
  local rc=$?
  echo "$name rc=$rc $(cat gpurun_out/rh_$name.json)"
  [ $rc -eq 0 ] || { tail -15 gpurun_out/rh_$name.err; return $rc; }
}
run psgd_pw 29541 --graph-mode piecewise &&
run psgd_eager 29542 --graph-mode none &&
run dense_eager 29543 --reducer dense --graph-mode none &&
run dense_pw 29544 --reducer dense --graph-mode piecewise &&
run psgd_full 29545 --graph-mode full
