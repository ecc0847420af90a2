# Full GPU suite; BranchLink / slab-cap A/B; kernel tables; 1-rank RCCL rehearsal (no profiler).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/gputests.log | tail -12
case $rc in 0|1) ;; *) echo "pytest rc=$rc (crash/timeout): stopping"; exit 1 ;; esac
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
b bert8 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bert8_nolnk NDP_LN_LINKS=0 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bert8_noqkv NDP_PACKED_QKV=0 python bench.py --model distilbert --rank 8 --steps 20 --warmup 5 || exit 1
for gb in 64 512; do
  b br_$gb python bench.py --global-batch $gb --steps 60 &&
  b nobr_$gb NDP_BRANCH_LINKS=0 python bench.py --global-batch $gb --steps 60 &&
  b br2_$gb python bench.py --global-batch $gb --steps 60 || exit 1
done
b cur_256 python bench.py --global-batch 256 --steps 60 && b cur_128 python bench.py --global-batch 128 --steps 60 || exit 1
rh() {  # 1-rank RCCL rehearsal of the N>1 path
  local name=$1; shift
  NDP_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29577 bench.py "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
rh rh_ov_64 --global-batch 64 --steps 60 --overlap on && rh rh_ser_64 --global-batch 64 --steps 60 --overlap off &&
rh rh_ov_512 --steps 60 --overlap on && rh rh_ser_512 --steps 60 --overlap off || exit 1
bash tools/gpu_r2_prof.sh r18_b512 "" r18_b64 "--global-batch 64"
