# Round-end evidence: full GPU suite, smoke(), default bench, and every reference config.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gputests_final.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/gputests_final.log | tail -8
case $rc in 0|1) ;; *) echo "pytest rc=$rc (crash/timeout): stopping"; exit 1 ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -10 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
b() {  # name, bench args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/fin_$name.json 2> gpurun_out/fin_$name.err || { tail -5 gpurun_out/fin_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/fin_$name.json)"
}
b default &&
b r18_dense --reducer dense --steps 60 &&
b r18_256 --global-batch 256 --steps 60 && b r18_128 --global-batch 128 --steps 60 && b r18_64 --global-batch 64 --steps 60 &&
b r50_dense --model resnet50 --reducer dense --steps 20 --warmup 5 &&
b r50_psgd --model resnet50 --steps 20 --warmup 5 &&
b r152_psgd --model resnet152 --steps 20 --warmup 5 &&
b bert4 --model distilbert --rank 4 --steps 20 --warmup 5 &&
b bert8 --model distilbert --rank 8 --steps 20 --warmup 5 &&
b bert16 --model distilbert --rank 16 --steps 20 --warmup 5 &&
b bert_dense --model distilbert --reducer dense --steps 20 --warmup 5
