# Verification at the final round-2 state: full GPU suite, smoke(), default bench + shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gputests_verify.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/gputests_verify.log | tail -8
case $rc in 0|1) ;; *) echo "pytest rc=$rc (crash/timeout): stopping"; exit 1 ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_verify.log 2>&1 || { tail -10 gpurun_out/smoke_verify.log; exit 1; }
tail -1 gpurun_out/smoke_verify.log
b() {  # name, bench args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/ver_$name.json 2> gpurun_out/ver_$name.err || { tail -5 gpurun_out/ver_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ver_$name.json)"
}
b default && b r18_256 --global-batch 256 --steps 60 && b r18_128 --global-batch 128 --steps 60 &&
b r18_64 --global-batch 64 --steps 60 && b bert8 --model distilbert --rank 8 --steps 20 --warmup 5
