# Pinned MFMA/LDS interleave for the stem / 3x3-s2 / 1x1-s2 forwards too (NDP_CONV_VARIANT=8).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NDP_CONV_VARIANT=8 timeout -k 10 300 python -u -m pytest tests/test_conv_direct.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s8_tests.log 2>&1 || { tail -20 gpurun_out/s8_tests.log; exit 1; }
tail -1 gpurun_out/s8_tests.log
b() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  echo "$name $(python3 tools/jline.py gpurun_out/ab_$name.json)"
}
for gb in 512 64; do
  b s0_$gb python bench.py --global-batch $gb --steps 60 &&
  b s8_$gb NDP_CONV_VARIANT=8 python bench.py --global-batch $gb --steps 60 &&
  b s0b_$gb python bench.py --global-batch $gb --steps 60 &&
  b s8b_$gb NDP_CONV_VARIANT=8 python bench.py --global-batch $gb --steps 60 || exit 1
done
