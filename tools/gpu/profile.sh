#!/bin/bash
# rocprofv3 kernel table of the timed bench steps (tools/prof_summary.py): OUT/kernels_TAG.md
#   tools/gpu/profile.sh OUT TAG NSTEPS [bench args...]
# e.g. tools/gpu/profile.sh gpurun_out/p b64 20 --global-batch 64
# The step marker is the stem convolution (runs once per ResNet step); MARKER overrides it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1; TAG=$2; N=$3; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
MARKER=${MARKER:-conv_fwd_kernel<7, 7}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_$TAG" -o run -- \
  python3 bench.py --no-supervise --steps $((N + 5)) --warmup 5 "$@" > "$OUT/prof_$TAG.out" 2>&1 \
  || { echo "profile $TAG failed"; tail -5 "$OUT/prof_$TAG.out"; exit 1; }
f=$(find "$OUT/prof_$TAG" -name '*kernel_trace.csv' | head -n 1)
{
  echo "<!-- regenerate: tools/gpu/profile.sh OUT $TAG $N $* -->"
  python3 tools/prof_summary.py "$f" --steps "$N" --marker "$MARKER" --top 90
} > "$OUT/kernels_$TAG.md"
head -5 "$OUT/kernels_$TAG.md"
rm -rf "$OUT/prof_$TAG"
