#!/bin/bash
# Run a list of GPU steps, each under its own time limit, stopping at the first failure.
#   tools/gpu/run_steps.sh OUTDIR "SECS|NAME|command" ...
# Each step's stdout+stderr goes to OUTDIR/NAME.log; a progress line is printed per step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  secs=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  tail -n 4 "$OUT/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
