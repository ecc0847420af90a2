#!/bin/bash
# Full verification at HEAD: GPU test suite, smoke(), then the headline + strong-scaling
# shapes + reference configs through tools/gpu/bench.sh.
#   tools/gpu/verify.sh OUT [quick]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" "$OUT/pytest.log" | tail -2; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -n 1 "$OUT/smoke.log"
if [ "$2" = quick ]; then
  tools/gpu/bench.sh "$OUT" "b512|" "b64|--global-batch 64"
else
  tools/gpu/bench.sh "$OUT" "b512|" "b256|--global-batch 256" "b128|--global-batch 128" "b64|--global-batch 64" \
    "dense512|--reducer dense" "r152|--model resnet152" "r50d|--model resnet50 --reducer dense" \
    "r50p|--model resnet50" "bert8|--model distilbert --rank 8"
fi
