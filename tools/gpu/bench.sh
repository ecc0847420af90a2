#!/bin/bash
# Run bench.py for a list of configurations; one JSON line per config into OUT/bench.jsonl.
#   tools/gpu/bench.sh OUT "label|--bench --args" ["label2|..."] ...
# e.g. tools/gpu/bench.sh gpurun_out/b "b512|" "b64|--global-batch 64" "r152|--model resnet152"
# Environment A/B arms: prefix the args with VAR=value words ("nobn|NDP_X=0 --global-batch 64").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-30}
WARM=${WARM:-10}
for spec in "$@"; do
  label=${spec%%|*}
  rest=${spec#*|}
  envs=(); args=()
  for w in $rest; do
    if [[ $w == NDP_*=* || $w == HIP_*=* ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps "$STEPS" --warmup "$WARM" "${args[@]}" \
    > "$OUT/$label.json" 2> "$OUT/$label.err" || { echo "$label FAILED"; tail -5 "$OUT/$label.err"; exit 1; }
  line=$(grep '^{' "$OUT/$label.json" | tail -n 1)
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); d['ab_arm']=sys.argv[2]; print(json.dumps(d))" \
    "$line" "$spec" >> "$OUT/bench.jsonl"
  echo "$label $(python3 tools/jline.py "$OUT/$label.json")"
done
