#!/bin/bash
# rocprofv3 kernel statistics of one command: OUT/TAG_stats.csv (+ a short top list on stdout)
#   tools/gpu/kstats.sh OUT TAG cmd...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1; TAG=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- "$@" > "$OUT/prof_$TAG.out" 2>&1 \
  || { echo "profile $TAG failed"; tail -5 "$OUT/prof_$TAG.out"; exit 1; }
f=$(find "$OUT/prof_$TAG" -name '*kernel_stats.csv' | head -n 1)
cp "$f" "$OUT/${TAG}_stats.csv"
python3 - "$OUT/${TAG}_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e3:10.1f} us {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:110]}")
PY
rm -rf "$OUT/prof_$TAG"
