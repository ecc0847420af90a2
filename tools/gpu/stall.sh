#!/bin/bash
# SQ stall / activity counters per kernel for a small program (one rocprofv3 pass per counter set)
#   tools/gpu/stall.sh OUT prog.py [args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/st$i" -o run -- python3 "$@" > "$OUT/st$i.out" 2>&1 \
    || { echo "pass $i failed"; tail -5 "$OUT/st$i.out"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.defaultdict(set)
for f in glob.glob(f"{out}/st*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[k].add(r.get("Dispatch_Id"))
for k, d in acc.items():
    if "wino" not in k and "conv_" not in k: continue
    n = max(1, len(cnt[k]) // 2)
    print(k, "dispatches", n)
    for c in sorted(d): print(f"   {c:28s} {d[c] / n:14.0f}")
PY
