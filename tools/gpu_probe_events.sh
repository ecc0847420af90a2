set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pe -o run -- python3 tools/probe_events.py > gpurun_out/pe.out 2>&1; rc=$?
tail -3 gpurun_out/pe.out
f=$(find gpurun_out/pe -name '*kernel_trace.csv' | head -n 1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), r["Kernel_Name"][:20]) for r in csv.DictReader(open(sys.argv[1])))
rows = rows[-30:]
t0 = rows[0][0]
for s, e, q, n in rows:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{q} {n}")
PY
rm -rf gpurun_out/pe
exit $rc
