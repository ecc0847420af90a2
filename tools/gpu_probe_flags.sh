set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf -o run -- python3 tools/probe_flags.py > gpurun_out/pf.out 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/pf.out | tail -3
f=$(find gpurun_out/pf -name '*kernel_trace.csv' | head -n 1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
t0 = None
sel = [r for r in rows if "flag_" in r[3] or "psgd_p_kernel" in r[3] or "conv_fwd_kernel<7, 7" in r[3] or "rank1_step" in r[3]]
t0 = sel[0][0]
for s, e, q, n in sel[-60:]:
    print(f"{(s - t0) / 1e3:12.1f} {(e - s) / 1e3:10.1f} q{q} {n[:40]}")
PY
rm -rf gpurun_out/pf
exit $rc
