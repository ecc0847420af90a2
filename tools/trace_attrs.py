#!/usr/bin/env python3
"""Per-kernel launch attributes and durations from a rocprofv3 kernel_trace.csv (last dispatch of each kernel)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tag = sys.argv[2] if len(sys.argv) > 2 else ""
by = collections.OrderedDict()
for r in rows:
    by.setdefault(r["Kernel_Name"][:60], []).append(r)
for name, rs in by.items():
    r = rs[-1]
    keys = ("LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z")
    durs = [round((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3, 2) for x in rs]
    print(tag, name, {k: r.get(k) for k in keys}, "us:", durs[-3:])
