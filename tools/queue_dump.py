#!/usr/bin/env python3
"""Dump the tail of a rocprofv3 kernel trace, collapsing runs of same-queue same-kernel rows."""
import csv
import re
import sys

rows = []
with open(sys.argv[1], newline="") as f:
    for r in csv.DictReader(f):
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:60]))
rows.sort()
tail = rows[-int(sys.argv[2]):]
t0 = tail[0][0]
i = 0
while i < len(tail):
    j = i
    while j + 1 < len(tail) and tail[j + 1][2] == tail[i][2] and tail[j + 1][3] == tail[i][3]:
        j += 1
    s, e = tail[i][0], tail[j][1]
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  q{tail[i][2]:>3} x{j - i + 1:<4} {tail[i][3]}")
    i = j + 1
