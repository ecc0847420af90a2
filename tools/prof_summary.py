#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV over the last K training steps.

Steps are delimited by a marker kernel that runs once per step (default: the PowerSGD
fused update kernel).  Prints per-kernel µs/step, launches/step, GPU-busy and wall time
per step as a markdown table (committed under profiles/).

    python tools/prof_summary.py run_kernel_trace.csv --steps 20 --marker psgd_update_kernel
"""
import argparse
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)", "anon")
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    return name[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="psgd_update_kernel")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sequence", default=None, help="also write the last step's kernel sequence here")
    a = ap.parse_args()
    rows = []
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < a.steps + 1:
        print(f"only {len(marks)} marker kernels found", file=sys.stderr)
        k = max(1, len(marks) - 1)
    else:
        k = a.steps
    lo, hi = marks[-k - 1] + 1, marks[-1] + 1
    win = rows[lo:hi]
    wall = win[-1][1] - rows[marks[-k - 1]][1]
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for s, e, n in win:
        agg[short(n)][0] += e - s
        agg[short(n)][1] += 1
        busy += e - s
    print(f"# kernel summary over last {k} steps (marker `{a.marker}`)\n")
    print(f"- wall per step: {wall / k / 1e3:.1f} µs; GPU kernel-busy per step: {busy / k / 1e3:.1f} µs; "
          f"launches per step: {len(win) / k:.0f}\n")
    print("| kernel | µs/step | launches/step | % busy |")
    print("|---|---:|---:|---:|")
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[: a.top]:
        print(f"| `{n}` | {t / k / 1e3:.1f} | {c / k:.1f} | {100 * t / busy:.1f} |")
    if a.sequence:  # one step in launch order: µs, gap before it, name (find who launches what)
        last = rows[marks[-2] + 1: marks[-1] + 1]
        with open(a.sequence, "w") as f:
            prev = rows[marks[-2]][1]
            for s, e, n in last:
                f.write(f"{(e - s) / 1e3:8.1f} {(s - prev) / 1e3:6.1f}  {short(n)}\n")
                prev = e


if __name__ == "__main__":
    main()
