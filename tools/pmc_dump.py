#!/usr/bin/env python3
"""Mean of every collected PMC counter per kernel (plus mean duration from a kernel trace).

    python tools/pmc_dump.py --counters a.csv b.csv --trace t.csv [--match tgemm]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    return re.sub(r"\(.*", "", name).replace("void ", "")[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counters", nargs="+", required=True)
    ap.add_argument("--trace", nargs="*", default=[])
    ap.add_argument("--match", default="ndp::")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for c in a.counters:
        for r in csv.DictReader(open(c, newline="")):
            k = short(r["Kernel_Name"])
            if a.match in k:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = collections.defaultdict(list)
    for t in a.trace:
        for r in csv.DictReader(open(t, newline="")):
            k = short(r["Kernel_Name"])
            if a.match in k:
                durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, v in vals.items():
        d = durs.get(k)
        print(f"## {k}  dispatches={max(len(x) for x in v.values())}  mean_us={sum(d) / len(d) / 1e3:.2f}" if d else f"## {k}")
        for cn in sorted(v):
            xs = v[cn]
            print(f"  {cn:32s} {sum(xs) / len(xs):.4g}")


if __name__ == "__main__":
    main()
