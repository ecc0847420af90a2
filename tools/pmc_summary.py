#!/usr/bin/env python3
"""Per-kernel PMC summary from rocprofv3 --pmc CSVs (+ the same run's kernel trace).

    python tools/pmc_summary.py --counters run_counter_collection.csv [--trace run_kernel_trace.csv]
        [--match psgd_,seg_reduce,conv_] [--skip 1]

Prints one row per kernel (mean per dispatch over the matching dispatches): duration,
HBM-side bytes (FETCH_SIZE doubled — on gfx950 it reports half of a coalesced stream's
bytes, MI355X_MICROARCH.md — plus WRITE_SIZE, both KB), achieved GB/s, f32 MFMA TFLOP/s
(SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 FLOP), MFMA-busy cycles per CU-cycle of the dispatch
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs)), L2 hit rate and the LDS bank-conflict
share of LDS-active cycles, when those counters were collected.
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    name = re.sub(r"\(.*", "", name).replace("void ", "")
    return name[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counters", nargs="+", required=True)
    ap.add_argument("--trace", nargs="*", default=[])
    ap.add_argument("--match", default="ndp::")
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    pats = [p for p in a.match.split(",") if p]
    dur = {}
    for t in a.trace:
        with open(t, newline="") as f:
            for r in csv.DictReader(f):
                dur[(t, r.get("Dispatch_Id") or r.get("Correlation_Id"))] = (
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), short(r["Kernel_Name"]))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    names = {}
    for c in a.counters:
        with open(c, newline="") as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                if pats and not any(p in k for p in pats):
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                names[did] = k
    durs = collections.defaultdict(list)
    for (_, did), (d, k) in dur.items():
        if pats and not any(p in k for p in pats):
            continue
        durs[k].append(d)
    mean = lambda xs: sum(xs) / len(xs) if xs else float("nan")  # noqa: E731
    print("| kernel | dispatches | µs | HBM read MB (2x FETCH) | HBM write MB | GB/s | MFMA f32 TFLOP/s | "
          "MFMA busy / CU-cycle % | L2 hit % | LDS conflict % |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in sorted(vals, key=lambda k: -mean(durs.get(k, [0])) * len(durs.get(k, [1]))):
        v = vals[k]
        us = mean(durs.get(k, [])) / 1e3 if durs.get(k) else float("nan")
        rd = 2 * mean(v.get("FETCH_SIZE", [])) * 1024 / 1e6
        wr = mean(v.get("WRITE_SIZE", [])) * 1024 / 1e6
        gbs = (rd + (wr if wr == wr else 0)) / (us * 1e-6) / 1e3 if us == us and us > 0 else float("nan")
        gui = mean(v.get("GRBM_GUI_ACTIVE", []))
        mfma = mean(v.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        mops = mean(v.get("SQ_INSTS_VALU_MFMA_MOPS_F32", []))
        tflops = mops * 512 / (us * 1e-6) / 1e12 if us == us and us > 0 and mops == mops else float("nan")
        hit, miss = mean(v.get("TCC_HIT_sum", [])), mean(v.get("TCC_MISS_sum", []))
        lds, conf = mean(v.get("SQ_LDS_IDX_ACTIVE", [])), mean(v.get("SQ_LDS_BANK_CONFLICT", []))
        n = max((len(x) for x in v.values()), default=0)
        f = lambda x, p=1: "-" if x != x else f"{x:.{p}f}"  # noqa: E731
        print(f"| `{k}` | {n} | {f(us)} | {f(rd, 2)} | {f(wr, 2)} | {f(gbs, 0)} | {f(tflops)} | "
              f"{f(100 * mfma / (gui * a.cus) if gui == gui and gui else float('nan'))} | "
              f"{f(100 * hit / (hit + miss) if hit + miss else float('nan'))} | "
              f"{f(100 * conf / lds if lds else float('nan'))} |")


if __name__ == "__main__":
    main()
