#!/usr/bin/env python3
"""Per-step timeline statistics from a rocprofv3 --kernel-trace CSV: wall, busy (union of
kernel intervals), idle, time with >= 2 kernels in flight (overlap), per-queue busy time —
the evidence that side-stream bucket / PowerSGD-group work runs concurrently with backward.

Steps are delimited by the START of a marker kernel launched once per step (default: the
ResNet stem convolution).

    python tools/prof_timeline.py run_kernel_trace.csv --steps 20 [--dump last_step.txt]
"""
import argparse
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)", "anon")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")[:90]


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def overlap_len(iv):
    """Time covered by >= 2 intervals."""
    ev = []
    for s, e in iv:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    depth, last, tot = 0, None, 0
    for t, d in ev:
        if depth >= 2 and last is not None:
            tot += t - last
        depth += d
        last = t
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="conv_fwd_kernel<7, 7")
    ap.add_argument("--dump", default=None, help="write the last step's kernels (start, dur, queue, name)")
    a = ap.parse_args()
    rows = []
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, r["Kernel_Name"]))
    rows.sort()
    marks = [r[0] for r in rows if a.marker in r[3]]
    if len(marks) < 3:
        sys.exit(f"only {len(marks)} marker kernels")
    k = min(a.steps, len(marks) - 1)
    bounds = marks[-k - 1:]
    stats = collections.defaultdict(float)
    per_q = collections.defaultdict(float)
    last = None
    for i in range(k):
        t0, t1 = bounds[i], bounds[i + 1]
        win = [r for r in rows if t0 <= r[0] < t1]
        iv = [(max(s, t0), min(e, t1)) for s, e, _, _ in win]
        stats["wall"] += t1 - t0
        stats["busy"] += union_len(iv)
        stats["overlap"] += overlap_len(iv)
        stats["kernel_sum"] += sum(e - s for s, e in iv)
        stats["launches"] += len(win)
        for s, e, q, _ in win:
            per_q[q] += e - s
        last = (t0, win)
    us = lambda v: v / k / 1e3  # noqa: E731  (ns -> us per step)
    print(f"# timeline over last {k} steps (marker `{a.marker}`)\n")
    print("| per step | µs |")
    print("|---|---:|")
    print(f"| wall | {us(stats['wall']):.1f} |")
    print(f"| GPU busy (union of kernels) | {us(stats['busy']):.1f} |")
    print(f"| idle | {us(stats['wall'] - stats['busy']):.1f} |")
    print(f"| >= 2 kernels in flight (overlap) | {us(stats['overlap']):.1f} |")
    print(f"| sum of kernel durations | {us(stats['kernel_sum']):.1f} |")
    print(f"| launches | {stats['launches'] / k:.0f} |")
    print("\n| queue | kernel µs/step |")
    print("|---|---:|")
    for q, v in sorted(per_q.items(), key=lambda x: -x[1]):
        print(f"| {q} | {us(v):.1f} |")
    if a.dump and last is not None:
        t0, win = last
        with open(a.dump, "w") as f:
            for s, e, q, n in win:
                f.write(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {short(n)}\n")


if __name__ == "__main__":
    main()
