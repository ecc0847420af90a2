#!/usr/bin/env python3
"""Link-bandwidth scaling curves: PowerSGD vs dense all-reduce at 1/10/100 Gb (+ native xGMI).

The reference's experiments ran over physical 1/10/100 GbE links (README.md:2).  The GPU
boxes have no root (no ``tc``), so links are emulated: every collective is followed by a
wall-clock stall of ``alpha + 8 * ring_wire_bytes / bandwidth`` on the HIP stream
(``parallel/comm.py`` LinkModel, ``ops.delay_ns``).

Two modes:
  measure  — run ``bench.py`` under torchrun for each (reducer, link) at ``--gpus N``
             (needs N GPUs); prints a markdown table of samples/s.
  model    — take the measured 1-GPU step time of each reducer (runs bench.py at N=1) and
             add the link model's time for that reducer's collectives at N ranks (the
             collectives of a step are serial after backward in the PowerSGD engine, and
             the dense arm's buckets are charged serially too: an upper bound on its comm).

    python tools/bandwidth_sweep.py --mode model --gpus 8 --model distilbert --rank 4
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_bench(args, reducer, link, gpus):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--model", args.model, "--reducer", reducer, "--rank", str(args.rank), "--link", link]
    if args.batch:
        cmd += ["--batch", str(args.batch)]
    if gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(29600 + hash((reducer, link)) % 200)] + cmd[1:]
        cmd += ["--gpus", str(gpus)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout)
    for line in reversed(out.stdout.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"bench failed: {out.stderr[-2000:]}")


def collectives(rec, reducer):
    """(payload bytes per collective) for one step of the given reducer."""
    if reducer.startswith("powersgd"):
        total = rec["bytes_per_step"]
        # [P | rank-1] and Q: split by the reference accounting is not needed for the
        # ring model (time is linear in bytes) beyond the per-collective alpha
        return [total / 2.0, total / 2.0]
    n = max(1, int(round(rec["dense_bytes_per_step"] / (25 * 1024 * 1024))))
    return [rec["dense_bytes_per_step"] / n] * n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["measure", "model"], default="model")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--rank", type=int, default=4)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--timeout", type=int, default=900)
    args = ap.parse_args()
    from network_distributed_pytorch_amd.parallel.comm import LINK_PRESETS

    links = ["none", "100g", "10g", "1g"]
    rows = []
    if args.mode == "measure":
        for red in ("powersgd", "dense"):
            for link in links:
                rec = run_bench(args, red, link, args.gpus)
                rows.append((red, link, rec["value"], rec["ms_per_step"], rec["bytes_per_step"], "measured"))
    else:
        for red in ("powersgd", "dense"):
            base = run_bench(args, red, "none", 1)
            gb = base["config"]["per_gpu_batch"] * args.gpus
            for link in links:
                t = base["ms_per_step"] / 1e3
                if link != "none":
                    lm = LINK_PRESETS[link]
                    t += sum(lm.seconds(int(b), args.gpus) for b in collectives(base, red))
                rows.append((red, link, gb / t, 1e3 * t, base["bytes_per_step"],
                             "modelled: measured 1-GPU step + link model"))
    print(f"| reducer | link | samples/s (N={args.gpus}) | ms/step | bytes/step | how |")
    print("|---|---|---:|---:|---:|---|")
    for r in rows:
        print(f"| {r[0]} | {r[1]} | {r[2]:.1f} | {r[3]:.2f} | {r[4]} | {r[5]} |")


if __name__ == "__main__":
    main()
