#!/usr/bin/env python3
"""Link-bandwidth scaling curves: PowerSGD vs dense all-reduce at 1/10/100 Gb (reference
README.md:2: "Internel / 1Gb / 10Gb / 100Gb distributed learning experiment").

The GPU boxes have no root (no ``tc``) and one GPU per call, so links are emulated: after
every collective the stream that carries it stalls for ``alpha + 8 * ring_wire_bytes /
bandwidth`` with ring wire bytes ``2 (N-1)/N * payload`` (``parallel/comm.py`` LinkModel,
``ops.delay_ns``).  The per-collective payloads are the real ones of each engine
(``sync.collective_payloads()``: PowerSGD [P_g, Q_g] per overlap group + the rank-1
buffer; dense: one per bucket).

Modes:
  emulate — ONE GPU, ``bench.py --link L --emulate-world N``: the real training step runs
            and the pacing kernels really stall the comm stream, so whatever overlap the
            engine achieves with backward is part of the number.  Label: "emulated on 1 GPU".
  model   — the measured 1-GPU step time + the link time of every collective added
            serially (no overlap credited: an upper bound on the step time).
  measure — real N-GPU runs with link pacing (needs an N-GPU node).

    python tools/bandwidth_sweep.py --mode emulate --gpus 8 --model distilbert --rank 4
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_bench(args, reducer, link, gpus, emulate=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--model", args.model, "--reducer", reducer, "--rank", str(args.rank), "--link", link,
           "--weak-too", "off", "--overlap", args.overlap]
    if args.batch:
        cmd += ["--batch", str(args.batch)]
    if emulate:
        cmd += ["--emulate-world", str(emulate)]
        if not args.model.startswith("distilbert") and not args.batch:
            cmd += ["--global-batch", str(512 // emulate)]  # the per-GPU shape of the N-GPU strong run
    if gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(29600 + hash((reducer, link)) % 200)] + cmd[1:]
        cmd += ["--gpus", str(gpus)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout)
    for line in reversed(out.stdout.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"bench failed: {out.stderr[-2000:]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["emulate", "model", "measure"], default="emulate")
    ap.add_argument("--gpus", type=int, default=8, help="N of the (emulated) ring")
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--rank", type=int, default=4)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--timeout", type=int, default=900)
    ap.add_argument("--links", default="none,100g,10g,1g")
    ap.add_argument("--reducers", default="powersgd,dense")
    ap.add_argument("--jsonl", default=None, help="append every bench record here")
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="on",
                    help="gradient sync overlapped with backward on EVERY arm, the 'none' link included "
                         "(the shipped N > 1 default), so the rows differ only in the link")
    args = ap.parse_args()
    from network_distributed_pytorch_amd.parallel.comm import LINK_PRESETS

    links = args.links.split(",")
    rows = []
    for red in args.reducers.split(","):
        base = None
        for link in links:
            if args.mode == "measure":
                rec = run_bench(args, red, link, args.gpus)
                how = f"measured, {args.gpus} GPUs"
            elif args.mode == "emulate":
                rec = run_bench(args, red, link, 1, emulate=args.gpus)
                how = f"emulated on 1 GPU (N={args.gpus} ring charged)"
            else:
                base = base or run_bench(args, red, "none", 1, emulate=args.gpus)
                rec = dict(base)
                t = base["ms_per_step"] / 1e3
                if link != "none":
                    lm = LINK_PRESETS[link]
                    t += sum(lm.seconds(int(b), args.gpus) for b in base["collective_payloads"])
                rec["ms_per_step"] = 1e3 * t
                how = "modelled: measured 1-GPU step + serial link time"
            per_gpu = rec["config"]["per_gpu_batch"]
            sps = per_gpu * args.gpus / (rec["ms_per_step"] / 1e3)
            rows.append((red, link, sps, rec["ms_per_step"], rec["bytes_per_step"],
                         len(rec.get("collective_payloads") or []), how))
            if args.jsonl:
                with open(args.jsonl, "a") as f:
                    f.write(json.dumps({"mode": args.mode, "link": link, "reducer": red, "n": args.gpus, **rec}) + "\n")
    print(f"| reducer | link | samples/s (N={args.gpus}, whole job) | ms/step | bytes/step/rank | collectives | how |")
    print("|---|---|---:|---:|---:|---:|---|")
    for r in rows:
        print(f"| {r[0]} | {r[1]} | {r[2]:.1f} | {r[3]:.2f} | {r[4]} | {r[5]} | {r[6]} |")


if __name__ == "__main__":
    main()
