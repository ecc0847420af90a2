"""Render `profiles/link_curves.md` tables from the bandwidth_sweep JSONL records.

    python tools/link_curves_md.py profiles/r3/link_curves.jsonl > tables.md

One table per (model, emulated N): PowerSGD vs dense side by side, per link setting.
"""
import json
import sys
from collections import OrderedDict


def main(path):
    recs = [json.loads(ln) for ln in open(path) if ln.strip()]
    groups = OrderedDict()
    for r in recs:
        groups.setdefault((r["config"]["model"], r["n"]), {})[(r["reducer"], r["link"])] = r
    out = []
    for (model, n), g in groups.items():
        any_r = next(iter(g.values()))
        b = any_r["config"]["per_gpu_batch"]
        title = ("DistilBERT IMDb-shape (seq 512)" if model == "distilbert" else
                 f"{model} CIFAR-shape") + f", PowerSGD r=4 vs dense, emulated N={n} (per-GPU batch {b})"
        out += [f"## {title}", "",
                "| link | PowerSGD samples/s | PowerSGD ms/step | dense samples/s | dense ms/step | PowerSGD speed-up | "
                "collectives (PowerSGD / dense) |",
                "|---|---:|---:|---:|---:|---:|---:|"]
        for link in ("none", "100g", "10g", "1g"):
            p, d = g.get(("powersgd", link)), g.get(("dense", link))
            if p is None or d is None:
                continue
            # whole emulated job: N x per-GPU batch / step
            sp, sd = n * b * 1000.0 / p["ms_per_step"], n * b * 1000.0 / d["ms_per_step"]
            out.append(f"| {link} | {sp:,.0f} | {p['ms_per_step']:.2f} | {sd:,.0f} | {d['ms_per_step']:.2f} | "
                       f"{d['ms_per_step'] / p['ms_per_step']:.2f}x | {len(p['collective_payloads'])} / "
                       f"{len(d['collective_payloads'])} |")
        p = g.get(("powersgd", "none"))
        d = g.get(("dense", "none"))
        if p and d:
            out += ["", f"bytes all-reduced per rank per step: PowerSGD {p['bytes_per_step']:,} vs dense "
                        f"{d['bytes_per_step']:,} ({d['bytes_per_step'] / p['bytes_per_step']:.1f}x less)."]
        out.append("")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1])
