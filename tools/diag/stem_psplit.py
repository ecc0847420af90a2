"""Stem 7x7/2 forward (with the BN statistics epilogue) per output-row split (conv.hip PSPLIT)
and per-GPU batch: median µs of 50 launches after warm-up.  One JSON line per (batch, split).

    python tools/diag/stem_psplit.py > gpurun_out/stem_psplit.jsonl
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from network_distributed_pytorch_amd.ops._ext import ext  # noqa: E402


def main():
    X = ext()
    geom = [3, 32, 32, 64, 7, 7, 2, 3]
    for B in (64, 128, 256, 512):
        x = torch.randn(B, 3, 32, 32, device="cuda")
        w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
        y = torch.empty(B, 64, 16, 16, device="cuda")
        for ps in (1, 2, 4):
            X.conv_set_stem_psplit(ps)
            S = int(X.conv_stats_slices(geom, B))
            stats = torch.empty(64 * S * 2, device="cuda", dtype=torch.float64)
            for _ in range(5):
                X.conv_fwd(x, w, y, geom, None, False, stats)
            ts = []
            for _ in range(7):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    X.conv_fwd(x, w, y, geom, None, False, stats)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 50)
            print(json.dumps({"batch": B, "psplit": ps, "us": round(statistics.median(ts), 2)}), flush=True)
    X.conv_set_stem_psplit(0)


if __name__ == "__main__":
    main()
