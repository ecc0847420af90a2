"""A/B of the attention backward's accumulator chains (csrc/attention.hip NCH = 1 / 2) at the
DistilBERT bench shape (B=16, S=512, H=12, head 64, padding + dropout 0.1).  Times forward +
backward of ops.attention with CUDA events (median of 7 reps of 20 iterations) and checks each arm
against fp64 explicit math.  One JSON line per arm.

    python tools/diag/attn_chains.py > gpurun_out/attn_chains.jsonl

Needs the ``attn_set_chains`` binding, which exists at commit 831b94e only (the two-chain
variant was measured slower and removed; profiles/r5/attn_chains.md).
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from network_distributed_pytorch_amd.ops._ext import ext
from network_distributed_pytorch_amd.ops.attention import attention, attention_reference, dropout_keep_mask


def main():
    dev = "cuda"
    B, S, H, p = 16, 512, 12, 0.1
    g = torch.Generator(device="cpu").manual_seed(2)
    q, k, v = (torch.randn(B, S, H, 64, generator=g).to(dev).requires_grad_() for _ in range(3))
    mask = torch.ones(B, S, dtype=torch.long, device=dev)
    for b in range(B):
        mask[b, 64 + 29 * b:] = 0
    seed = torch.tensor([777], dtype=torch.int32, device=dev)
    go = torch.randn(B, S, H, 64, generator=g).to(dev)
    keep = dropout_keep_mask(777, B, H, S, p, device=dev)
    qd, kd, vd = (t.detach().double().requires_grad_() for t in (q, k, v))
    r = attention_reference(qd, kd, vd, mask, p_drop=p, keep=keep)
    gr = torch.autograd.grad(r, (qd, kd, vd), go.double())
    for nch in (1, 2, 1, 2):
        ext().attn_set_chains(nch)
        o = attention(q, k, v, mask, p_drop=p, seed=seed)
        gq = torch.autograd.grad(o, (q, k, v), go)
        err = max(((a.double() - b).abs().max() / (b.abs().max() + 1e-12)).item() for a, b in zip(gq, gr))
        times = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                o = attention(q, k, v, mask, p_drop=p, seed=seed)
                torch.autograd.grad(o, (q, k, v), go)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / 20)
        print(json.dumps({"chains": nch, "fwd_bwd_us": round(statistics.median(times), 1),
                          "max_rel_err_vs_fp64": err}), flush=True)
    ext().attn_set_chains(1)


if __name__ == "__main__":
    main()
