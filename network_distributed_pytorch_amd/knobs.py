"""The framework's A/B switches, in one place.

Every native fusion is on by default; each was adopted by a measured A/B on 1x MI355X (the
verdicts are in the docstrings of the modules named below and in profiles/r*/README.md).
``NDP_FUSION_OFF`` — a comma-separated list of the names below, or ``all`` — turns fusions
off for an A/B arm or a bisection without touching the code; tests flip the module
constants directly.  The remaining environment variables are operational, not tuning:

  NDP_COMM / NDP_NATIVE_COMM / NDP_FORCE_COLLECTIVES / NDP_SIDE_PRIORITY /
  NDP_FLAG_WAIT_US / NDP_EVENT_FLAGS        data plane (parallel/comm.py, csrc/comm.cpp, csrc/ipc.hip)
  NDP_PSGD_OVERLAP / NDP_PSGD_GROUPS         PowerSGD overlap with backward (parallel/powersgd.py)
  NDP_BACKEND / NDP_BENCH_FAIL               bench.py (process-group backend, fault injection)
  NDP_SUP_DIR / NDP_SUP_ROLE / NDP_SUP_LEVEL supervisor plumbing (utils/supervisor.py)
"""
from __future__ import annotations

import os

__all__ = ["FUSIONS", "fusion_on"]

FUSIONS = {
    "slab_links": "split-K conv slabs summed by the neighbouring BN kernel (models/resnet.py, ops/slablink.py)",
    "branch_links": "downsample-block grad-x of conv1 + 1x1 downsample shared in place (ops/gradlink.py)",
    "conv_bnstats": "BN forward statistics from the direct-conv epilogue (ops/conv.py)",
    "bn_bwd_stats": "BN backward statistics from the grad-x epilogue / pool backward (ops/batchnorm.py)",
    "bn_vec4": "float4 single-launch small-map BN kernel (csrc/batchnorm.hip; off: the scalar one)",
    "winograd": "F(2x2,3x3) Winograd for the layer1 3x3 forward / grad-x (csrc/winograd.hip)",
    "wino_pair": "a conv's grad-x and grad-W in one launch (csrc/winograd.hip, csrc/conv.hip pairs)",
    "ds_fwd_pair": "a downsample block's conv1 and 1x1 downsample forward in one launch (csrc/conv.hip)",
    "stem_pool": "stem BN -> ReLU -> max-pool in one pass (ops/batchnorm.py)",
    "stem_bwd": "stem max-pool backward + BN backward apply from the pooled gradient in one pass (ops/batchnorm.py)",
    "bn_pair": "downsample block's bn2 + downsample BN + ReLU in one launch per direction (ops/batchnorm.py)",
    "defer_gradw": "grad-W slab sums / folds batched at the end of backward (ops/gradfinish.py)",
    "grad_arena": "dense-arm gradients written straight into the bucket arena (ops/gradarena.py)",
    "tgemm": "strided / tabled MFMA GEMM convs for 1x1 layers (ops/tgconv.py)",
    "tuned_gemms": "hipBLASLt algorithm table for the Toeplitz GEMMs (ops/gemm_tuning.py)",
    "lazy_ef": "PowerSGD error feedback formed in the next P pass (parallel/powersgd.py)",
    "psgd_fin": "PowerSGD P / Q split-K sums, rank-1 pack and rank-1 step inside the P / Q / update launches",
    "defer_uploads": "capture-safe table uploads batched per graph (utils/graph.py)",
    "fused_ce": "native softmax cross-entropy (ops/loss.py)",
    "fused_ln": "native residual add + LayerNorm (+ dropout) (ops/layernorm.py)",
    "ln_links": "DistilBERT residual gradients folded into the sublayer GEMMs (models/distilbert.py)",
    "packed_qkv": "one QKV projection GEMM over the three weights in place (models/distilbert.py)",
    "fused_gelu": "native GELU backward + bias column sums (ops/linear.py)",
}

_OFF = {t.strip() for t in os.environ.get("NDP_FUSION_OFF", "").split(",") if t.strip()}
_unknown = _OFF - set(FUSIONS) - {"all"}
if _unknown:
    raise ValueError(f"NDP_FUSION_OFF: unknown fusion(s) {sorted(_unknown)}; known: {sorted(FUSIONS)}")


def fusion_on(name: str) -> bool:
    """Whether fusion ``name`` (a key of :data:`FUSIONS`) is enabled in this process."""
    if name not in FUSIONS:
        raise KeyError(name)
    return "all" not in _OFF and name not in _OFF
