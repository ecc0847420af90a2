"""Measured GEMM solution table for the framework's library GEMMs (PyTorch TunableOp).

The plain library GEMMs left in a step — the Toeplitz convolutions of ResNet layer3 /
layer4 (models/conv_gemm.py), the classifier heads and DistilBERT's projections — are
skinny fp32 products (M = per-GPU batch = 64 .. 512 rows) that are latency-bound on 256 CUs.
hipBLASLt's default heuristic picks a tile per shape without measuring; PyTorch-ROCm's
TunableOp can instead time every rocBLAS / hipBLASLt solution for a shape and remember the
fastest.  ``tuning/gemm_gfx950.csv`` is that table, measured on MI355X for the shapes of the
bench configurations (ResNet-18/50/152 at per-GPU batch 512 / 256 / 128 / 64, DistilBERT):
ResNet-18 PowerSGD r=4 went 2.042 -> 1.980 ms/step at batch 512 and 1.121 -> 1.052 ms at
batch 64 (profiles/r2/gemm_tuning.md).

:func:`enable` turns TunableOp on with tuning OFF and loads the table: listed shapes use the
measured solution, every other shape the library default (exactly the untuned behaviour).
Nothing is timed at run time and nothing is written.  The table carries TunableOp's
validator lines (PyTorch / HIP / hipBLASLt / rocBLAS versions, gfx arch); on any mismatch
TunableOp rejects it and :func:`enable` switches TunableOp back off.

Environment:
  NDP_FUSION_OFF=tuned_gemms do not load the table (library defaults)
  PYTORCH_TUNABLEOP_ENABLED  set by the user: TunableOp is theirs, :func:`enable` does nothing
                             (how the table is (re)measured: tools/gpu_r2_tunable.sh)

Determinism: the selected solutions are plain (non-atomic) kernels; tests/test_gemm_tuning_gpu.py
checks bitwise repeatability and fp64 agreement of every tabled shape.
"""
from __future__ import annotations

import os
import warnings

import torch
from ..knobs import fusion_on

__all__ = ["TABLE", "enable", "disable", "enabled", "table_shapes"]

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "gemm_gfx950.csv")

_STATE = {"enabled": False}


def table_shapes(path: str = TABLE):
    """[(op, params)] of the solution lines of a TunableOp table (no validators)."""
    out = []
    with open(path) as f:
        for line in f:
            parts = line.strip().split(",")
            if len(parts) >= 3 and parts[0] != "Validator":
                out.append((parts[0], parts[1]))
    return out


def enabled() -> bool:
    return _STATE["enabled"]


def enable(path: str = TABLE) -> bool:
    """Load the measured solution table (idempotent).  Returns True when it is in use."""
    if _STATE["enabled"]:
        return True
    if not fusion_on("tuned_gemms") or "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return False
    if not torch.cuda.is_available() or torch.version.hip is None or not os.path.exists(path):
        return False
    tun = torch.cuda.tunable
    tun.tuning_enable(False)                   # never time solutions at run time
    tun.set_filename(path, insert_device_ordinal=False)
    tun.enable(True)
    ok = bool(tun.read_file(path)) and len(tun.get_results()) > 0
    if not ok:                                 # validator mismatch (other ROCm / torch / arch)
        tun.enable(False)
        warnings.warn(f"GEMM solution table {path} does not match this ROCm/PyTorch/GPU; "
                      "using library default GEMMs")
        return False
    _STATE["enabled"] = True
    return True


def disable() -> None:
    """Back to library-default GEMMs (tests / A-B runs)."""
    if _STATE["enabled"]:
        torch.cuda.tunable.enable(False)
        _STATE["enabled"] = False
