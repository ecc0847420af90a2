"""The index algebra of the tgemm conv kernels (csrc/tgemm.hip), checked on CPU: the GEMM
descriptions the launchers build (``tg_describe``: composite operand strides, M/N/K) are emulated with fp64 torch gathers and must reproduce conv2d forward, grad-x and
grad-W exactly.  The GPU tests (tests/test_tgconv_gpu.py) then only exercise the kernel."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd.ops import native_available

pytestmark = pytest.mark.skipif(not native_available(), reason="extension not built")

CASES = [
    (3, 8, 8, 8, 12, 1, 1, 0),    # pointwise, 8x8 map
    (2, 16, 4, 4, 8, 1, 1, 0),    # pointwise, 4x4
    (2, 6, 2, 2, 4, 1, 1, 0),     # pointwise, 2x2
    (3, 7, 16, 16, 5, 1, 1, 0),   # pointwise, 16x16
]


def _off(idx, i):
    so, si, sh = idx
    return (i >> sh) * so + (i & ((1 << sh) - 1)) * si


def _emulate(d, a_flat, b_flat, out_numel):
    M, N, K = d["M"], d["N"], d["K"]
    m, n, k = torch.arange(M), torch.arange(N), torch.arange(K)
    A = a_flat[_off(d["am"], m)[:, None] + _off(d["ak"], k)[None, :]]
    B = b_flat[_off(d["bk"], k)[:, None] + _off(d["bn"], n)[None, :]]
    C = A @ B
    out = torch.full((out_numel,), float("nan"), dtype=C.dtype)
    out[(_off(d["cm"], m)[:, None] + _off(d["cn"], n)[None, :]).reshape(-1)] = C.reshape(-1)
    return out, A, B


def _coalesced(d):
    """The load mapping walks the operand's unit-stride index across lanes."""
    step = lambda idx: _off(idx, torch.tensor(1)).item() - _off(idx, torch.tensor(0)).item()  # noqa: E731
    a_ok = step(d["ak"]) == 1 if d["akf"] else (step(d["am"]) == 1 or d["M"] == 1)
    b_ok = step(d["bn"]) == 1 if d["bnf"] else step(d["bk"]) == 1
    return a_ok and b_ok


@pytest.mark.parametrize("case", CASES)
def test_tgemm_index_algebra(case):
    from network_distributed_pytorch_amd.ops import ext

    B, C, H, W, Co, k, s, p = case
    geom = [C, H, W, Co, k, k, s, p]
    torch.manual_seed(0)
    x = torch.randn(B, C, H, W, dtype=torch.float64)
    w = torch.randn(Co, C, k, k, dtype=torch.float64)
    y = F.conv2d(x, w, stride=s, padding=p)
    dy = torch.randn_like(y)
    d0 = ext().tg_describe(geom, B, 0)
    out, _, _ = _emulate(d0, w.reshape(-1), x.reshape(-1), y.numel())
    assert torch.allclose(out, y.reshape(-1), atol=1e-10), "forward"
    d1 = ext().tg_describe(geom, B, 1)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=s, padding=p)
    out, _, _ = _emulate(d1, w.reshape(-1), dy.reshape(-1), x.numel())
    assert torch.allclose(out, dx_ref.reshape(-1), atol=1e-10), "grad-x"
    d2 = ext().tg_describe(geom, B, 2)
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=s, padding=p)
    out, _, _ = _emulate(d2, dy.reshape(-1), x.reshape(-1), w.numel())
    assert torch.allclose(out, dw_ref.reshape(-1), atol=1e-10), "grad-W"
    for d in (d0, d1, d2):
        assert _coalesced(d), d
        assert d["splits"] >= 1


def test_tgemm_small_maps_not_covered():
    """The small-map tabled family was deleted (round 6): 3x3 / strided convs and 1x1 maps have
    no tgemm path (they run on the direct / Toeplitz paths)."""
    from network_distributed_pytorch_amd.ops import ext

    for geom in ([256, 2, 2, 256, 3, 3, 1, 1], [128, 4, 4, 256, 1, 1, 2, 0], [512, 1, 1, 2048, 1, 1, 1, 0]):
        assert ext().tg_plan(geom, 64)[0] == -1, geom
