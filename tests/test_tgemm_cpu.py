"""The index algebra of the tgemm conv kernels (csrc/tgemm.hip), checked on CPU: the GEMM
descriptions the launchers build (``tg_describe``: composite operand strides, tap table,
M/N/K) are emulated with fp64 torch gathers and must reproduce conv2d forward, grad-x and
grad-W exactly.  The GPU tests (tests/test_tgconv_gpu.py) then only exercise the kernel."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd.ops import native_available

pytestmark = pytest.mark.skipif(not native_available(), reason="extension not built")

CASES = [
    (3, 8, 8, 8, 12, 1, 1, 0),    # pointwise, 8x8 map
    (2, 16, 4, 4, 8, 1, 1, 0),    # pointwise, 4x4
    (5, 12, 1, 1, 20, 1, 1, 0),   # pointwise, 1x1 map
    (2, 6, 2, 2, 4, 1, 1, 0),     # pointwise, 2x2
    (3, 5, 2, 2, 7, 3, 1, 1),     # small: 3x3 on 2x2
    (2, 4, 4, 4, 6, 3, 2, 1),     # small: 3x3/2, 4x4 -> 2x2
    (2, 4, 4, 4, 6, 1, 2, 0),     # small: 1x1/2, 4x4 -> 2x2
    (4, 6, 2, 2, 3, 3, 2, 1),     # small: 3x3/2, 2x2 -> 1x1
    (3, 7, 1, 1, 5, 3, 1, 1),     # small: 3x3 on 1x1 (center tap)
    (2, 3, 2, 2, 5, 1, 2, 0),     # small: 1x1/2, 2x2 -> 1x1
]


def _off(idx, i):
    so, si, sh = idx
    return (i >> sh) * so + (i & ((1 << sh) - 1)) * si


def _emulate(d, a_flat, b_flat, out_numel):
    M, N, K = d["M"], d["N"], d["K"]
    m, n, k = torch.arange(M), torch.arange(N), torch.arange(K)
    A = a_flat[_off(d["am"], m)[:, None] + _off(d["ak"], k)[None, :]]
    if d["gather"]:
        bk_sh, bn_sh = d["bk"][2], d["bn"][2]
        tab = torch.tensor(d["tab"])
        t = tab[((k & ((1 << bk_sh) - 1)) << bn_sh)[:, None] | (n & ((1 << bn_sh) - 1))[None, :]]
        idx = (k >> bk_sh)[:, None] * d["bk"][0] + (n >> bn_sh)[None, :] * d["bn"][0] + t.clamp(min=0)
        B = torch.where(t >= 0, b_flat[idx], torch.zeros((), dtype=b_flat.dtype))
    else:
        B = b_flat[_off(d["bk"], k)[:, None] + _off(d["bn"], n)[None, :]]
    C = A @ B
    out = torch.full((out_numel,), float("nan"), dtype=C.dtype)
    out[(_off(d["cm"], m)[:, None] + _off(d["cn"], n)[None, :]).reshape(-1)] = C.reshape(-1)
    return out, A, B


def _coalesced(d):
    """The load mapping walks the operand's unit-stride index across lanes."""
    step = lambda idx: _off(idx, torch.tensor(1)).item() - _off(idx, torch.tensor(0)).item()  # noqa: E731
    a_ok = step(d["ak"]) == 1 if d["akf"] else (step(d["am"]) == 1 or d["M"] == 1)
    if d["gather"]:
        return a_ok
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
    pw = k == 1 and s == 1 and p == 0
    d0 = ext().tg_describe(geom, B, 0)
    out, _, _ = _emulate(d0, w.reshape(-1) if pw else x.reshape(-1), x.reshape(-1) if pw else w.reshape(-1), y.numel())
    assert torch.allclose(out, y.reshape(-1), atol=1e-10), "forward"
    d1 = ext().tg_describe(geom, B, 1)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=s, padding=p)
    out, _, _ = _emulate(d1, w.reshape(-1) if pw else dy.reshape(-1), dy.reshape(-1) if pw else w.reshape(-1),
                         x.numel())
    assert torch.allclose(out, dx_ref.reshape(-1), atol=1e-10), "grad-x"
    d2 = ext().tg_describe(geom, B, 2)
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=s, padding=p)
    if pw:
        out, _, _ = _emulate(d2, dy.reshape(-1), x.reshape(-1), w.numel())
        assert torch.allclose(out, dw_ref.reshape(-1), atol=1e-10), "grad-W"
    else:  # dW_big^T [(co,o), (c,i)] = dY^T X, folded into dW by toeplitz_fold
        out, _, _ = _emulate(d2, dy.reshape(-1), x.reshape(-1), d2["M"] * d2["N"])
        want = dy.reshape(B, -1).t() @ x.reshape(B, -1)
        assert torch.allclose(out, want.reshape(-1), atol=1e-10), "grad-W_big"
    for d in (d0, d1, d2):
        assert _coalesced(d), d
        assert d["splits"] >= 1
