"""DistilBERT model-level fusions vs their unfused forms (same weights, dropout off):
packed QKV projection read in place by the attention kernels, and LayerNorm residual
gradients folded into the next GEMM (GradLink).  A GEMM with beta = 1 / a wider N may pick
another library solution, so gradients are compared with a tolerance relative to each
parameter's largest entry."""
import pytest
import torch

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.models import distilbert as dmod
from network_distributed_pytorch_amd.models.distilbert import distilbert_base

pytestmark = pytest.mark.gpu


def _grads(m, ids, am, lab):
    m.zero_grad(set_to_none=True)
    loss = m(ids, attention_mask=am, labels=lab)[0]
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("packed,links", [(True, True), (True, False), (False, True)])
def test_distilbert_fusions_match_unfused(device, monkeypatch, packed, links):
    assert ops.native_available()
    torch.manual_seed(0)
    m = distilbert_base(2, dropout=0.0, attention_dropout=0.0, seq_classif_dropout=0.0).to(device).train()
    B, S = 4, 256
    ids = torch.randint(0, 30522, (B, S), device=device)
    am = torch.ones(B, S, dtype=torch.long, device=device)
    am[1, 200:] = 0
    lab = torch.randint(0, 2, (B,), device=device)
    monkeypatch.setattr(dmod, "PACKED_QKV", packed)
    monkeypatch.setattr(dmod, "LN_LINKS", links)
    l1, g1 = _grads(m, ids, am, lab)
    monkeypatch.setattr(dmod, "PACKED_QKV", False)
    monkeypatch.setattr(dmod, "LN_LINKS", False)
    l0, g0 = _grads(m, ids, am, lab)
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-6)
    assert g1.keys() == g0.keys()
    for n in g0:
        if n.endswith("k_lin.bias"):
            # softmax is invariant to a per-query constant on the scores, so the key bias
            # gets an exactly-zero gradient: both runs hold rounding noise only
            ref = g0[n.replace("k_lin", "v_lin")].abs().max().item()
            assert g1[n].abs().max().item() < 1e-3 * ref and g0[n].abs().max().item() < 1e-3 * ref, n
            continue
        scale = g0[n].abs().max().item() + 1e-12
        torch.testing.assert_close(g1[n], g0[n], rtol=1e-3, atol=2e-4 * scale, msg=n)


def test_packed_qkv_in_place_in_powersgd_arena(device):
    """In the PowerSGD parameter arena q / k / v weights (and biases) are consecutive: the
    packed projection reads them in place (no concatenation copy) and leaves leaf-only
    ``.grad`` views (no per-pass torch.cat, no non-leaf .grad access)."""
    import warnings

    from network_distributed_pytorch_amd.ops.linear import _adjacent
    from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDOptimizer

    torch.manual_seed(0)
    m = distilbert_base(2, dropout=0.0, attention_dropout=0.0, seq_classif_dropout=0.0).to(device).train()
    ref = distilbert_base(2, dropout=0.0, attention_dropout=0.0, seq_classif_dropout=0.0).to(device).train()
    ref.load_state_dict(m.state_dict())
    PowerSGDOptimizer(m.parameters(), lr=1e-3, rank=4)  # re-points the parameters into its arena
    att = m.distilbert.transformer.layer[0].attention
    assert _adjacent((att.q_lin.weight, att.k_lin.weight, att.v_lin.weight)) is not None
    assert _adjacent((att.q_lin.bias, att.k_lin.bias, att.v_lin.bias)) is not None
    ids = torch.randint(0, 30522, (2, 128), device=device)
    am = torch.ones(2, 128, dtype=torch.long, device=device)
    lab = torch.randint(0, 2, (2,), device=device)
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # a non-leaf .grad access would warn
        l1, g1 = _grads(m, ids, am, lab)
    l0, g0 = _grads(ref, ids, am, lab)
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-6)
    for n in g0:
        if n.endswith("k_lin.bias"):
            continue
        scale = g0[n].abs().max().item() + 1e-12
        torch.testing.assert_close(g1[n], g0[n], rtol=1e-3, atol=2e-4 * scale, msg=n)
