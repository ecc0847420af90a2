"""Measured GEMM solution table (ops/gemm_tuning.py): well-formed, loads on MI355X, and the
tuned solutions keep a ResNet-18 step bitwise repeatable and equal (to fp32 rounding) to the
library-default GEMMs."""
import pytest
import torch

from network_distributed_pytorch_amd.ops import gemm_tuning


def test_table_well_formed():
    lines = open(gemm_tuning.TABLE).read().splitlines()
    val = {l.split(",")[1]: l.split(",")[2] for l in lines if l.startswith("Validator")}
    assert val["GCN_ARCH_NAME"].startswith("gfx950")
    assert {"PT_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION"} <= set(val)
    shapes = gemm_tuning.table_shapes()
    assert len(shapes) >= 20 and len(set(shapes)) == len(shapes)
    assert all(op.startswith("Gemm") for op, _ in shapes)
    # the ResNet-18 Toeplitz GEMMs of the headline (batch 512) and N = 8 (batch 64) shapes
    params = {p for _, p in shapes}
    assert "tn_1024_512_1024_ld_1024_1024_1024" in params and "tn_1024_64_1024_ld_1024_1024_1024" in params


def test_enable_is_noop_without_gpu(monkeypatch):
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    assert gemm_tuning.enable() is False and not gemm_tuning.enabled()


def _step(model, x, y):
    model.zero_grad(set_to_none=True)
    torch.nn.functional.cross_entropy(model(x), y).backward()
    torch.cuda.synchronize()
    return [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.gpu
def test_tuned_gemms_deterministic_and_exact(device, monkeypatch):
    from network_distributed_pytorch_amd.models import build_resnet

    # the one MIOpen call left in ResNet-18 (strided 3x3 grad-x) may accumulate atomically
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)

    was = gemm_tuning.enabled()
    assert gemm_tuning.enable(), "the shipped table must load on the MI355X image"
    try:
        torch.manual_seed(0)
        model = build_resnet(18).to(device)
        x = torch.randn(64, 3, 32, 32, device=device)
        y = torch.randint(0, 10, (64,), device=device)
        a = _step(model, x, y)
        b = _step(model, x, y)
        for ga, gb in zip(a, b):
            assert torch.equal(ga, gb)  # tuned solutions: no atomics, bitwise repeatable
        gemm_tuning.disable()
        ref = _step(model, x, y)
        for ga, gr in zip(a, ref):
            scale = gr.abs().max().item() + 1e-12
            assert (ga - gr).abs().max().item() <= 1e-4 * scale
    finally:
        gemm_tuning.disable()
        if was:
            gemm_tuning.enable()


@pytest.mark.gpu
def test_tuned_gemms_deterministic_distilbert(device):
    """DistilBERT's tabled projection / FFN GEMM shapes (batch 16 x 512 tokens): bitwise
    repeatable fwd + bwd with the table on."""
    from network_distributed_pytorch_amd.models import build_model

    was = gemm_tuning.enabled()
    assert gemm_tuning.enable()
    try:
        torch.manual_seed(0)
        model = build_model("distilbert").to(device)
        ids = torch.randint(0, 30522, (16, 512), device=device)
        mask = torch.ones_like(ids)
        labels = torch.randint(0, 2, (16,), device=device)
        grads = []
        for _ in range(2):
            torch.manual_seed(1)  # same dropout masks
            model.zero_grad(set_to_none=True)
            model(ids, attention_mask=mask, labels=labels)[0].backward()
            torch.cuda.synchronize()
            grads.append([p.grad.detach().clone() for p in model.parameters() if p.grad is not None])
        assert len(grads[0]) > 50
        for a, b in zip(*grads):
            assert torch.equal(a, b)
    finally:
        gemm_tuning.disable()
        if was:
            gemm_tuning.enable()
