"""Direct fp32-MFMA convolutions (csrc/conv.hip) vs an fp64 CPU oracle (F.conv2d), every
direction of every class, including the 3x3 stride-2 grad-x on the zero-inserted dY."""
import pytest
import torch
import torch.nn.functional as F

# (cin, cout, k, stride, pad, hw, batch) — the ResNet CIFAR-shape classes
# small batches run split-K forward / grad-x (+ slab sum) and 1-image grad-W slices
CASES = [(64, 64, 3, 1, 1, 8, 8), (128, 128, 3, 1, 1, 4, 16), (64, 128, 3, 2, 1, 8, 8), (3, 64, 7, 2, 3, 32, 4),
         (128, 64, 3, 1, 1, 8, 4), (64, 192, 3, 1, 1, 4, 16), (64, 64, 3, 1, 1, 8, 64), (128, 128, 3, 1, 1, 4, 64),
         (64, 64, 3, 1, 1, 8, 6), (64, 128, 1, 2, 0, 8, 8), (64, 128, 1, 2, 0, 8, 64), (256, 512, 1, 2, 0, 8, 16),
         (64, 128, 3, 2, 1, 8, 64), (128, 128, 3, 2, 1, 8, 32), (64, 128, 3, 2, 1, 8, 512),
         (128, 256, 1, 2, 0, 4, 16), (128, 256, 1, 2, 0, 4, 64), (128, 256, 1, 2, 0, 4, 512),
         (512, 1024, 1, 2, 0, 4, 32), (3, 64, 7, 2, 3, 32, 64), (3, 64, 7, 2, 3, 32, 256)]


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,s,p,hw,B", CASES)
def test_direct_conv_vs_fp64(device, cin, cout, k, s, p, hw, B):
    from network_distributed_pytorch_amd.ops.conv import conv2d_direct, direct_plan

    torch.manual_seed(0)
    x = torch.randn(B, cin, hw, hw, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, dtype=torch.float64) / (cin * k * k) ** 0.5
    xd = x.float().to(device).requires_grad_(True)
    wd = w.float().to(device).requires_grad_(True)
    plan = direct_plan(xd, wd, s, p)
    assert plan is not None
    y = conv2d_direct(xd, wd, s, p)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=p)
    g = torch.randn_like(yr)
    yr.backward(g)
    y.backward(g.float().to(device))
    for got, ref, name in ((y, yr, "y"), (xd.grad, xr.grad, "dx"), (wd.grad, wr.grad, "dw")):
        got = got.detach().cpu().double()
        err = (got - ref).abs().max().item()
        scale = ref.abs().max().item()
        assert err <= 2e-6 * scale * (cin * k * k) ** 0.5 + 1e-6, (name, err, scale)


@pytest.mark.gpu
def test_stem_row_blocks_bitwise(device):
    """The stem forward split into 1 / 2 / 4 output-row blocks per image (conv.hip PSPLIT):
    every output pixel keeps its own k-ordered MFMA chain, so y is bitwise the same."""
    from network_distributed_pytorch_amd.ops._ext import ext

    torch.manual_seed(2)
    B = 32
    x = torch.randn(B, 3, 32, 32, device=device)
    w = torch.randn(64, 3, 7, 7, device=device) * 0.1
    geom = [3, 32, 32, 64, 7, 7, 2, 3]
    outs = []
    try:
        for ps in (1, 2, 4):
            ext().conv_set_stem_psplit(ps)
            y = torch.empty(B, 64, 16, 16, device=device)
            assert ext().conv_fwd(x, w, y, geom, None, False) == 1
            outs.append(y)
    finally:
        ext().conv_set_stem_psplit(0)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.gpu
def test_direct_conv_deterministic(device):
    from network_distributed_pytorch_amd.ops.conv import conv2d_direct

    torch.manual_seed(1)
    x = torch.randn(64, 64, 8, 8, device=device, requires_grad=True)  # split-K at batch 64
    w = torch.randn(64, 64, 3, 3, device=device, requires_grad=True)
    outs = []
    for _ in range(2):
        x.grad = w.grad = None
        y = conv2d_direct(x, w, 1, 1)
        y.backward(torch.ones_like(y))
        outs.append((y.detach().clone(), x.grad.clone(), w.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_direct_plan_rejects_other_shapes(device):
    from network_distributed_pytorch_amd.ops.conv import direct_plan

    x = torch.randn(8, 64, 16, 16, device=device)
    w = torch.randn(64, 64, 3, 3, device=device)
    assert direct_plan(x, w, 1, 1) is None
    x = torch.randn(6, 128, 4, 4, device=device)  # batch not a multiple of the 4-image fwd tile
    assert direct_plan(x, torch.randn(128, 128, 3, 3, device=device), 1, 1) is None


@pytest.mark.gpu
def test_direct_plan_adapts_to_batch(device):
    """Strong-scaling shapes: split-K + finer grad-W slices at small batch, none at 512."""
    from network_distributed_pytorch_amd.ops.conv import direct_plan

    w = torch.randn(128, 128, 3, 3, device=device)
    small = direct_plan(torch.randn(64, 128, 4, 4, device=device), w, 1, 1)
    big = direct_plan(torch.randn(512, 128, 4, 4, device=device), w, 1, 1)
    assert small[4] > 1 and small[5] > 1 and small[2] < big[2]
    assert big[4] == 1 and big[5] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,hw,B", [(64, 128, 8, 64), (64, 128, 8, 512), (128, 256, 4, 16), (128, 256, 4, 64),
                                           (128, 256, 4, 512)])
def test_strided_1x1_dgrad_addend(device, cin, cout, hw, B):
    """1x1 stride-2 grad-x with an addend (the downsample block's sibling grad-x): the even-pixel
    scatter epilogue / split-K sum writes dx + addend, odd pixels = addend, vs fp64."""
    from network_distributed_pytorch_amd.ops._ext import ext
    from network_distributed_pytorch_amd.ops.conv import direct_plan

    torch.manual_seed(5)
    x = torch.randn(B, cin, hw, hw, device=device)
    w = torch.randn(cout, cin, 1, 1, device=device) / cin ** 0.5
    plan = direct_plan(x, w, 2, 0)
    assert plan is not None
    geom, ksd = plan[0], plan[5]
    dy = torch.randn(B, cout, hw // 2, hw // 2, device=device)
    add = torch.randn_like(x)
    dx = torch.empty_like(x)
    part = torch.empty(ksd * dy.numel() // cout * cin, device=device) if ksd > 1 else None
    ext().conv_dgrad(dy, w, dx, list(geom), part, add, False)
    ref = F.conv_transpose2d(dy.double().cpu(), w.double().cpu(), stride=2, output_padding=1) + add.double().cpu()
    err = (dx.double().cpu() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,s,B,hw", [(64, 64, 1, 512, 8), (128, 64, 1, 512, 8), (64, 128, 2, 512, 8),
                                            (64, 64, 1, 1024, 8), (128, 128, 1, 512, 4), (128, 128, 1, 1024, 4),
                                            (256, 128, 1, 512, 4),
                                            # split-K (small per-GPU batches): slabs summed in order
                                            (64, 64, 1, 64, 8), (64, 64, 1, 128, 8), (64, 128, 2, 64, 8),
                                            (128, 128, 1, 64, 4), (128, 128, 1, 128, 4)])
def test_winograd_vs_direct_vs_fp64(device, cin, cout, s, B, hw):
    """Winograd F(2x2,3x3) (csrc/winograd.hip: layer1 / layer2 forward and grad-x, the stride-2 class's
    grad-x on the zero-inserted dY) against the direct MFMA kernels and an fp64 oracle: its error
    stays within a small factor of the direct kernels' and of the fp64 tolerance; bitwise
    run-to-run.  The Winograd path must actually be taken (conv_wino) for these shapes."""
    from network_distributed_pytorch_amd.ops.conv import wino_dirs
    from network_distributed_pytorch_amd.ops._ext import ext
    from network_distributed_pytorch_amd.ops.conv import conv2d_direct, set_winograd

    torch.manual_seed(6)
    x = torch.randn(B, cin, hw, hw, dtype=torch.float64)
    w = torch.randn(cout, cin, 3, 3, dtype=torch.float64) / (cin * 9) ** 0.5
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=1)
    g = torch.randn_like(yr)
    yr.backward(g)
    geom = (cin, hw, hw, cout, 3, 3, s, 1)
    set_winograd(True)
    assert bool(ext().conv_wino(list(geom), B, True)), "grad-x should take the Winograd kernel"
    assert s == 2 or bool(ext().conv_wino(list(geom), B, False)), "forward should take the Winograd kernel"
    res = {}
    try:
        for wino in (True, False, True):
            set_winograd(wino)
            xd = x.float().to(device).requires_grad_(True)
            wd = w.float().to(device).requires_grad_(True)
            y = conv2d_direct(xd, wd, s, 1)
            y.backward(g.float().to(device))
            out = (y.detach().cpu().double(), xd.grad.cpu().double(), wd.grad.cpu().double())
            if wino in res:
                for a, b in zip(res[wino], out):
                    assert torch.equal(a, b)  # deterministic
            res[wino] = out
    finally:
        set_winograd(True)
    for i, (ref, name) in enumerate(((yr, "y"), (xr.grad, "dx"), (wr.grad, "dw"))):
        scale = ref.abs().max().item()
        ew = (res[True][i] - ref).abs().max().item() / scale
        ed = (res[False][i] - ref).abs().max().item() / scale
        print(f"{name}: winograd rel err {ew:.2e}, direct {ed:.2e}")
        assert ew <= 4e-6 * (cin * 9) ** 0.5, (name, ew, ed)


@pytest.mark.gpu
def test_wino_bank_matches_per_layer_transforms(device):
    """ResNet-18 at batch 512 (Winograd layer1): the model's WinoBank (one transform launch per
    forward for every Winograd layer) == per-layer transforms, bitwise, across SGD steps."""
    from network_distributed_pytorch_amd.models import build_resnet
    from network_distributed_pytorch_amd.models.conv_gemm import GemmConv2d

    torch.manual_seed(7)
    a = build_resnet(18, 10).to(device)
    b = build_resnet(18, 10).to(device)
    b.load_state_dict(a.state_dict())
    for m in b.modules():
        if isinstance(m, GemmConv2d):
            m.wbank = None
    x = torch.randn(512, 3, 32, 32, device=device)
    y = torch.randint(0, 10, (512,), device=device)
    for _ in range(3):
        losses = []
        for m in (a, b):
            m.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(p.grad, alpha=-0.05)
            losses.append(loss.detach())
        assert torch.equal(losses[0], losses[1])
    assert len(a.layer1[0].conv1.wbank.members) >= 4
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)


@pytest.mark.gpu
def test_wino_bank_bottleneck_alternating_batches(device):
    """A Bottleneck ResNet whose set of Winograd layers changes with the batch size (ADVICE r5:
    at batch 20 the first Winograd layer is layer2.0.conv2, at batch 64 it is layer1's): the
    bank, alternating batches 64 and 20 (and first touched at 20 by a no-grad forward), stays
    bitwise equal to per-layer transforms across SGD steps."""
    from network_distributed_pytorch_amd.models import build_resnet
    from network_distributed_pytorch_amd.models.conv_gemm import GemmConv2d
    torch.manual_seed(8)
    a = build_resnet(50, 10).to(device)
    b = build_resnet(50, 10).to(device)
    b.load_state_dict(a.state_dict())
    for m in b.modules():
        if isinstance(m, GemmConv2d):
            m.wbank = None
    xs = {B: torch.randn(B, 3, 32, 32, device=device) for B in (64, 20)}
    ys = {B: torch.randint(0, 10, (B,), device=device) for B in (64, 20)}
    with torch.no_grad():  # first touch at the small batch
        for m in (a, b):
            m(xs[20])
    for B in (64, 20, 64, 20, 64):
        losses = []
        for m in (a, b):
            m.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(xs[B]), ys[B])
            loss.backward()
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(p.grad, alpha=-0.05)
            losses.append(loss.detach())
        assert torch.equal(losses[0], losses[1]), B
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)
    # the premise: a pass at each batch size is led by a different Winograd layer
    bank = next(m.wbank for m in a.modules() if isinstance(m, GemmConv2d) and m.wbank is not None)
    assert set(bank._lead) == {64, 20} and bank._lead[64] != bank._lead[20], bank._lead
