"""HIP-kernel numerics vs an fp64 PyTorch oracle on one MI355X (gfx950).

Each kernel is checked against a plain PyTorch reference of the same op, over shapes that
hit every code path: float4 and scalar (m % 4 != 0) paths, r clamping (r = min(n, m, R)),
tall / wide matrices, 1..4 MFMA column groups (R up to 40), 4-D conv weights, empty
high-rank / rank-1 groups, split-K slabs.  Determinism (bitwise repeatability) is checked
for every stage, because replica consistency across ranks depends on it.
"""
import pytest
import torch

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.parallel.powersgd import (PowerSGDOptimizer, PowerSGDReducer,
                                                                orthogonalize)
from network_distributed_pytorch_amd.parallel.tensor_buffer import TensorBuffer

from .oracle import mgs, powersgd_round, reference_bits

pytestmark = pytest.mark.gpu


def _native_loaded():
    assert ops.native_available(), "native extension must be loaded on the GPU box"
    return ops.ext()


def test_extension_is_loaded(device):
    X = _native_loaded()
    assert X.SIZEOF_MATGEOM == 64 and X.SIZEOF_MATPTRS == 64


@pytest.mark.parametrize("n,r", [(64, 4), (1000, 4), (2048, 16), (7, 5), (30522, 8), (513, 33), (300, 64)])
def test_orth_matches_fp64_mgs(device, n, r):
    g = torch.Generator(device="cpu").manual_seed(n * 31 + r)
    P = torch.randn(n, r, generator=g)
    ref = mgs(P.double())
    out = orthogonalize(P.clone().to(device)).cpu().double()
    assert torch.allclose(out, ref, atol=2e-4, rtol=1e-3), (out - ref).abs().max()
    # orthonormal columns
    eye = out.t() @ out
    assert torch.allclose(eye, torch.eye(r, dtype=torch.float64), atol=1e-3)


SHAPE_SETS = [
    [(64, 3, 7, 7), (64,), (64,), (128, 64, 3, 3), (128,), (1000, 512), (1000,)],
    [(5, 7), (9, 1030), (3,), (300, 33), (17, 2, 3)],
    [(512, 4608), (512,)],
    [(30, 40), (64, 64)],       # no rank-1 tensors (quirk Q6 must not crash)
]


@pytest.mark.parametrize("shapes", SHAPE_SETS)
@pytest.mark.parametrize("R", [1, 4, 8, 16, 20, 40])
def test_reducer_native_matches_oracle(device, shapes, R):
    _native_loaded()
    torch.manual_seed(0)
    Ms = [torch.randn(s) for s in shapes]
    red = PowerSGDReducer(714, device, 0, True, rank=R)
    grad_in = [m.to(device) for m in Ms]
    grad_out = [torch.zeros_like(m) for m in grad_in]
    mems = [torch.zeros_like(m) for m in grad_in]
    # two calls: first (random Q), second (warm-started Q)
    for call in range(2):
        Qs = [red._buf.q_view(i).clone() for i in range(len(red._buf.shapes))] if red._buf else None
        bits = red.reduce(grad_in, grad_out, mems)
        if Qs is None:
            # first call: reconstruct the Q the reducer drew (private generator, deterministic)
            import numpy as np
            rng = np.random.RandomState(714)
            Qs = []
            for s in shapes:
                if len(s) <= 1:
                    continue
                n = s[0]
                m = int(torch.Size(s).numel()) // n
                gen = torch.Generator(device=device)
                gen.manual_seed(int(rng.randint(1_000_000_000)))
                Qs.append(torch.randn(m, min(n, m, R), generator=gen, device=device).cpu())
        outs, mm, newQ = powersgd_round([Ms], [q.cpu() for q in Qs], R)
        assert bits == reference_bits(shapes, R)
        for o, ref in zip(grad_out, outs):
            scale = ref.abs().max().item() + 1e-6
            assert torch.allclose(o.cpu().double(), ref, atol=2e-4 * scale, rtol=1e-3), (call, o.shape)
        for k, (m_, ref) in enumerate(zip(mems, mm[0])):
            if ref is None:
                assert torch.count_nonzero(m_) == 0  # rank-1 memories are never written
            else:
                scale = Ms[k].abs().max().item() + 1e-6  # residual is relative to M
                assert torch.allclose(m_.cpu().double(), ref, atol=2e-4 * scale, rtol=1e-3)
        # EF identity M = out + mem exactly as computed in fp32 (reducer.py:163)
        for m_in, o, m_ in zip(grad_in, grad_out, mems):
            if m_in.dim() > 1:
                assert torch.equal(m_, m_in - o)


def test_reducer_deterministic(device):
    _native_loaded()
    shapes = SHAPE_SETS[0]
    torch.manual_seed(1)
    Ms = [torch.randn(s, device=device) for s in shapes]
    res = []
    for _ in range(2):
        red = PowerSGDReducer(714, device, 0, True, rank=4)
        out = [torch.zeros_like(m) for m in Ms]
        mem = [torch.zeros_like(m) for m in Ms]
        red.reduce(Ms, out, mem)
        red.reduce(Ms, out, mem)
        res.append([o.clone() for o in out] + [red._buf.q_warm.clone()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _make_model(device):
    torch.manual_seed(3)
    m = torch.nn.Sequential(
        torch.nn.Conv2d(3, 16, 3, bias=False), torch.nn.BatchNorm2d(16), torch.nn.ReLU(),
        torch.nn.Conv2d(16, 8, 3), torch.nn.Flatten(), torch.nn.Linear(8 * 4 * 4, 10))
    return m.to(device)


@pytest.mark.parametrize("write_grad", [False, True])
def test_fused_optimizer_matches_torch_path(device, write_grad):
    _native_loaded()
    ma, mb = _make_model(device), _make_model(device)
    mb.load_state_dict(ma.state_dict())
    oa = PowerSGDOptimizer(ma.parameters(), lr=0.1, momentum=0.9, rank=4, write_grad=write_grad)
    ob = PowerSGDOptimizer(mb.parameters(), lr=0.1, momentum=0.9, rank=4, write_grad=write_grad, native=False)
    assert oa.native and not ob.native
    torch.manual_seed(5)
    for step in range(4):
        # batch 64 > rank: the per-matrix gradients are not rank-deficient, so MGS is
        # well conditioned and both paths must agree to fp32 rounding
        x = torch.randn(64, 3, 8, 8, device=device)
        y = torch.randint(0, 10, (64,), device=device)
        for m, o in ((ma, oa), (mb, ob)):
            o.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
        ba, bb = oa.step(), ob.step()
        assert ba == bb
        for pa, pb in zip(ma.parameters(), mb.parameters()):
            assert torch.allclose(pa, pb, atol=1e-5, rtol=1e-4), step
        assert torch.allclose(oa.e, ob.e, atol=1e-5, rtol=1e-3), (oa.e - ob.e).abs().max()
        assert torch.allclose(oa.m, ob.m, atol=1e-5, rtol=1e-3), (oa.m - ob.m).abs().max()
        if write_grad:
            for pa, pb in zip(ma.parameters(), mb.parameters()):
                assert torch.allclose(pa.grad, pb.grad, atol=1e-5, rtol=1e-4)


def test_tensor_buffer_native(device):
    _native_loaded()
    ts = [torch.randn(s, device=device) for s in [(3,), (5, 7), (1,), (130,), (2, 2, 2)]]
    tb = TensorBuffer(ts)
    assert tb.buffer.is_cuda and len(tb) == 5
    assert torch.equal(tb.buffer, torch.cat([t.reshape(-1) for t in ts]))
    for i, t in enumerate(ts):
        assert torch.equal(tb[i], t)
    tb.buffer.mul_(4.0)
    outs = [torch.empty_like(t) for t in ts]
    tb.unpack(outs, div=4.0)
    for o, t in zip(outs, ts):
        assert torch.equal(o, t)
    tb.unpack(outs)
    for o, t in zip(outs, ts):
        assert torch.equal(o, 4 * t)


def test_seg_reduce_chunks(device):
    _native_loaded()
    src = torch.randn(3 * 4100 + 7, device=device)
    dst = torch.empty(4100, device=device)
    plan = ops.SegPlan([(src, dst, 3, 4100, 2.0)], device)
    plan.run()
    ref = (src[:4100] + src[4100:8200] + src[8200:12300]) / 2.0
    assert torch.allclose(dst, ref, atol=1e-6)
    # unaligned (scalar path)
    dst2 = torch.empty(4099, device=device)
    ops.SegPlan([(src[1:], dst2, 1, 0, 1.0)], device).run()
    assert torch.equal(dst2, src[1:4100])


@pytest.mark.parametrize("n", [1, 4, 1023, 1 << 20])
def test_sgd_momentum_and_add(device, n):
    _native_loaded()
    x, g, b = (torch.randn(n, device=device) for _ in range(3))
    x2, g2, b2 = x.clone(), g.clone(), b.clone()
    ops.sgd_momentum_(x, g, b, 0.1, 0.9, 2.0)
    b2.mul_(0.9).add_(g2 / 2.0)
    x2.add_(b2, alpha=-0.1)
    assert torch.allclose(b, b2, atol=1e-6) and torch.allclose(x, x2, atol=1e-6)
    out = torch.empty_like(x)
    ops.add(x, g, out)
    assert torch.equal(out, x + g)


def test_checksum_and_delay(device):
    _native_loaded()
    x = torch.randn(1 << 20, device=device)
    assert abs(ops.checksum(x) - x.double().sum().item()) < 1e-6 * x.abs().sum().item()
    assert ops.checksum(x) == ops.checksum(x)
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ops.delay_ns(20_000_000)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert 0.015 < dt < 0.5, dt


def test_lazy_error_feedback_bitwise(device):
    """Lazy error feedback (the update pass skips e = M - P Q^T; the next P pass forms it with
    the same arithmetic) is bitwise the eager formula: parameters, momentum and the
    materialised error memory after every step, and the checkpoint state.  Gradients are
    set directly (a library conv's backward is not bitwise repeatable between two models)."""
    _native_loaded()
    ma, mb = _make_model(device), _make_model(device)
    mb.load_state_dict(ma.state_dict())
    oa = PowerSGDOptimizer(ma.parameters(), lr=0.1, momentum=0.9, rank=4)
    ob = PowerSGDOptimizer(mb.parameters(), lr=0.1, momentum=0.9, rank=4)
    assert oa.lazy_ef
    ob.lazy_ef = False
    assert torch.equal(oa.x, ob.x)
    gen = torch.Generator(device="cpu").manual_seed(6)
    for step in range(5):
        grads = [torch.randn(p.shape, generator=gen).to(device) for p in ma.parameters()]
        for m, o in ((ma, oa), (mb, ob)):
            o.zero_grad()
            for p, gr in zip(m.parameters(), grads):
                p.grad = gr.clone()
            o.step()
        assert torch.equal(oa.x, ob.x) and torch.equal(oa.m, ob.m), step
        if step % 2 == 1:  # materialising mid-run must not change the trajectory
            assert torch.equal(oa.e, ob.e), step
    sa, sb = oa.state_dict(), ob.state_dict()
    assert torch.equal(sa["error"], sb["error"]) and torch.equal(sa["q_warm"], sb["q_warm"])


@pytest.mark.parametrize("rank", [4, 8])
def test_fused_split_k_finish_bitwise(device, rank):
    """In-kernel split-K finish (P / Q last-arriver sums, rank-1 pack in the P launch, rank-1
    step in the update launch; csrc/powersgd.hip PFin / QFin / R1Step) == the separate seg_reduce
    / rank1_step launches, bitwise: same chunk order.  The model has matrices with several P
    chunks (m > 1024) and several Q chunks (n > 64), and <= 1-D parameters."""
    _native_loaded()
    torch.manual_seed(3)
    net = lambda: torch.nn.Sequential(torch.nn.Linear(2100, 300), torch.nn.LayerNorm(300),  # noqa: E731
                                      torch.nn.Linear(300, 130, bias=False), torch.nn.Linear(130, 9)).to(device)
    ma, mb = net(), net()
    mb.load_state_dict(ma.state_dict())
    oa = PowerSGDOptimizer(ma.parameters(), lr=0.1, momentum=0.9, rank=rank)
    ob = PowerSGDOptimizer(mb.parameters(), lr=0.1, momentum=0.9, rank=rank)
    assert oa.buf.fused
    ob.buf.fused = False
    assert max(oa.buf.p_chunks) > 1 and max(oa.buf.q_chunks) > 1
    gen = torch.Generator(device="cpu").manual_seed(9)
    for step in range(4):
        grads = [torch.randn(p.shape, generator=gen).to(device) for p in ma.parameters()]
        for m, o in ((ma, oa), (mb, ob)):
            o.zero_grad()
            for p, gr in zip(m.parameters(), grads):
                p.grad = gr.clone()
            o.step()
        assert torch.equal(oa.buf.comm_buf, ob.buf.comm_buf), step
        assert torch.equal(oa.buf.q_memory, ob.buf.q_memory), step
        assert torch.equal(oa.x, ob.x) and torch.equal(oa.m, ob.m), step
    # the reference-API reducer takes the same fused path
    from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDReducer
    ts = [torch.randn(s, device=device) for s in [(300, 2100), (300,), (130, 300), (9, 130), (9,)]]
    outs = []
    for fused in (True, False):
        red = PowerSGDReducer(714, device, rank=rank)
        go = [torch.zeros_like(t) for t in ts]
        mo = [torch.zeros_like(t) for t in ts]  # <= 1-D memories are never written (reducer.py)
        red.reduce(ts, go, mo)  # sizes the plan
        red._buf.fused = fused
        red._bind_key = None
        red.reduce(ts, go, mo)
        outs.append((go, mo))
    for a, b in zip(outs[0][0] + outs[0][1], outs[1][0] + outs[1][1]):
        assert torch.equal(a, b)
