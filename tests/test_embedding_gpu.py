"""Native embedding backward (csrc/embedding.hip) vs an fp64 index_add oracle; determinism;
replay inside a hipGraph (PyTorch-ROCm's rocPRIM-sort backward faulted there)."""
import pytest
import torch

from network_distributed_pytorch_amd.ops.embedding import Embedding

pytestmark = pytest.mark.gpu


def _oracle(ids, g, V, pad):
    gw = torch.zeros(V, g.shape[-1], dtype=torch.float64)
    flat = ids.reshape(-1).cpu()
    keep = flat != pad if pad is not None else torch.ones_like(flat, dtype=torch.bool)
    gw.index_add_(0, flat[keep], g.reshape(-1, g.shape[-1]).double().cpu()[keep])
    return gw


@pytest.mark.parametrize("B,S,V,D,pad", [(16, 512, 30522, 768, 0), (3, 7, 11, 8, None), (2, 5000, 97, 16, 3)])
def test_embedding_backward_vs_fp64(device, B, S, V, D, pad):
    torch.manual_seed(0)
    emb = Embedding(V, D, padding_idx=pad).to(device)
    ids = torch.randint(0, V, (B, S), device=device)
    ids[:, :3] = 1 if V > 1 else 0            # duplicated ids
    if pad is not None:
        ids[:, -5:] = pad                      # padding rows get no gradient
    g = torch.randn(B, S, D, device=device)
    emb(ids).backward(g)
    ref = _oracle(ids, g, V, pad)
    err = (emb.weight.grad.double().cpu() - ref).abs().max().item()
    assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err
    if pad is not None:
        assert emb.weight.grad[pad].abs().max().item() == 0.0


def test_embedding_backward_deterministic(device):
    torch.manual_seed(1)
    emb = Embedding(1000, 64).to(device)
    ids = torch.randint(0, 50, (8, 512), device=device)  # heavy duplication
    g = torch.randn(8, 512, 64, device=device)
    outs = []
    for _ in range(3):
        emb.weight.grad = None
        emb(ids).backward(g)
        outs.append(emb.weight.grad.clone())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


def test_embedding_backward_graph_replay(device):
    """Captured forward+backward replayed with new ids every step == eager, 20 replays."""
    torch.manual_seed(2)
    V, D = 30522, 64
    emb = Embedding(V, D, padding_idx=0).to(device)
    gen = torch.Generator(device="cpu").manual_seed(3)
    batches = [torch.randint(0, V, (16, 512), generator=gen).to(device) for _ in range(4)]
    gs = [torch.randn(16, 512, D, generator=gen).to(device) for _ in range(4)]
    static_ids, static_g = batches[0].clone(), gs[0].clone()

    def fwd_bwd():
        emb.weight.grad = None
        emb(static_ids).backward(static_g)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fwd_bwd()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fwd_bwd()
    for i in range(20):
        static_ids.copy_(batches[i % 4])
        static_g.copy_(gs[i % 4])
        graph.replay()
        torch.cuda.synchronize()
        ref = _oracle(batches[i % 4], gs[i % 4], V, 0)
        err = (emb.weight.grad.double().cpu() - ref).abs().max().item()
        assert err <= 1e-5, (i, err)
