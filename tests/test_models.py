"""Model definitions: torchvision / HF key compatibility and parameter counts."""
import pytest
import torch

from network_distributed_pytorch_amd.models import build_model, distilbert_base, resnet18


@pytest.mark.parametrize("depth,params,tensors", [(18, 11689512, 62), (50, 25557032, 161), (152, 60192808, 467)])
def test_resnet_param_counts(depth, params, tensors):
    m = build_model(f"resnet{depth}", 1000)
    ps = list(m.parameters())
    assert sum(p.numel() for p in ps) == params
    assert len(ps) == tensors


def test_resnet_torchvision_keys():
    sd = resnet18().state_dict()
    for k in ["conv1.weight", "bn1.running_mean", "bn1.num_batches_tracked", "layer1.0.conv1.weight",
              "layer2.0.downsample.0.weight", "layer2.0.downsample.1.running_var", "layer4.1.bn2.bias",
              "fc.weight", "fc.bias"]:
        assert k in sd
    assert sd["fc.weight"].shape == (1000, 512)
    assert build_model("resnet50").state_dict()["layer1.0.conv3.weight"].shape == (256, 64, 1, 1)


def test_resnet_forward_cifar_shape():
    m = resnet18(num_classes=10)
    assert m(torch.randn(2, 3, 32, 32)).shape == (2, 10)


def test_distilbert_counts():
    m = distilbert_base()
    ps = list(m.named_parameters())
    assert len(ps) == 104
    assert sum(p.numel() for _, p in ps) == 66955010
    assert ps[0][0] == "distilbert.embeddings.word_embeddings.weight"
    assert ps[-1][0] == "classifier.bias"


def test_distilbert_matches_hf_transformers():
    transformers = pytest.importorskip("transformers")
    cfg = transformers.DistilBertConfig(n_layers=2, dim=64, hidden_dim=128, n_heads=4, vocab_size=500,
                                        max_position_embeddings=64)
    hf = transformers.DistilBertForSequenceClassification(cfg).eval()
    from network_distributed_pytorch_amd.models.distilbert import DistilBertConfig, DistilBertForSequenceClassification
    ours = DistilBertForSequenceClassification(DistilBertConfig(n_layers=2, dim=64, hidden_dim=128, n_heads=4,
                                                                vocab_size=500, max_position_embeddings=64)).eval()
    hf_names = [n for n, _ in hf.named_parameters()]
    our_names = [n for n, _ in ours.named_parameters()]
    assert hf_names == our_names  # same names AND registration order (P/Q layout, Q-init order)
    ours.load_state_dict(hf.state_dict(), strict=False)
    ids = torch.randint(1, 500, (3, 20))
    mask = torch.ones_like(ids)
    mask[1, 12:] = 0
    labels = torch.tensor([0, 1, 1])
    with torch.no_grad():
        a = hf(input_ids=ids, attention_mask=mask, labels=labels)
        b = ours(ids, attention_mask=mask, labels=labels)
    assert torch.allclose(a.logits, b.logits, atol=1e-5)
    assert torch.allclose(a.loss, b[0], atol=1e-6)
