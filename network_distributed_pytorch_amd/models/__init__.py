"""Model families: ResNet (torchvision keys), DistilBERT (HF keys), toy MLP."""
from .distilbert import DistilBertConfig, DistilBertForSequenceClassification, distilbert_base
from .mlp import ToyMLP
from .resnet import (BasicBlock, Bottleneck, ResNet, build_resnet, resnet18, resnet34, resnet50,
                     resnet101, resnet152)

__all__ = [
    "ResNet", "BasicBlock", "Bottleneck", "build_resnet", "resnet18", "resnet34", "resnet50",
    "resnet101", "resnet152", "DistilBertConfig", "DistilBertForSequenceClassification",
    "distilbert_base", "ToyMLP", "build_model",
]


def build_model(name: str, num_classes=None, fused_bn: bool = True, gemm_convs: bool = True,
                fused_attention: bool = True):
    """``num_classes`` defaults to the reference's heads: 1000 (ImageNet ResNet), 2 (IMDb)."""
    name = name.lower()
    if name.startswith("resnet"):
        return build_resnet(int(name[len("resnet"):]), 1000 if num_classes is None else num_classes,
                            fused_bn=fused_bn, gemm_convs=gemm_convs)
    if name in ("distilbert", "distilbert-base", "distilbert-base-uncased"):
        return distilbert_base(num_labels=2 if num_classes is None else num_classes,
                               fused_attention=fused_attention)
    if name in ("mlp", "toy_mlp"):
        return ToyMLP()
    raise ValueError(f"unknown model {name!r}")
