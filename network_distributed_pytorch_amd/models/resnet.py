"""ResNet-18/34/50/101/152 with torchvision-compatible ``state_dict`` keys and parameter order.

The reference uses ``torchvision.models.resnet50/152(pretrained=True)``
(ddp_guide_cifar10/ddp_init.py:108, ddp_powersgd_guide_cifar10/ddp_init.py:111), keeping the
ImageNet 1000-class head on CIFAR-10 (quirk Q13; ``num_classes`` makes it configurable).
torchvision is not installed and there is no network, so this is a self-contained
definition: same module names (``conv1``, ``bn1``, ``layer{1..4}.{i}.conv{1,2,3}``,
``downsample.{0,1}``, ``fc``), same registration order (so the PowerSGD P/Q layout and the
Q-init RNG order match the reference exactly), same init (Kaiming-normal fan_out convs,
BN = (1, 0)).  Weights are random (the GPU box has no network for pretrained downloads);
checkpoints written by torchvision load with ``load_state_dict`` unchanged.

MI355X notes: every conv is a :class:`~network_distributed_pytorch_amd.models.conv_gemm.GemmConv2d`
(native direct fp32-MFMA kernels for the stem / layer1 / layer2 CIFAR shapes, Toeplitz
GEMMs for layer3 / layer4, MIOpen elsewhere).  Every BatchNorm is a
:class:`~network_distributed_pytorch_amd.ops.batchnorm.BatchNormAct2d` (``fused_bn=True``):
BN, the residual add and the ReLU of each block run as two fused gfx950 kernels per
direction (same parameters/buffers/state_dict keys as ``nn.BatchNorm2d``).
``gemm_convs=False`` restores plain MIOpen everywhere.
"""
from __future__ import annotations

import os
from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from ..ops.batchnorm import BatchNormAct2d, bn_pair_act
from ..ops.conv import WinoBank, flush_forward, hold_forward
from ..ops.gradlink import BranchLink, GradLink
from ..ops.linear import Linear
from ..ops.pool import MaxPool2d
from ..ops.slablink import SlabLink
from .conv_gemm import GemmConv2d, ToeplitzBank
from ..knobs import fusion_on

__all__ = ["ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet34", "resnet50", "resnet101",
           "resnet152", "build_resnet"]

# split-K slab hand-off between direct convs and fused BN (ops/slablink.py; NDP_FUSION_OFF=slab_links
# or tests flip it for A/B)
SLAB_LINKS = fusion_on("slab_links")
# downsample blocks: conv1 / downsample grad-x accumulated in place (ops/gradlink.BranchLink)
BRANCH_LINKS = fusion_on("branch_links")


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    # GemmConv2d == nn.Conv2d (same params / state_dict); small feature maps run as GEMMs
    return GemmConv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return GemmConv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 norm=nn.BatchNorm2d):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = norm(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = norm(planes)
        self.downsample = downsample
        self.stride = stride
        self.fused = norm is BatchNormAct2d

    def forward(self, x, grad_in=None, grad_out=None):
        """``grad_in`` / ``grad_out`` (ops/slablink.SlabLink, fused training only): conv1's
        split-K grad-x slabs (+ the residual addend) go to the PREVIOUS block's BN2, whose
        output gradient they are, and this block's BN2 takes the next block's (ResNet.forward
        chains them): one sum launch fewer per block boundary."""
        if self.fused:  # conv -> BN+ReLU ; conv -> BN + identity + ReLU (fused kernels)
            train = x.is_cuda and torch.is_grad_enabled() and self.training
            if not (train and SLAB_LINKS):
                grad_in = grad_out = None
            # identity block: BN2's residual gradient is folded into conv1's grad-x
            # (ops/gradlink.py) instead of an autograd add of the two branches
            link = GradLink() if self.downsample is None and train and x.requires_grad else None
            # split-K conv slabs summed inside the neighbouring BN kernels (ops/slablink.py):
            # conv1 -> bn1, conv2 -> bn2, downsample conv -> its BN (forward), and conv2's
            # grad-x -> the gradient bn1's backward reads
            s1, s2, g1, sd = ((SlabLink(), SlabLink(), SlabLink(), SlabLink()) if train and SLAB_LINKS
                              else (None,) * 4)
            identity = x
            # downsample block: conv1 and the 1x1 downsample share one grad-x buffer (Toeplitz
            # layers; ops/gradlink.BranchLink) instead of an autograd add of the two
            br = (BranchLink() if BRANCH_LINKS and train and self.downsample is not None and x.requires_grad
                  else None)
            if self.downsample is not None and br is None:
                # x's gradient is autograd's sum of two grad-x tensors: conv1's cannot be left
                # as unsummed slabs for the previous BN2
                grad_in = None
            cds = None  # the downsample conv's output, its BN paired with bn2 (bn_pair_act)
            held = False
            if self.downsample is not None:
                ds = self.downsample
                if train and len(ds) == 2 and isinstance(ds[0], GemmConv2d) and isinstance(ds[1], BatchNormAct2d):
                    # its forward may wait for conv1's and share the launch (ops/conv.hold_forward)
                    held = x.is_cuda
                    with hold_forward(held):
                        cds = ds[0](x, slab_out=sd, branch=br)
                else:
                    identity = ds(x)
            c1 = self.conv1(x, link=link, slab_out=s1, grad_slab=grad_in, branch=br)
            if held:
                flush_forward()  # the downsample forward, if conv1 did not take it
            out = self.bn1(c1, relu=True, slab_in=s1, grad_slab=g1)
            c2 = self.conv2(out, slab_out=s2, grad_slab=g1)
            if cds is not None:
                y = bn_pair_act(self.bn2, self.downsample[1], c2, cds, slab_in=s2, slab_in2=sd, grad_slab=grad_out)
                if y is not None:
                    return y
                identity = self.downsample[1](cds, slab_in=sd)
            return self.bn2(c2, residual=identity, relu=True, link=link, slab_in=s2, grad_slab=grad_out)
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 norm=nn.BatchNorm2d):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = norm(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = norm(planes)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = norm(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.fused = norm is BatchNormAct2d

    def forward(self, x):
        if self.fused:  # the BasicBlock plumbing, one conv / BN pair more
            train = x.is_cuda and torch.is_grad_enabled() and self.training
            # identity block: BN3's residual gradient is folded into conv1's grad-x (the tgemm
            # pointwise epilogue / split-K sum) instead of an autograd add of the two branches
            link = GradLink() if self.downsample is None and train and x.requires_grad else None
            # split-K conv slabs summed inside the neighbouring BN kernels: conv1 -> bn1,
            # conv2 -> bn2, conv3 -> bn3, downsample conv -> its BN (forward); conv2's grad-x ->
            # bn1's backward, conv3's grad-x -> bn2's backward
            s1, s2, s3, g1, g2, sd = (tuple(SlabLink() for _ in range(6)) if train and SLAB_LINKS
                                      else (None,) * 6)
            identity = x
            if self.downsample is not None:
                ds = self.downsample
                if train and len(ds) == 2 and isinstance(ds[0], GemmConv2d) and isinstance(ds[1], BatchNormAct2d):
                    identity = ds[1](ds[0](x, slab_out=sd), slab_in=sd)
                else:
                    identity = ds(x)
            out = self.bn1(self.conv1(x, link=link, slab_out=s1), relu=True, slab_in=s1, grad_slab=g1)
            out = self.bn2(self.conv2(out, slab_out=s2, grad_slab=g1), relu=True, slab_in=s2, grad_slab=g2)
            return self.bn3(self.conv3(out, slab_out=s3, grad_slab=g2), residual=identity, relu=True, link=link,
                            slab_in=s3)
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 fused_bn: bool = True, gemm_convs: bool = True):
        super().__init__()
        self.norm = BatchNormAct2d if fused_bn else nn.BatchNorm2d
        self.fused = fused_bn
        self.inplanes = 64
        self.conv1 = GemmConv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = self.norm(64)
        self.relu = nn.ReLU(inplace=True)
        # native deterministic pool when fused kernels are on (no params: state_dict unchanged)
        self.maxpool = (MaxPool2d if fused_bn else nn.MaxPool2d)(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        # native deterministic bias gradient (ops/linear.py; ATen's multi-block reduce was
        # found unreliable under hipGraph replay), same parameters / state_dict as nn.Linear
        self.fc = (Linear if fused_bn else nn.Linear)(512 * block.expansion, num_classes)
        bank = ToeplitzBank()  # every Toeplitz layer's W_big in one launch per forward
        wbank = WinoBank()     # every Winograd layer's weight transforms in one launch per forward
        for m in self.modules():
            if isinstance(m, GemmConv2d):
                m.gemm = gemm_convs
                m.direct = gemm_convs
                m.bank = bank
                m.wbank = wbank
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # includes BatchNormAct2d
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    @staticmethod
    def _chain(blocks, x):
        """Run consecutive BasicBlocks with a SlabLink at each boundary: block i+1's conv1 grad-x
        slabs are summed by block i's BN2 backward (ops/slablink.py)."""
        prev = None
        for i, blk in enumerate(blocks):
            nxt = SlabLink() if i + 1 < len(blocks) else None
            x = blk(x, grad_in=prev, grad_out=nxt)
            prev = nxt
        return x

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       self.norm(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, norm=self.norm)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, norm=self.norm))
        return nn.Sequential(*layers)

    def forward(self, x):
        if self.fused:  # the stem conv's epilogue hands its BN the statistics (ops/slablink.py)
            s0 = SlabLink() if (SLAB_LINKS and x.is_cuda and torch.is_grad_enabled() and self.training) else None
            x = self.conv1(x, slab_out=s0)
            # BN -> ReLU -> max-pool in one pass, the BN output never stored (ops/batchnorm.py)
            pooled = self.bn1.relu_maxpool(x, self.maxpool, slab_in=s0)
            x = pooled if pooled is not None else self.maxpool(self.bn1(x, relu=True, slab_in=s0))
        else:
            x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        # the chained path calls the blocks directly: not when hooks sit on the layer modules
        # (they would not fire)
        train_links = (self.fused and SLAB_LINKS and self.training and x.is_cuda and torch.is_grad_enabled()
                       and all(isinstance(b, BasicBlock) for b in self.layer1)
                       and not any(m._forward_hooks or m._forward_pre_hooks
                                   for m in (self.layer1, self.layer2, self.layer3, self.layer4)))
        if train_links:  # block-boundary grad-x slab links (BasicBlock grad_in / grad_out)
            x = self._chain(list(self.layer1) + list(self.layer2), x)
            x = self._chain(list(self.layer3) + list(self.layer4), x)
        else:
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        # 1x1 feature map (32x32 inputs): the average is the value itself; flatten skips a
        # mean kernel forward and its broadcast-divide backward (bitwise identical)
        x = torch.flatten(x if x.shape[-2:] == (1, 1) else self.avgpool(x), 1)
        return self.fc(x)


_CFG = {
    18: (BasicBlock, [2, 2, 2, 2]),
    34: (BasicBlock, [3, 4, 6, 3]),
    50: (Bottleneck, [3, 4, 6, 3]),
    101: (Bottleneck, [3, 4, 23, 3]),
    152: (Bottleneck, [3, 8, 36, 3]),
}


def build_resnet(depth: int, num_classes: int = 1000, fused_bn: bool = True, gemm_convs: bool = True) -> ResNet:
    if depth not in _CFG:
        raise ValueError(f"unsupported ResNet depth {depth}; choose from {sorted(_CFG)}")
    block, layers = _CFG[depth]
    return ResNet(block, layers, num_classes=num_classes, fused_bn=fused_bn, gemm_convs=gemm_convs)


def resnet18(num_classes: int = 1000, **_) -> ResNet:
    return build_resnet(18, num_classes)


def resnet34(num_classes: int = 1000, **_) -> ResNet:
    return build_resnet(34, num_classes)


def resnet50(num_classes: int = 1000, **_) -> ResNet:
    return build_resnet(50, num_classes)


def resnet101(num_classes: int = 1000, **_) -> ResNet:
    return build_resnet(101, num_classes)


def resnet152(num_classes: int = 1000, **_) -> ResNet:
    return build_resnet(152, num_classes)
