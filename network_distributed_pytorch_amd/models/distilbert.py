"""DistilBERT-base for sequence classification, HF-``state_dict``-compatible.

The reference fine-tunes ``DistilBertForSequenceClassification.from_pretrained(
'distilbert-base-uncased')`` on IMDb (ddp_powersgd_distillBERT_IMDb/ddp_init.py:150-152).
There is no network, so weights are random-init (HF init: N(0, 0.02) linear/embedding,
zero bias, LayerNorm (1, 0)).  Parameter names and registration order equal HF's
(``distilbert.embeddings.word_embeddings.weight`` ... ``classifier.bias``: 104 tensors,
66,955,010 parameters for the default config), so the PowerSGD P/Q layout, the byte
count per step and checkpoints interchange with ``transformers``.

On the GPU (fp32, head dim 64) attention runs the fused flash-style HIP kernels of
``ops/attention.py`` (csrc/attention.hip): the [B, H, S, S] score / probability tensors
never reach HBM.  ``fused_attention=False`` (or CPU / autocast) runs the explicit
QK^T -> mask -> softmax -> dropout -> PV math.  No Triton/AOTriton path is used.
"""
from __future__ import annotations

import dataclasses
import math
import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.attention import attention, attention_qkv, fused_ok
from ..ops.embedding import Embedding
from ..ops.gradlink import GradLink
from ..ops.layernorm import AddLayerNorm
from ..ops.linear import Linear, linear_gelu, packed_qkv
from ..ops.loss import cross_entropy as native_ce
from ..knobs import fusion_on

__all__ = ["DistilBertConfig", "DistilBertForSequenceClassification", "distilbert_base"]

# one packed QKV projection read in place by the attention kernels (NDP_FUSION_OFF=packed_qkv: three)
PACKED_QKV = fusion_on("packed_qkv")
# LayerNorm residual gradients folded into the next GEMM (NDP_FUSION_OFF=ln_links: autograd adds)
LN_LINKS = fusion_on("ln_links")


@dataclasses.dataclass
class DistilBertConfig:
    vocab_size: int = 30522
    max_position_embeddings: int = 512
    dim: int = 768
    n_layers: int = 6
    n_heads: int = 12
    hidden_dim: int = 3072
    dropout: float = 0.1
    attention_dropout: float = 0.1
    seq_classif_dropout: float = 0.2
    num_labels: int = 2
    pad_token_id: int = 0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    fused_attention: bool = True   # not an HF field: selects csrc/attention.hip on the GPU


class Embeddings(nn.Module):
    def __init__(self, c: DistilBertConfig):
        super().__init__()
        # native deterministic backward (graph-replayable; ops/embedding.py)
        self.word_embeddings = Embedding(c.vocab_size, c.dim, padding_idx=c.pad_token_id)
        self.position_embeddings = Embedding(c.max_position_embeddings, c.dim)
        self.LayerNorm = AddLayerNorm(c.dim, eps=c.layer_norm_eps)
        self.LayerNorm.native = c.fused_attention  # native kernels on/off together
        self.dropout = nn.Dropout(c.dropout)
        self._pos = {}

    def _pos_ids(self, b: int, s: int, device) -> torch.Tensor:
        # [B, S] position ids, built once per shape (no arange launch per pass)
        key = (b, s, str(device))
        if key not in self._pos:
            self._pos[key] = torch.arange(s, device=device).expand(b, s).contiguous()
        return self._pos[key]

    def forward(self, input_ids, seed=None):
        b, s = input_ids.shape
        if input_ids.is_cuda and self.LayerNorm.native:
            # per-token position rows: the native embedding backward sums them over the batch
            # (no broadcast-add + ATen reduce); the word + position add rides in the fused LN
            pos = self.position_embeddings(self._pos_ids(b, s, input_ids.device))
            # the dropout rides in the LayerNorm kernels (hash mask regenerated in backward)
            return self.LayerNorm(self.word_embeddings(input_ids), residual=pos,
                                  p_out=self.dropout.p if self.training else 0.0, seed=seed)
        pos = torch.arange(s, device=input_ids.device)
        x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None]
        return self.dropout(self.LayerNorm(x))


class MultiHeadSelfAttention(nn.Module):
    def __init__(self, c: DistilBertConfig):
        super().__init__()
        self.n_heads = c.n_heads
        self.dim = c.dim
        self.q_lin = Linear(c.dim, c.dim)
        self.k_lin = Linear(c.dim, c.dim)
        self.v_lin = Linear(c.dim, c.dim)
        self.out_lin = Linear(c.dim, c.dim)
        self.dropout = nn.Dropout(c.attention_dropout)
        self.fused = c.fused_attention

    def forward(self, x, mask: Optional[torch.Tensor], link=None, seed=None):
        """``link`` (ops/gradlink.GradLink): the block's residual gradient, folded into the
        first projection's grad-x GEMM.  ``seed``: the fused kernels' dropout seed (device
        int32; None draws one)."""
        bs, s, d = x.shape
        h = self.n_heads
        dh = d // h
        if self.fused and PACKED_QKV and x.is_cuda and x.dtype == torch.float32 and dh == 64:
            # one packed projection GEMM [B*S, 3D] over the three weights in place (consecutive
            # in the PowerSGD arena: no copy; ops/linear.packed_qkv), read in place by the
            # fused attention kernels (ops/attention.attention_qkv)
            qkv = packed_qkv(x, self.q_lin, self.k_lin, self.v_lin, link)
            ctx = attention_qkv(qkv, h, mask, self.dropout.p if self.training else 0.0, seed=seed)
            return self.out_lin(ctx.reshape(bs, s, d))
        q4 = self.q_lin(x, link=link).view(bs, s, h, dh)
        if self.fused and fused_ok(q4):
            ctx = attention(q4, self.k_lin(x).view(bs, s, h, dh), self.v_lin(x).view(bs, s, h, dh), mask,
                            self.dropout.p if self.training else 0.0, seed=seed)
            return self.out_lin(ctx.reshape(bs, s, d))

        def split(t):
            return t.view(bs, s, h, dh).transpose(1, 2)

        q = q4.transpose(1, 2) / math.sqrt(dh)
        k = split(self.k_lin(x))
        v = split(self.v_lin(x))
        scores = torch.matmul(q, k.transpose(-1, -2))
        if mask is not None:
            scores = scores.masked_fill((mask == 0).view(bs, 1, 1, s), torch.finfo(scores.dtype).min)
        w = self.dropout(F.softmax(scores, dim=-1))
        ctx = torch.matmul(w, v).transpose(1, 2).reshape(bs, s, d)
        return self.out_lin(ctx)


class FFN(nn.Module):
    def __init__(self, c: DistilBertConfig):
        super().__init__()
        self.lin1 = Linear(c.dim, c.hidden_dim)
        self.lin2 = Linear(c.hidden_dim, c.dim)
        self.dropout = nn.Dropout(c.dropout)

    def forward(self, x, link=None, dropout: bool = True):
        """``dropout=False``: the caller applies this dropout (fused into the block's
        LayerNorm)."""
        # lin1 + exact GELU share one fused native backward pass (ops/linear.linear_gelu)
        h = self.lin2(linear_gelu(x, self.lin1.weight, self.lin1.bias, link))
        return self.dropout(h) if dropout else h


class TransformerBlock(nn.Module):
    def __init__(self, c: DistilBertConfig):
        super().__init__()
        self.attention = MultiHeadSelfAttention(c)
        # residual add + LayerNorm fused into one gfx950 kernel per direction (ops/layernorm.py)
        self.sa_layer_norm = AddLayerNorm(c.dim, eps=c.layer_norm_eps)
        self.ffn = FFN(c)
        self.output_layer_norm = AddLayerNorm(c.dim, eps=c.layer_norm_eps)
        self.sa_layer_norm.native = self.output_layer_norm.native = c.fused_attention

    def forward(self, x, mask, seeds=None):
        """``seeds``: [2] device int32 dropout seeds (attention, FFN) or None (drawn per call)."""
        s0, s1 = (seeds[0:1], seeds[1:2]) if seeds is not None else (None, None)
        # residual gradients: deposited by the fused LayerNorm backward, added in place by the
        # sublayer's first GEMM (ops/gradlink.GradLink) instead of an autograd add
        lk = self._link(self.sa_layer_norm, x)
        x = self.sa_layer_norm(self.attention(x, mask, link=lk, seed=s0), residual=x, link=lk)
        lk = self._link(self.output_layer_norm, x)
        # the FFN's output dropout rides in the LayerNorm kernels (hash mask, no mask tensor)
        return self.output_layer_norm(self.ffn(x, link=lk, dropout=False), residual=x, link=lk,
                                      p_in=self.ffn.dropout.p if self.training else 0.0, seed=s1)

    def _link(self, ln, x):
        if LN_LINKS and self.training and torch.is_grad_enabled() and x.requires_grad and ln.fused_ok(x, x):
            return GradLink()
        return None


class Transformer(nn.Module):
    def __init__(self, c: DistilBertConfig):
        super().__init__()
        self.layer = nn.ModuleList([TransformerBlock(c) for _ in range(c.n_layers)])

    def forward(self, x, mask, seeds=None):
        if mask is not None and x.is_cuda:
            mask = mask.to(torch.int32).contiguous()   # once per pass, not per layer
        for i, blk in enumerate(self.layer):
            x = blk(x, mask, seeds[2 * i: 2 * i + 2] if seeds is not None else None)
        return x


class DistilBertModel(nn.Module):
    def __init__(self, c: DistilBertConfig):
        super().__init__()
        self.embeddings = Embeddings(c)
        self.transformer = Transformer(c)

    def forward(self, input_ids, attention_mask=None):
        seeds = None
        if self.training and input_ids.is_cuda and self.embeddings.LayerNorm.native:
            # every fused dropout site's seed in ONE draw (13 for 6 layers) instead of one
            # generator launch per site
            n = 2 * len(self.transformer.layer) + 1
            seeds = torch.randint(0, 2 ** 31 - 1, (n,), device=input_ids.device, dtype=torch.int32)
        x = self.embeddings(input_ids, seeds[-1:] if seeds is not None else None)
        return self.transformer(x, attention_mask, seeds)


class SequenceClassifierOutput(tuple):
    """``outputs[0]`` is the loss when labels are given (ddp_init.py:189-191 indexing)."""

    @property
    def loss(self):
        return self[0] if len(self) == 2 else None

    @property
    def logits(self):
        return self[-1]


class DistilBertForSequenceClassification(nn.Module):
    def __init__(self, config: Optional[DistilBertConfig] = None):
        super().__init__()
        c = config or DistilBertConfig()
        self.config = c
        self.distilbert = DistilBertModel(c)
        self.pre_classifier = Linear(c.dim, c.dim)
        self.classifier = Linear(c.dim, c.num_labels)
        self.dropout = nn.Dropout(c.seq_classif_dropout)
        self.apply(self._init)

    def _init(self, m):
        std = self.config.initializer_range
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, std)
            if m.padding_idx is not None:
                with torch.no_grad():
                    m.weight[m.padding_idx].zero_()
        elif isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    def forward(self, input_ids, attention_mask=None, labels=None):
        hidden = self.distilbert(input_ids, attention_mask)
        pooled = self.dropout(F.relu(self.pre_classifier(hidden[:, 0])))
        logits = self.classifier(pooled)
        if labels is not None:
            lg, lb = logits.view(-1, self.config.num_labels), labels.view(-1)
            # native kernels on: the fused gfx950 cross-entropy (ops/loss.py), same math
            loss = native_ce(lg, lb) if self.config.fused_attention else F.cross_entropy(lg, lb)
            return SequenceClassifierOutput((loss, logits))
        return SequenceClassifierOutput((logits,))


def distilbert_base(num_labels: int = 2, **overrides) -> DistilBertForSequenceClassification:
    return DistilBertForSequenceClassification(DistilBertConfig(num_labels=num_labels, **overrides))
