"""BERT (Devlin et al. 2018) for pre-training, written from scratch — config 5
of BASELINE.json: BERT-Large (24 x 1024, 16 heads, FFN 4096, vocab 30522,
336M parameters) bf16, trained with fp16 gradient compression + Adasum.

MI355X choices: bf16 weights and activations end to end (fp32 master weights
live in mivod's fused optimizer), Q/K/V as one [3H, H] projection GEMM, the
MLM head evaluated only on the masked positions (the MLPerf/NVIDIA trick: the
vocab GEMM shrinks ~6x at 15% masking), no torch.compile / Triton — the GEMMs
are hipBLASLt via torch.matmul, attention is mivod's own path
(``mivod.ops.attention``), and every bias / GELU / dropout / residual /
LayerNorm chain is one fused kernel each way (``mivod.ops.transformer``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.bn import tap
from ..ops.transformer import bias_dropout_add_ln, bias_gelu


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02

    @classmethod
    def large(cls, **kw):
        return cls(**kw)

    @classmethod
    def base(cls, **kw):
        return cls(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                   intermediate_size=3072, **kw)

    @classmethod
    def tiny(cls, **kw):
        d = dict(vocab_size=512, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                 intermediate_size=128, max_position_embeddings=64)
        d.update(kw)
        return cls(**d)


class BertEmbeddings(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden_size)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids):
        s = input_ids.shape[1]
        pos = torch.arange(s, device=input_ids.device)
        x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None] + \
            self.token_type_embeddings(token_type_ids)
        return self.dropout(bias_dropout_add_ln(x, None, None, self.LayerNorm))


class BertSelfAttention(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.h = c.num_attention_heads
        self.d = c.hidden_size // c.num_attention_heads
        self.qkv = nn.Linear(c.hidden_size, 3 * c.hidden_size)
        self.dense = nn.Linear(c.hidden_size, c.hidden_size)
        self.p_attn = c.attention_probs_dropout_prob
        self.dropout = nn.Dropout(c.hidden_dropout_prob)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)

    def forward(self, x, mask_bias):
        from ..ops.attention import attention
        b, s, hd = x.shape
        qkv = self.qkv(x).view(b, s, 3, self.h, self.d)
        ctx = attention(qkv, mask_bias, self.p_attn if self.training else 0.0)   # [b, s, h*d]
        # dense GEMM without bias; bias + dropout + residual + LayerNorm fused; the
        # residual use of x is tapped: its gradient joins x's producer LN backward
        return bias_dropout_add_ln(F.linear(ctx, self.dense.weight), self.dense.bias, tap(x),
                                   self.LayerNorm, self.dropout.p, self.training)


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.attention = BertSelfAttention(c)
        self.intermediate = nn.Linear(c.hidden_size, c.intermediate_size)
        self.output = nn.Linear(c.intermediate_size, c.hidden_size)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)

    def forward(self, x, mask_bias):
        a = self.attention(x, mask_bias)
        h = bias_gelu(F.linear(a, self.intermediate.weight), self.intermediate.bias)
        return bias_dropout_add_ln(F.linear(h, self.output.weight), self.output.bias, tap(a),
                                   self.LayerNorm, self.dropout.p, self.training)


class BertModel(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.config = c
        self.embeddings = BertEmbeddings(c)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.num_hidden_layers)])
        self.pooler = nn.Linear(c.hidden_size, c.hidden_size)

    def forward(self, input_ids, token_type_ids, attention_mask=None):
        x = self.embeddings(input_ids, token_type_ids)
        # built whenever a mask is given — no data-dependent host sync per forward
        # (packed pre-training batches pass attention_mask=None: every token valid)
        mask_bias = None
        if attention_mask is not None:
            mask_bias = (1.0 - attention_mask[:, None, None, :].to(x.dtype)) * -10000.0
        for lyr in self.layers:
            x = lyr(x, mask_bias)
        pooled = torch.tanh(self.pooler(x[:, 0]))
        return x, pooled


class BertForPreTraining(nn.Module):
    """MLM (tied decoder) + next-sentence-prediction heads."""

    def __init__(self, c: BertConfig):
        super().__init__()
        self.config = c
        self.bert = BertModel(c)
        self.transform = nn.Linear(c.hidden_size, c.hidden_size)
        self.transform_ln = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.decoder_bias = nn.Parameter(torch.zeros(c.vocab_size))
        self.nsp = nn.Linear(c.hidden_size, 2)
        self.apply(self._init)

    def _init(self, m):
        r = self.config.initializer_range
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, std=r)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, std=r)
        elif isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    def forward(self, input_ids, token_type_ids, attention_mask, masked_positions,
                masked_labels, nsp_labels):
        """Returns the pre-training loss.  ``masked_positions`` [b, m] index the
        masked tokens; ``masked_labels`` [b, m] (-100 = padding)."""
        seq, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        b, m = masked_positions.shape
        idx = masked_positions + torch.arange(b, device=seq.device)[:, None] * seq.shape[1]
        sel = seq.reshape(-1, seq.shape[-1]).index_select(0, idx.reshape(-1))
        t = bias_dropout_add_ln(bias_gelu(F.linear(sel, self.transform.weight),
                                          self.transform.bias), None, None, self.transform_ln)
        logits = F.linear(t, self.bert.embeddings.word_embeddings.weight, self.decoder_bias)
        mlm = F.cross_entropy(logits.float(), masked_labels.reshape(-1), ignore_index=-100)
        nsp = F.cross_entropy(self.nsp(pooled).float(), nsp_labels)
        return mlm + nsp


def synthetic_batch(c: BertConfig, batch: int, seq: int, device, mask_frac=0.15,
                    generator=None, with_mask: bool = False):
    """Synthetic pre-training batch of full-length (packed) sequences: the
    attention mask is None (every position valid) unless ``with_mask``."""
    g = generator
    ids = torch.randint(0, c.vocab_size, (batch, seq), device=device, generator=g)
    tt = torch.zeros(batch, seq, dtype=torch.long, device=device)
    tt[:, seq // 2:] = 1
    am = torch.ones(batch, seq, dtype=torch.long, device=device) if with_mask else None
    m = max(1, int(round(seq * mask_frac)))
    pos = torch.stack([torch.randperm(seq, device=device, generator=g)[:m]
                       for _ in range(batch)]).sort(dim=1).values
    labels = torch.randint(0, c.vocab_size, (batch, m), device=device, generator=g)
    nsp = torch.randint(0, 2, (batch,), device=device, generator=g)
    return ids, tt, am, pos, labels, nsp


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
