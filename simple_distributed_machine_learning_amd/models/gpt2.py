"""GPT-2 (small: 12 layers, d=768, 12 heads, ctx 1024, vocab 50257) split into pipeline
stages, bf16 (BASELINE config 5: "2-stage GPT-2-small transformer split bf16").

Stage 0 owns the token/position embeddings, the last stage owns ``ln_f`` + ``lm_head``;
the 12 blocks are divided evenly. Boundary tensor: [mb, S, 768] bf16 (1.5 MiB per sample
at S=1024) — the large-activation send that RCCL p2p overlaps with compute.

The output projection is untied from ``wte`` because the two live on different ranks
(documented deviation from the 124M tied checkpoint; +38.6M parameters on the last stage).
Linear layers (ops/linear.py) and LayerNorms accumulate their weight/bias gradients straight
into the flat gradient buffer (GEMM beta = 1, in-place bf16 reductions) instead of
materialise-then-add. Parameter names follow the common GPT-2 layout (wte, wpe, h.{i}.ln_1, h.{i}.attn.c_attn,
h.{i}.attn.c_proj, h.{i}.ln_2, h.{i}.mlp.c_fc, h.{i}.mlp.c_proj, ln_f, lm_head).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from .base import ModelSpec, PipelineStage
from ..ops.linear import Linear, linear, lm_head, mlp_gelu
from ..ops.transformer import (LayerNorm, add_layer_norm, causal_attention, cross_entropy_sum, embedding, gelu,
                               layer_norm_pass)
from ..parallel.tp import TPContext, column_slice, copy_to_tp, reduce_from_tp, shard_parameter


@dataclass
class GPT2Config:
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    vocab_size: int = 50257
    block_size: int = 1024
    dropout: float = 0.0


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_attn = Linear(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = Linear(cfg.n_embd, cfg.n_embd)
        self.n_head = cfg.n_head
        self.tp: TPContext = None

    def shard_tp(self, tp: TPContext):
        """Keep this rank's heads: the q/k/v columns of c_attn (column-parallel) and the matching
        input features of c_proj (row-parallel; its bias stays whole, added after the reduce)."""
        C = self.c_proj.weight.shape[0]
        cols = column_slice(C, tp)
        idx = torch.cat([torch.arange(cols.start, cols.stop) + i * C for i in range(3)])
        shard_parameter(self.c_attn, "weight", 0, idx)
        shard_parameter(self.c_attn, "bias", 0, idx)
        shard_parameter(self.c_proj, "weight", 1, cols)
        self.n_head //= tp.size
        self.tp = tp

    def forward(self, x):
        # HIP flash attention (bf16, head_dim 64) on ROCm; PyTorch SDPA elsewhere
        if self.tp is None:
            return self.c_proj(causal_attention(self.c_attn(x), self.n_head))
        a = causal_attention(self.c_attn(copy_to_tp(x, self.tp)), self.n_head)
        return reduce_from_tp(linear(a, self.c_proj.weight), self.tp) + self.c_proj.bias


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_fc = Linear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = Linear(4 * cfg.n_embd, cfg.n_embd)
        self.tp: TPContext = None

    def shard_tp(self, tp: TPContext):
        cols = column_slice(self.c_fc.weight.shape[0], tp)
        shard_parameter(self.c_fc, "weight", 0, cols)
        shard_parameter(self.c_fc, "bias", 0, cols)
        shard_parameter(self.c_proj, "weight", 1, cols)
        self.tp = tp

    def forward(self, x):
        if self.tp is None:  # GELU fused into the c_fc forward / c_proj input-gradient GEMM epilogues
            return mlp_gelu(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias)
        h = gelu(self.c_fc(copy_to_tp(x, self.tp)))
        return reduce_from_tp(linear(h, self.c_proj.weight), self.tp) + self.c_proj.bias


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = LayerNorm(cfg.n_embd)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = LayerNorm(cfg.n_embd)
        self.mlp = MLP(cfg)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class GPT2Stage(PipelineStage):
    def __init__(self, cfg: GPT2Config, stage_id: int, num_stages: int):
        super().__init__()
        if cfg.n_layer % num_stages:
            raise ValueError("n_layer must be divisible by num_stages")
        self.cfg = cfg
        self.stage_id, self.num_stages = stage_id, num_stages
        self.loss_kind = "ce"
        per = cfg.n_layer // num_stages
        if stage_id == 0:
            self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
            self.wpe = nn.Embedding(cfg.block_size, cfg.n_embd)
        self.h = nn.ModuleDict({str(i): Block(cfg) for i in range(stage_id * per, (stage_id + 1) * per)})
        if stage_id == num_stages - 1:
            self.ln_f = LayerNorm(cfg.n_embd)
            self.lm_head = Linear(cfg.n_embd, cfg.vocab_size, bias=False)
            # the vocabulary padded to a multiple of 64 rows in the flat storage (zero rows, zero gradient): the
            # lm_head's three GEMMs run on the hand-written kernels as 50304-wide GEMMs (ops/linear.py lm_head)
            self.flat_row_multiple = {"lm_head.weight": 64}
        self._init()

    supports_tp = True

    def shard_tp(self, tp: TPContext):
        """Tensor-parallel split of every block (parallel/tp.py); embeddings, LayerNorms and the
        vocabulary head stay replicated."""
        if self.cfg.n_head % tp.size:
            raise ValueError(f"n_head={self.cfg.n_head} is not divisible by tp={tp.size}")
        for blk in self.h.values():
            blk.attn.shard_tp(tp)
            blk.mlp.shard_tp(tp)
        self.tp = tp

    def _init(self):
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight"):
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * self.cfg.n_layer))
            elif p.dim() >= 2:
                nn.init.normal_(p, 0.0, 0.02)
            elif name.endswith("bias"):
                nn.init.zeros_(p)

    # ---- last stage: fused vocab cross-entropy (no fp32 copy of the [tokens, 50257] logits) --
    def head_fwd(self, x, target, ctx, train, loss_scale, stats=None):
        if not train:
            with torch.no_grad():
                logits = self(x)
                l, c, n, _ = cross_entropy_sum(logits.reshape(-1, logits.shape[-1]), target.reshape(-1), 1.0, False)
            return l, c, n
        if not self.is_first:
            x = x.detach().requires_grad_(True)
        with torch.enable_grad():
            logits = self(x)
        l, c, n, g = cross_entropy_sum(logits.detach().reshape(-1, logits.shape[-1]), target.reshape(-1),
                                       loss_scale, True)
        ctx["x"], ctx["logits"], ctx["glogits"] = x, logits, g.view_as(logits)
        return l, c, n

    def head_bwd(self, ctx):
        x, logits, g = ctx.pop("x"), ctx.pop("logits"), ctx.pop("glogits")
        torch.autograd.backward(logits, g)
        return None if self.is_first else x.grad

    def forward(self, x):
        if self.stage_id == 0:  # token + position embedding (HIP gather, deterministic backward)
            x = embedding(x, self.wte.weight, self.wpe.weight)
        last = self.stage_id == self.num_stages - 1
        blocks = list(self.h.values())
        if not blocks:
            return lm_head(self.ln_f(x), self.lm_head.weight) if last else x
        # each residual add is fused into the LayerNorm that reads its sum (ln_2 of the same block,
        # ln_1 of the next, ln_f at the end); the block maths is exactly Block.forward
        x, y = layer_norm_pass(x, blocks[0].ln_1)  # (x feeds ln_1 and the residual: one backward node for both)
        for i, blk in enumerate(blocks):
            x, y = add_layer_norm(x, blk.attn(y), blk.ln_2)
            m = blk.mlp(y)
            nxt = blocks[i + 1].ln_1 if i + 1 < len(blocks) else (self.ln_f if last else None)
            if nxt is None:
                x = x + m
            else:
                x, y = add_layer_norm(x, m, nxt)
        return lm_head(y, self.lm_head.weight) if last else x


def gpt2_spec(num_stages: int = 2, cfg: GPT2Config = None, seq_len: int = None, dtype=torch.bfloat16,
              name: str = "gpt2") -> ModelSpec:
    cfg = cfg or GPT2Config()
    S = min(seq_len or cfg.block_size, cfg.block_size)

    def build(s):
        return GPT2Stage(cfg, s, num_stages)

    def shape(s, mb):
        return (mb, S, cfg.n_embd)

    return ModelSpec(name=name, num_stages=num_stages, build_stage=build, boundary_shape=shape,
                     boundary_dtype=dtype, input_kind="tokens", param_dtype=dtype, vocab_size=cfg.vocab_size,
                     seq_len=S)
