"""Tensor parallelism inside a pipeline stage (Megatron-style column/row-parallel Linear).

Not in the reference (SURVEY.md §2b lists TP as an optional extension for the GPT-2 stages).
A TP group of ``tp`` ranks holds one pipeline stage together:

* column-parallel Linear (``c_attn``, ``mlp.c_fc``): each rank keeps a slice of the output
  features (for ``c_attn`` the q/k/v columns of its own attention heads), so attention and GELU
  run on local data;
* row-parallel Linear (``attn.c_proj``, ``mlp.c_proj``): each rank keeps the matching slice of
  the input features; the partial outputs are summed with ONE RCCL all-reduce per sub-layer,
  then the (replicated) bias is added.

Two autograd functions carry the communication: :func:`copy_to_tp` (identity forward,
all-reduce of the input gradient backward) in front of a column-parallel layer, and
:func:`reduce_from_tp` (all-reduce forward, identity backward) after a row-parallel one.
Everything else in the stage (LayerNorms, embeddings, ``lm_head``) is replicated. Its
gradients are identical on every TP rank, because the all-reduce in the backward of
``copy_to_tp`` gives every rank the same residual-stream gradient, so the data-parallel
all-reduce is the only gradient sync.

On MI355X the TP group is one node's xGMI mesh (every GPU pair has a direct link). Each
all-reduce moves 2·(tp-1)/tp of a [tokens, 768] bf16 activation per sub-layer.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch


@dataclass
class TPContext:
    size: int
    rank: int
    group: Optional[object]  # None when size == 1
    transport: Optional[object] = None  # parallel/p2p.py Transport of the rank


def _all_reduce(x: torch.Tensor, ctx: TPContext) -> torch.Tensor:
    if ctx.size == 1:
        return x
    x = x.contiguous()
    ctx.transport.all_reduce(x, group=ctx.group, async_op=False)
    return x


class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(c, x, ctx: TPContext):
        c.tp = ctx
        return x

    @staticmethod
    def backward(c, g):
        return _all_reduce(g.clone(), c.tp), None


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(c, x, ctx: TPContext):
        return _all_reduce(x.clone(), ctx)

    @staticmethod
    def backward(c, g):
        return g, None


def copy_to_tp(x: torch.Tensor, ctx: Optional[TPContext]) -> torch.Tensor:
    if ctx is None or ctx.size == 1:
        return x
    return _CopyToTP.apply(x, ctx)


def reduce_from_tp(x: torch.Tensor, ctx: Optional[TPContext]) -> torch.Tensor:
    if ctx is None or ctx.size == 1:
        return x
    return _ReduceFromTP.apply(x, ctx)


def column_slice(n: int, ctx: TPContext) -> slice:
    if n % ctx.size:
        raise ValueError(f"{n} features cannot be split over tp={ctx.size}")
    per = n // ctx.size
    return slice(ctx.rank * per, (ctx.rank + 1) * per)


def shard_parameter(module: torch.nn.Module, name: str, dim: int, index) -> None:
    """Replace ``module.<name>`` by the slice ``index`` (a tensor of indices or a slice) along ``dim``."""
    p = getattr(module, name)
    with torch.no_grad():
        data = p.data.index_select(dim, index) if torch.is_tensor(index) else p.data.narrow(
            dim, index.start, index.stop - index.start)
    setattr(module, name, torch.nn.Parameter(data.clone().contiguous(), requires_grad=p.requires_grad))
