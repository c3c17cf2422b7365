"""Measured link constants for the placement model (parallel/placement.py), taken on the job's own process group
before the placement is chosen.

``LinkModel``'s defaults are estimates (a sustained per-link rate, a per-collective latency). A multi-GPU bench
run measures them instead, on the collectives the placements actually issue, and feeds the measured model into
``placement.choose``; the JSON carries both. The reference moves its boundary with RPC round trips
(/root/reference/simple_distributed.py:47-49, :71, :112); these are the RCCL (or Gloo) operations that replace them:

* ``allreduce_us``: the gradient all-reduce of the headline MLP's 101,770 fp32 parameters (407 KB), the only
  collective of the ``dp`` placement (reference step :112-113 becomes backward + all-reduce + SGD);
* ``collective_us``: an all-to-all of 1 KiB per peer, i.e. the fixed cost of one boundary collective (``rotate``);
* ``gbps``: per-link bytes/s of an all-to-all carrying ``boundary_bytes`` spread over the peers (the boundary of a
  ``rotate`` wave; every peer gets its own share, so the busiest link carries bytes / (N - 1));
* ``pair_gbps``: one direction of an isend / irecv exchange of ``boundary_bytes`` between the GPUs of a pair
  (rank ^ 1), the reference's own cut (``pp2dp``).

Every timing is the MAX over ranks of the median of ``reps`` repetitions, each bracketed by a device sync (a
collective's whole latency, as an exposed step pays it).
"""
from __future__ import annotations

import statistics
import time
from typing import Dict

import torch
import torch.distributed as dist


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _time(fn, dev, reps: int, warm: int = 2) -> float:
    for _ in range(warm):
        fn()
    _sync(dev)
    ts = []
    for _ in range(reps):
        if dev.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[dev.index])
        else:
            dist.barrier()
        _sync(dev)
        t0 = time.perf_counter()
        fn()
        _sync(dev)
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def _max_over_ranks(vals, dev):
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def measure(dev: torch.device, boundary_bytes: int, param_count: int = 101_770, reps: int = 5) -> Dict[str, float]:
    """Measure the link constants on the default process group (world size N > 1). ``dev``: where the group's
    tensors live (the GPU for RCCL, the CPU for Gloo)."""
    n, rank = dist.get_world_size(), dist.get_rank()
    grads = torch.zeros(param_count, dtype=torch.float32, device=dev)
    t_ar = _time(lambda: dist.all_reduce(grads), dev, reps)

    small_in = torch.zeros(256 * n, dtype=torch.float32, device=dev)  # 1 KiB per peer
    small_out = torch.empty_like(small_in)
    t_small = _time(lambda: dist.all_to_all_single(small_out, small_in), dev, reps)

    per_peer = max(256, int(boundary_bytes) // (4 * max(1, n - 1)))  # fp32 elements per peer
    big_in = torch.zeros(per_peer * n, dtype=torch.float32, device=dev)
    big_out = torch.empty_like(big_in)
    t_big = _time(lambda: dist.all_to_all_single(big_out, big_in), dev, reps)

    pair = rank ^ 1
    t_pair = 0.0
    nb = max(256, int(boundary_bytes) // 4)
    if n % 2 == 0:
        sbuf = torch.zeros(nb, dtype=torch.float32, device=dev)
        rbuf = torch.empty_like(sbuf)

        def exchange():
            ops = [dist.P2POp(dist.isend, sbuf, pair), dist.P2POp(dist.irecv, rbuf, pair)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()

        t_pair = _time(exchange, dev, reps)
    t_ar, t_small, t_big, t_pair = _max_over_ranks([t_ar, t_small, t_big, t_pair], dev)
    coll_us = t_small * 1e6
    link_bytes = per_peer * 4  # one peer's share: what the busiest link carries
    big_us = max(t_big * 1e6 - coll_us, 1e-3)
    out = {
        "world_size": n,
        "backend": dist.get_backend(),
        "allreduce_us": round(t_ar * 1e6, 2),
        "allreduce_bytes": param_count * 4,
        "collective_us": round(coll_us, 2),
        "alltoall_us": round(t_big * 1e6, 2),
        "alltoall_bytes_per_peer": link_bytes,
        "gbps": round(link_bytes / big_us / 1e3, 3),
        "reps": reps,
    }
    if t_pair > 0:
        out["pair_us"] = round(t_pair * 1e6, 2)
        out["pair_bytes"] = nb * 4
        out["pair_gbps"] = round(nb * 4 / max(t_pair * 1e6 - coll_us, 1e-3) / 1e3, 3)
    return out


def link_model(meas: Dict[str, float]):
    """A ``placement.LinkModel`` with the measured rate and per-collective cost (other fields: defaults)."""
    from .placement import LinkModel

    lm = LinkModel()
    if meas.get("gbps", 0) > 0:
        lm.gbps = float(meas["gbps"])
    if meas.get("collective_us", 0) > 0:
        lm.collective_us = float(meas["collective_us"])
    return lm
