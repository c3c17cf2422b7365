"""Where the two stages of the headline MLP run on an N-GPU node: a link/compute cost model.

The reference places stage 0 on rank 0 and stage 1 on rank 1 and moves every boundary tensor
between them (/root/reference/simple_distributed.py:33-37, :47-49, :71, :112). On MI355X the
784-128-10 MLP computes a sample in ~1.4 ns, while its boundary costs 512 B forward plus 40 B back
(factored gradient, parallel/pipeline.py) — ~11 ns on one xGMI link. So where the boundary goes is
the main decision of a multi-GPU run, and it is made here from a model instead of by default:

``pp2dp``     the reference's placement, replicated: GPU pairs (stage 0 | stage 1) with the
              Chimera schedule (both directions, so both GPUs do equal work), data-parallel over
              N/2 pairs; every boundary byte goes over the pair's ONE link.
``rotate``    every GPU owns a data shard and hosts both stages; an equal share of every wave's
              rows runs stage 1 on each peer, so the boundary fans out over all N-1 links.
``dp``        both stages on every GPU, nothing crosses (rows stay on their owner); only the
              gradient all-reduce uses the links.
``balanced``  rotate with the cross-GPU fraction phi chosen so that the boundary traffic the
              links carry stays under the compute it overlaps (``link_budget`` of the step).

The model (documented in README "Multi-GPU placement") is deliberately simple:

* compute per GPU = rows x ns/row of what it runs (fused stage 0 + 1 for the rows it keeps, stage 0 or stage 1
  alone for crossing rows) + a fixed per-step cost (measured on one MI355X, ``ComputeModel``);
* link time = the busiest link's bytes / ``LinkModel.gbps`` + one launch latency per collective;
* the exchange overlaps compute (the transfers run on RCCL streams beside the kernels of other
  waves and of the local rows): step = max(compute, link) + the part that cannot overlap (the
  first wave's forward exchange when nothing local is left to compute, a fixed ``exposed``
  fraction of the link time);
* gradient all-reduce: ring over N GPUs of the parameter bytes, priced by the path the engine runs
  (``dp_split``, default: what ``dp_split_default()`` says the engine does). With the split on and nothing
  crossing GPUs (dp) the first layer's weight gradient runs as two hidden-unit ranges and range 0's
  all-reduce overlaps range 1's kernel (parallel/pipeline.py, SDML_DP_SPLIT), so only range 1's half plus
  what range 0's collective does not hide is exposed: ``half + max(0, half - wgrad/2)`` plus the split's
  own cost (``ComputeModel.split_us``); with it off (and for the other placements) the whole all-reduce
  follows the last backward, exposed, plus the separate optimizer launch the all-reduce forces
  (``ComputeModel.dp_step_us``), which bench.py's HIP-graph replay of the ``dp`` step mostly removes
  (``ComputeModel.dp_graph_step_us``: the stream hand-offs to and from the collective are graph edges).

``choose`` returns the placement with the smallest predicted step; among placements within 2% of
it, the one that moves the most boundary bytes across GPUs (the split the benchmark is about).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Dict, Optional, Tuple

PLACEMENTS = ("auto", "balanced", "rotate", "dp", "pp2dp")


@dataclass
class LinkModel:
    # sustained RCCL bytes/s per xGMI link and direction while kernels share the GPU (MI355X: 7 links
    # of 153.6 GB/s bidirectional peak each; RCCL all-to-all reaches roughly 2/3 of a direction's peak)
    gbps: float = 50.0
    links: int = 7
    collective_us: float = 12.0   # launch + handshake per collective
    exposed: float = 0.15         # fraction of the link time that cannot hide under compute
    link_budget: float = 0.75     # balanced: keep the busiest link busy at most this share of the step
    # measured gradient all-reduce of the parameters (parallel/linkprobe.py); None: the ring formula below
    allreduce_us: Optional[float] = None


@dataclass
class ComputeModel:
    """Per-row costs of the 784-128-10 stages on one MI355X at 131072 rows per GPU, from the round-5 kernel tables.

    * rows that stay on their owner run the fused uint8 forward + classifier head and the factored weight gradient:
      69.3 + 68.5 us (profiles/r5_bench_n1_w2_staged_kernel_stats.txt) -> ``fused_ns``;
    * rows whose stage 1 runs elsewhere (and pp2dp) run the plain uint8 forward + weight gradient on the owner, 61.8
      + 72.1 us -> ``s0_ns``, and the standalone block head on the peer, 28.5 us -> ``s1_ns``
      (profiles/r5_bench_n1_unfused_kernel_stats.txt, SDML_FUSE_HEAD=0);
    * ``fixed_us``: the slab + head reduction with the fused SGD (11 us) and the launch gaps, i.e. the N = 1 step
      (0.1515 ms, profiles/r5_bench_n1_head_dpp.jsonl..w2_staged runs) minus its fused kernels;
    * ``dp_step_us``: what a step with a gradient all-reduce costs on top at N > 1 before any link time - the
      reduction can no longer apply SGD in the same launch, a separate optimizer launch follows the collective, plus
      the collective's host and stream overhead: the one-rank RCCL harness (tools/bench_dp_split.py) runs the N > 1
      path in 0.1754 ms against 0.1515 (profiles/r5_dpsplit_one_rank_rccl.jsonl);
    * ``dp_graph_step_us``: the same when the step (collective included) replays from a HIP graph, as bench.py runs
      ``dp`` at N > 1: 0.1533 vs 0.1498 ms on the same harness, where the eager step pays ~25 us between the
      reduction and the optimizer launch for the two cross-stream waits around the collective
      (profiles/r5_dp_graph_one_rank_rccl.jsonl);
    * ``split_us``: the split weight gradient's own extra cost (same harness: 0.2099 vs 0.1754 ms);
    * ``wgrad_ns``: the weight gradient alone (the split hides range 0's all-reduce under half of it)."""
    fused_ns: float = 1.051
    s0_ns: float = 1.022
    s1_ns: float = 0.217
    fixed_us: float = 13.7
    wgrad_ns: float = 0.523
    act_bytes: int = 512          # boundary activation per row (128 fp32)
    grad_bytes: int = 40          # factored boundary gradient per row (10 fp32)
    param_bytes: int = 101_770 * 4
    dp_step_us: float = 24.0
    dp_graph_step_us: float = 3.5
    split_us: float = 34.5


def dp_split_default() -> bool:
    """Whether the engine splits the data-parallel gradient all-reduce (parallel/pipeline.py reads the same
    variable): the model must price the path that runs."""
    import os

    return os.environ.get("SDML_DP_SPLIT", "0") == "1"


def predict(placement: str, n: int, batch_per_gpu: int, waves: int = 2, phi: Optional[float] = None,
            link: LinkModel = LinkModel(), comp: ComputeModel = ComputeModel(),
            dp_split: Optional[bool] = None, graph: Optional[bool] = None) -> Dict[str, float]:
    """Predicted step of ``placement`` at ``n`` GPUs (weak scaling: ``batch_per_gpu`` rows per GPU). ``graph``:
    the step replays from a HIP graph (default: what bench.py does, i.e. for ``dp`` without the split)."""
    if dp_split is None:
        dp_split = dp_split_default()
    if graph is None:
        graph = placement == "dp" and not dp_split
    B = float(batch_per_gpu)
    row = comp.act_bytes + comp.grad_bytes
    if n == 1:
        placement, phi = "dp", 0.0
    if placement == "rotate":
        phi = (n - 1) / n
    if placement == "dp":
        phi = 0.0
    if placement == "pp2dp":
        compute_us = B * (comp.s0_ns + comp.s1_ns) / 1e3 + comp.fixed_us
    else:  # rows kept on their owner run fused; for the crossing share the owner runs stage 0, a peer stage 1
        phi_c = (n - 1) / n if placement == "rotate" else float(phi or 0.0)
        compute_us = B * ((1 - phi_c) * comp.fused_ns + phi_c * (comp.s0_ns + comp.s1_ns)) / 1e3 + comp.fixed_us
    if placement == "pp2dp":
        if n % 2:
            raise ValueError("pp2dp needs an even number of GPUs")
        # Chimera: each GPU runs stage 0 for its own B rows and stage 1 for its partner's B rows;
        # all B rows' boundary crosses the pair's single link in each direction
        link_bytes = B * row
        ncoll = 4 * waves  # per micro-batch: act + grad, both directions
        phi = 1.0
        cross_bytes = B * row
    else:
        phi = float(phi or 0.0)
        cross_bytes = phi * B * row
        link_bytes = cross_bytes / max(1, n - 1)
        ncoll = 2 * waves if phi > 0 else 0
    link_us = link_bytes / (link.gbps * 1e3) + ncoll * link.collective_us
    if n > 1:  # ring all-reduce of the gradients (2 (n-1)/n of the bytes per GPU, over 2 ring links), or as measured
        ar_us = (link.allreduce_us if link.allreduce_us is not None
                 else 2 * (n - 1) / n * comp.param_bytes / (2 * link.gbps * 1e3) + link.collective_us)
        if dp_split and (placement == "dp" or (placement != "pp2dp" and phi == 0)):
            # split: two half collectives, range 0's under range 1's kernel
            half = (ar_us - link.collective_us) / 2 + link.collective_us
            ar_us = half + max(0.0, half - B * comp.wgrad_ns / 2e3) + comp.split_us
        ar_us += comp.dp_graph_step_us if graph else comp.dp_step_us
    else:
        ar_us = 0.0
    if link_bytes > 0:
        step_us = max(compute_us, link_us) + link.exposed * link_us + ar_us
    else:
        step_us = compute_us + ar_us
    return {
        "placement": placement, "n_gpus": n, "cross_fraction": round(phi, 4),
        "compute_ms": round(compute_us / 1e3, 4), "link_ms": round(link_us / 1e3, 4),
        "allreduce_ms": round(ar_us / 1e3, 4), "step_ms": round(step_us / 1e3, 4),
        "samples_per_s": round(n * B / (step_us / 1e6), 1),
        "boundary_bytes_per_gpu": int(cross_bytes), "busiest_link_bytes": int(link_bytes),
    }


def balanced_fraction(n: int, batch_per_gpu: int, link: LinkModel = LinkModel(),
                      comp: ComputeModel = ComputeModel(), waves: int = 2) -> float:
    """Largest phi whose busiest-link time stays within ``link_budget`` of the compute it overlaps."""
    if n == 1:
        return 0.0
    B = float(batch_per_gpu)
    compute_us = B * comp.fused_ns / 1e3 + comp.fixed_us  # (phi small: most rows stay)
    budget_us = link.link_budget * compute_us - 2 * waves * link.collective_us
    if budget_us <= 0:
        return 0.0
    per_link_bytes = budget_us * link.gbps * 1e3
    phi = per_link_bytes * (n - 1) / (B * (comp.act_bytes + comp.grad_bytes))
    phi = min(phi, (n - 1) / n)
    return max(0.0, round(phi * 64) / 64)  # a 1/64 grid: the same phi on every rank, readable in logs


def table(n: int, batch_per_gpu: int, waves: int = 2, link: LinkModel = LinkModel(),
          comp: ComputeModel = ComputeModel(), graph_dp: Optional[bool] = None) -> Dict[str, Dict[str, float]]:
    """Predictions of every placement. ``graph_dp``: whether the caller replays the ``dp`` step from a HIP graph
    (bench.py: RCCL transport at N > 1, graphs not off, no split); None: assume it does (predict's default)."""
    out = {}
    for p in ("balanced", "rotate", "dp", "pp2dp"):
        if p == "pp2dp" and (n % 2 or n == 1):
            continue
        phi = balanced_fraction(n, batch_per_gpu, link, comp, waves) if p == "balanced" else None
        graph = None if graph_dp is None else (bool(graph_dp) if p == "dp" else False)
        out[p] = predict(p, n, batch_per_gpu, waves, phi, link, comp, graph=graph)
    return out


def choose(n: int, batch_per_gpu: int, waves: int = 2, link: LinkModel = LinkModel(),
           comp: ComputeModel = ComputeModel(),
           graph_dp: Optional[bool] = None) -> Tuple[str, float, Dict[str, Dict[str, float]]]:
    """(placement, cross_fraction, predictions): the fastest predicted placement; within 2% of it,
    the one that sends the most boundary bytes across GPUs."""
    t = table(n, batch_per_gpu, waves, link, comp, graph_dp)
    best = min(v["step_ms"] for v in t.values())
    near = [p for p, v in t.items() if v["step_ms"] <= best * 1.02]
    pick = max(near, key=lambda p: (t[p]["boundary_bytes_per_gpu"], -t[p]["step_ms"]))
    return pick, t[pick]["cross_fraction"], t


def model_dict(link: LinkModel = LinkModel(), comp: ComputeModel = ComputeModel()) -> Dict[str, Dict[str, float]]:
    return {"link": asdict(link), "compute": asdict(comp)}


def markdown_table(ns=(2, 4, 8), batch_per_gpu: int = 131072) -> str:
    """README's placement table ("Multi-GPU placement"), generated from :func:`table` (tests/test_placement_doc.py
    checks that README holds exactly this text)."""
    rows = ["| N | predicted step (ms) and samples/s: `dp` | `balanced` (φ of the rows cross) | `rotate` (all links) "
            "| `pp2dp` (the reference's cut, per pair) |", "|---|---|---|---|---|"]
    for n in ns:
        t = table(n, batch_per_gpu)

        def cell(p):
            v = t[p]
            extra = f" (φ = {v['cross_fraction']})" if p == "balanced" else ""
            return f"{v['step_ms']:.3f} · {v['samples_per_s'] / 1e9:.2f} G{extra}"

        rows.append(f"| {n} | " + " | ".join(cell(p) for p in ("dp", "balanced", "rotate", "pp2dp")) + " |")
    return "\n".join(rows)
