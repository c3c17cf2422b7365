"""hipGraph capture of a whole training step.

At the reference's batch of 60 a step is a few microseconds of GPU work, and the host
cannot keep up. Python dispatch and ~10 kernel launches cost hundreds of microseconds, and
the reference's RPC round trips cost milliseconds (/root/reference/simple_distributed.py:108-113).
:class:`GraphedStep` records the engine's step once into a HIP graph and then replays it.
The recorded step covers data reads, every stage's forward and backward, the loss and
metrics, the fused SGD update, and the device step counter. A replay is one host call.

What changes between replays, and how it gets into the graph:

* data: the graph reads from static buffers, one per slice the engine asks for. A first,
  discarded capture discovers the slices, and the buffers are allocated outside the graph's
  pool. A buffer allocated inside the pool could alias memory that earlier nodes of the
  same graph reuse. Before each replay the step's real slices are copied into the buffers.
  These are device-to-device copies, because the datasets already live in HBM.
  ``direct_data=True`` (a device-resident dataset that a training loop cycles through, e.g.
  bench.py's synthetic batches): one graph per (dataset, start) that reads the dataset's own
  slices, so a replay moves no data at all (at batch 131072 the copy would be 103 MB of
  uint8 pixels, ~25 us of HBM traffic, per step). At most ``max_direct`` such graphs; a step
  past that cap runs eagerly.
* dropout: the fused kernels mix the engine's device step counter into their seeds. The
  graph increments that counter, so each replay draws fresh masks.
* the optimizer: the first step (momentum-buffer initialisation) runs eagerly, so the
  captured SGD launch is the steady-state update.

Constraints (checked): a CUDA/ROCm engine; a training step with an optimizer update; and
one process, unless ``allow_collectives``: RCCL collectives are captured then (the gradient
all-reduce, boundary all-to-alls); tests/test_graphs_gpu.py replays a step whose all-reduce runs on a
one-rank RCCL communicator. The returned
:class:`StepResult` tensors belong to the graph and are overwritten by the next replay, so
read them first. The ragged last batch of an epoch has a different shape and gets its own
graph. A failed capture falls back to eager execution and emits a warning.
"""
from __future__ import annotations

import time
import warnings
from typing import Dict, Optional, Tuple

import torch

from .pipeline import PipelineEngine, StepResult


class _StaticWindow:
    """Dataset seen by the engine during capture: every (kind, offset, n) slice it reads maps
    to a persistent buffer; :meth:`load` fills them from the real dataset for one step.

    ``discover`` mode (first capture) only records the slices and hands out placeholders;
    :meth:`freeze` then allocates the real buffers OUTSIDE any graph pool."""

    def __init__(self, real):
        self.real = real
        self.bufs: Dict[Tuple[str, int, int], torch.Tensor] = {}
        self.keys = []
        self.discover = True
        self.seq_len = getattr(real, "seq_len", None)
        self.n = len(real)

    def __len__(self):
        return self.n

    def _src(self, kind, start, n):
        return self.real.inputs(start, n) if kind == "x" else self.real.targets(start, n)

    def _buf(self, kind: str, start: int, n: int) -> torch.Tensor:
        key = (kind, start, n)
        if self.discover:
            if key not in self.keys:
                self.keys.append(key)
            return torch.empty_like(self._src(*key), memory_format=torch.contiguous_format)
        if key not in self.bufs:
            raise RuntimeError(f"graph capture read an undiscovered slice {key}")
        return self.bufs[key]

    def freeze(self):
        self.discover = False
        for key in self.keys:
            self.bufs[key] = torch.empty_like(self._src(*key), memory_format=torch.contiguous_format)

    def inputs(self, start: int, n: int) -> torch.Tensor:
        return self._buf("x", start, n)

    def targets(self, start: int, n: int) -> torch.Tensor:
        return self._buf("y", start, n)

    def load(self, dataset, delta: int):
        """Copy the slices at (offset + delta) of ``dataset`` into the static buffers."""
        for (kind, start, n), buf in self.bufs.items():
            src = dataset.inputs(start + delta, n) if kind == "x" else dataset.targets(start + delta, n)
            buf.copy_(src, non_blocking=True)


class GraphedStep:
    """``step(dataset, start, batch_size, global_batch)`` == ``engine.run(..., train=True)``
    replayed from a captured HIP graph (one graph per (batch_size, global_batch))."""

    def __init__(self, engine: PipelineEngine, allow_collectives: bool = False, direct_data: bool = False,
                 max_direct: int = 16):
        if engine.device.type != "cuda":
            raise ValueError("GraphedStep needs a ROCm device engine")
        if engine.mesh.world_size > 1 and not allow_collectives:
            raise ValueError("GraphedStep: multi-process capture (RCCL in the graph) is opt-in: "
                             "pass allow_collectives=True")
        self.engine = engine
        self.direct = direct_data
        self.max_direct = max_direct
        self.eager_steps = 0
        # (graph, window, result, start, planes_current, relies_on_planes) per (batch, global batch)
        self.graphs: Dict[Tuple[int, Optional[int]], tuple] = {}
        self._planes_current = True
        self._relies_on_planes = False
        self.pool = None
        self.disabled = False
        self.replays = 0
        # eager warm-up steps and captures share one side stream: autograd's AccumulateGrad
        # nodes remember the stream they were created on, and a capture on a different stream
        # would make them synchronise with it (not permitted while capturing)
        self.stream = torch.cuda.Stream(device=engine.device)

    def _plane_caches(self):
        """(cache, weight) of every derived weight cache a captured step relies on (ops.PlaneCache)."""
        return [(m.plane_cache, m.layers()[0].weight) for m in self.engine.stages.values()
                if getattr(m, "plane_cache", None) is not None]

    def _caches_current(self) -> bool:
        """A replay reuses the plane caches the way they were at capture (valid, kept current by the
        captured SGD step); a torch in-place write to a weight since (checkpoint load, user edit) bumps
        its version and makes them stale."""
        from ..ops import PlaneCache

        ep = self.engine.flat.param_epoch
        return all(c.token == PlaneCache.token_of(w, ep) for c, w in self._plane_caches())

    def _record(self, win, start, batch_size, global_batch, pool):
        eng = self.engine
        gs, steps, zero = eng.global_step, eng.optimizer.steps, eng.flat.grads_zero
        epoch, tokens = eng.flat.param_epoch, [c.token for c, _ in self._plane_caches()]
        # a graph captured while the caches were current reads them without re-splitting: its replays
        # are only valid while they stay current (see __call__)
        self._relies_on_planes = bool(self._plane_caches()) and self._caches_current()
        g = torch.cuda.CUDAGraph()
        # from now on buffers the engine replaces stay alive: this graph replays into their addresses
        eng.graph_retain = True
        eng.bufs.retain = True
        torch.cuda.synchronize(eng.device)
        # thread_local: only this thread's unsafe API calls invalidate the capture - not the RCCL process group's
        # watchdog thread, which polls the events of earlier (eager) collectives while a step is being captured
        with torch.cuda.graph(g, pool=pool, stream=self.stream, capture_error_mode="thread_local"):
            res = eng.run(win, start, batch_size, train=True, global_batch=global_batch)
        # whether the captured step keeps the weight planes current (the one-launch small-batch step
        # does not write them: its replays must leave the caches invalid, as the eager step does)
        self._planes_current = all(c.token is not None for c, _ in self._plane_caches())
        # capture recorded but did not execute the step: restore the host-side state
        eng.global_step, eng.optimizer.steps, eng.flat.grads_zero = gs, steps, zero
        eng.flat.param_epoch = epoch
        for (c, _), t in zip(self._plane_caches(), tokens):
            c.token = t
        return g, res

    def _capture(self, dataset, start: int, batch_size: int, global_batch: Optional[int]):
        if self.direct:  # the graph reads the dataset's own slices: keyed by (dataset, start), holds the dataset
            g, res = self._record(dataset, start, batch_size, global_batch, self.pool)
            if self.pool is None:
                self.pool = g.pool()
            self.engine.flat.grads_zero = True
            return g, dataset, res, start, self._planes_current, self._relies_on_planes
        win = _StaticWindow(dataset)
        g, _ = self._record(win, start, batch_size, global_batch, None)  # discover the data slices
        del g
        win.freeze()
        g, res = self._record(win, start, batch_size, global_batch, self.pool)
        if self.pool is None:
            self.pool = g.pool()
        # the graph ends with the optimizer's fused zero_grad, like the eager step
        self.engine.flat.grads_zero = True
        return g, win, res, start, self._planes_current, self._relies_on_planes

    def _eager(self, dataset, start, batch_size, global_batch):
        cur = torch.cuda.current_stream(self.engine.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            res = self.engine.run(dataset, start, batch_size, train=True, global_batch=global_batch)
        cur.wait_stream(self.stream)
        return res

    def __call__(self, dataset, start: int, batch_size: int, global_batch: Optional[int] = None) -> StepResult:
        eng = self.engine
        if self.disabled or eng.optimizer.steps == 0:
            return self._eager(dataset, start, batch_size, global_batch)
        key = (batch_size, global_batch) + ((id(dataset), start) if self.direct else ())
        t0 = time.perf_counter()
        if any(gr[5] for gr in self.graphs.values()) and not self._caches_current():
            # weights changed outside the captured step: graphs that read the cached weight planes would
            # use stale ones. Drop them; this step runs eagerly (re-splitting) and the next one recaptures.
            self.graphs = {k: gr for k, gr in self.graphs.items() if not gr[5]}
            return self._eager(dataset, start, batch_size, global_batch)
        if key not in self.graphs and self.direct and len(self.graphs) >= self.max_direct:
            self.eager_steps += 1
            return self._eager(dataset, start, batch_size, global_batch)
        if key not in self.graphs:
            try:
                self.graphs[key] = self._capture(dataset, start, batch_size, global_batch)
            except Exception as e:  # noqa: BLE001 - any capture failure: run eagerly from now on
                warnings.warn(f"hipGraph capture failed ({type(e).__name__}: {e}); running eagerly")
                self.disabled = True
                torch.cuda.synchronize(eng.device)
                return self._eager(dataset, start, batch_size, global_batch)
        g, win, res, cap_start, planes_current, _ = self.graphs[key]
        if not self.direct:
            win.load(dataset, start - cap_start)
        g.replay()
        eng.global_step += 1
        # the captured step's update: steps, epoch, cache tokens
        eng.optimizer.commit_fused(zero_grad=True, planes_current=planes_current)
        self.replays += 1
        return StepResult(res.loss_sum, res.correct, res.count, time.perf_counter() - t0)
