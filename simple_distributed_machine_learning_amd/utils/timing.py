"""Per-stage, per-phase step timing (SURVEY.md §5 "tracing": step timers per stage and phase).

The reference has no timers at all (/root/reference/simple_distributed.py:106-117). With
``PipelineEngine(..., timing=True)`` every forward, backward, receive-wait, gradient all-reduce
and optimizer launch of a step is bracketed by a pair of HIP events. The events are recorded
in stream order on the compute stream, so they measure device time. A receive-wait span is
the time the compute stream stalls on data from a peer, not host time. The events are read
once, after the step (one synchronisation, and only when timing is on). On CPU the spans are
host wall time.
"""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager, nullcontext
from typing import Dict

import torch


_NULL = nullcontext()


class PhaseTimer:
    def __init__(self, device: torch.device, enabled: bool):
        self.enabled = enabled
        self.cuda = enabled and device.type == "cuda"
        self.device = device
        self._spans = []  # (key, start, end)

    def span(self, phase: str, stage: int = -1):
        # (timing off, the step's hot path: one shared no-op context instead of a generator per span)
        return self._span(phase, stage) if self.enabled else _NULL

    @contextmanager
    def _span(self, phase: str, stage: int = -1):
        key = phase if stage < 0 else f"{phase}/stage{stage}"
        if self.cuda:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._spans.append((key, a, b))
        else:
            t0 = time.perf_counter()
            yield
            self._spans.append((key, t0, time.perf_counter()))

    def result(self) -> Dict[str, float]:
        """{phase[/stageK]: milliseconds summed over the step} (synchronises on CUDA)."""
        if not self.enabled:
            return {}
        out = defaultdict(float)
        if self.cuda and self._spans:
            self._spans[-1][2].synchronize()
        for key, a, b in self._spans:
            out[key] += a.elapsed_time(b) if self.cuda else (b - a) * 1e3
        self._spans = []
        return {k: round(v, 4) for k, v in sorted(out.items())}
