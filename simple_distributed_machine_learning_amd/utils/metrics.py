"""Logging + metrics.

* :func:`train_line` / :func:`test_line` reproduce the reference's print format byte for byte
  (/root/reference/simple_distributed.py:114-117 and :129-132).
* :class:`JsonlMetrics` appends one JSON object per event (samples/s, step ms, losses,
  per-phase timings) — the machine-readable stream the reference lacks.
* :class:`StepTimer` brackets device work with HIP events (no host sync until read).
"""
from __future__ import annotations

import json
import time
from pathlib import Path
from typing import Optional

import torch


def train_line(epoch: int, batch_idx: int, batch_len: int, dataset_len: int, num_batches: int, loss: float) -> str:
    return 'Train Epoch: {} [{}/{} ({:.0f}%)]\tLoss: {:.6f}'.format(
        epoch, batch_idx * batch_len, dataset_len, 100. * batch_idx / num_batches, loss)


def test_line(avg_loss: float, correct: int, n: int) -> str:
    return '\nTest set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n'.format(
        avg_loss, correct, n, 100.0 * correct / n)


class JsonlMetrics:
    def __init__(self, path: Optional[str], rank: int = 0):
        self.path = Path(path) if path else None
        self.rank = rank
        if self.path:
            self.path.parent.mkdir(parents=True, exist_ok=True)

    def log(self, **kv):
        if not self.path:
            return
        kv.setdefault("time", time.time())
        kv.setdefault("rank", self.rank)
        with open(self.path, "a") as f:
            f.write(json.dumps(kv, default=float) + "\n")


class StepTimer:
    """Device-side interval timer: HIP events on ROCm, perf_counter on CPU."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self._t0 = None
        self._e0 = self._e1 = None

    def start(self):
        if self.cuda:
            self._e0 = torch.cuda.Event(enable_timing=True)
            self._e1 = torch.cuda.Event(enable_timing=True)
            self._e0.record()
        else:
            self._t0 = time.perf_counter()

    def stop_ms(self) -> float:
        if self.cuda:
            self._e1.record()
            self._e1.synchronize()
            return self._e0.elapsed_time(self._e1)
        return (time.perf_counter() - self._t0) * 1e3
