"""Logging + metrics.

* :func:`train_line` / :func:`test_line` reproduce the reference's print format byte for byte
  (/root/reference/simple_distributed.py:114-117 and :129-132).
* :class:`JsonlMetrics` appends one JSON object per event (samples/s, step ms, losses,
  per-phase timings) — the machine-readable stream the reference lacks.
(Per-phase device timing lives in utils/timing.py's PhaseTimer.)
"""
from __future__ import annotations

import json
import time
from pathlib import Path
from typing import Optional


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

