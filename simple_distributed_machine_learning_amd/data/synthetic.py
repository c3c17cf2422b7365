"""On-device datasets.

The reference downloads MNIST with torchvision, keeps the first 1/10 of each split and
iterates it unshuffled in batches of 60 (/root/reference/simple_distributed.py:87-95).
Neither the network nor torchvision exists here, so:

* :class:`SyntheticMNIST` — counter-based, seed-deterministic MNIST-shape data
  ([N,1,28,28] float32 in [0,1], int64 labels in [0,10)), generated directly in HBM by a
  HIP kernel (or on the host by the bit-identical C++ twin). Every rank builds the same
  dataset locally, so labels never cross the wire. ``pixels="u8"`` stores the images the way
  MNIST ships them, as uint8 bytes k = round(255 x); ``ToTensor()`` (k / 255) is then applied
  by the consuming stage (fused into the first GEMM for the MLPs, ``ops.pixels_to_float``
  otherwise), which reads a quarter of the bytes.
* :class:`IdxMNIST` — reads real MNIST ``*-idx?-ubyte`` files if the user has them locally
  (no download), ``ToTensor()`` scaling like the reference.
* :class:`SyntheticTokens` — GPT-2 style token sequences for the transformer configs.
* :func:`batch_ranges` — the reference's DataLoader order: sequential, no shuffle,
  ``drop_last=False``.
"""
from __future__ import annotations

import gzip
import os
from pathlib import Path
from typing import Iterator, Optional, Tuple

import torch

from .._native import runtime


class Dataset:
    n: int

    def inputs(self, start: int, n: int) -> torch.Tensor:
        raise NotImplementedError

    def targets(self, start: int, n: int) -> torch.Tensor:
        raise NotImplementedError

    def __len__(self):
        return self.n


class SyntheticMNIST(Dataset):
    H = W = 28

    def __init__(self, n: int, seed: int = 1234, device="cpu", mode: str = "learnable", offset: int = 0,
                 image_range=None, pixels: str = "f32"):
        """``image_range=(lo, hi)``: materialise images only for samples [lo, hi) (labels for
        all n) — a rank that runs stage 0 only on its own shard needs no other images."""
        self.n = int(n)
        self.seed = int(seed)
        self.device = torch.device(device)
        self.mode = {"learnable": 0, "random": 1}[mode]
        self.offset = int(offset)  # sample-id offset (train/test splits use disjoint ids)
        self.lo, self.hi = (0, self.n) if image_range is None else (int(image_range[0]), int(image_range[1]))
        self.x = torch.empty((self.hi - self.lo, 1, self.H, self.W), dtype=torch.float32, device=self.device)
        self.y = torch.empty((self.n,), dtype=torch.int64, device=self.device)
        if self.n:
            self._fill()
        if pixels == "u8":
            # MNIST's storage format: bytes k = round(255 x) (deterministic fp32 ops: the same
            # bytes on every device); the float32 view of a sample is k / 255 (ToTensor)
            self.x = self.x.mul_(255.0).round_().to(torch.uint8)
        elif pixels != "f32":
            raise ValueError(f"pixels must be 'f32' or 'u8', got {pixels!r}")

    def _fill(self):
        if self.device.type == "cuda":
            from .._native import kernels

            k = kernels()
            if (self.lo, self.hi) == (0, self.n):
                k.synth_mnist(self.seed, self.offset, self.n, self.H, self.W, self.mode, self.x, self.y)
            else:
                scratch = torch.empty((self.n, 1, 1, 1), dtype=torch.float32, device=self.device)
                k.synth_mnist(self.seed, self.offset, self.n, 1, 1, self.mode, scratch, self.y)  # labels only
                ylo = torch.empty((self.hi - self.lo,), dtype=torch.int64, device=self.device)
                k.synth_mnist(self.seed, self.offset + self.lo, self.hi - self.lo, self.H, self.W, self.mode, self.x, ylo)
        else:
            rt = runtime()
            rt.synth_fill(self.seed, self.offset, self.n, self.H, self.W, self.mode, 0, self.y.data_ptr())
            rt.synth_fill(self.seed, self.offset + self.lo, self.hi - self.lo, self.H, self.W, self.mode,
                          self.x.data_ptr(), 0)

    def inputs(self, start, n):
        if start < self.lo or start + n > self.hi:
            raise IndexError(f"images [{start}, {start + n}) not materialised on this rank "
                             f"(have [{self.lo}, {self.hi}))")
        return self.x[start - self.lo:start - self.lo + n]

    def targets(self, start, n):
        return self.y[start:start + n]


def _read_idx(path: Path) -> torch.Tensor:
    op = gzip.open if path.suffix == ".gz" else open
    with op(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    ndim = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(ndim)]
    off = 4 + 4 * ndim
    t = torch.frombuffer(bytearray(data[off:]), dtype=torch.uint8)
    return t.reshape(dims)


class IdxMNIST(Dataset):
    """Real MNIST from local idx files; ``fraction`` mirrors the reference's ``len//10`` subset."""

    FILES = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
             False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}

    def __init__(self, root: str, train: bool, device="cpu", fraction: float = 0.1, pixels: str = "f32"):
        root = Path(root)
        img_name, lbl_name = self.FILES[train]

        def find(name):
            for cand in (root / name, root / (name + ".gz"), root / "MNIST" / "raw" / name,
                         root / "MNIST" / "raw" / (name + ".gz")):
                if cand.exists():
                    return cand
            raise FileNotFoundError(f"{name} not found under {root}")

        x = _read_idx(find(img_name)).unsqueeze(1)  # uint8, as stored
        if pixels == "f32":
            x = x.float().div_(255.0)  # ToTensor()
        elif pixels != "u8":
            raise ValueError(f"pixels must be 'f32' or 'u8', got {pixels!r}")
        y = _read_idx(find(lbl_name)).long()
        n = int(len(x) * fraction) if fraction < 1 else len(x)
        self.n = n
        self.x = x[:n].contiguous().to(device)
        self.y = y[:n].contiguous().to(device)

    def inputs(self, start, n):
        return self.x[start:start + n]

    def targets(self, start, n):
        return self.y[start:start + n]

    @staticmethod
    def available(root: Optional[str]) -> bool:
        if not root:
            return False
        try:
            IdxMNIST.FILES  # noqa: B018
            for name in IdxMNIST.FILES[True] + IdxMNIST.FILES[False]:
                ok = any(p.exists() for p in (Path(root) / name, Path(root) / (name + ".gz"),
                                              Path(root) / "MNIST" / "raw" / name))
                if not ok:
                    return False
            return True
        except Exception:  # noqa: BLE001
            return False


class SyntheticTokens(Dataset):
    """Token sequences: inputs [n, S] and next-token targets [n, S] (int64).

    Sequences follow a seeded first-order pattern (token_{t+1} = (a*token_t + b) mod V with
    probability 0.9, random otherwise) so a language model has something learnable.
    """

    def __init__(self, n: int, seq_len: int, vocab: int, seed: int = 1234, device="cpu"):
        self.n, self.seq_len, self.vocab = int(n), int(seq_len), int(vocab)
        g = torch.Generator().manual_seed(seed)
        a = 48271 % vocab or 1
        b = 12345 % vocab
        toks = torch.empty((self.n, self.seq_len + 1), dtype=torch.int64)
        toks[:, 0] = torch.randint(0, vocab, (self.n,), generator=g)
        noise = torch.rand((self.n, self.seq_len), generator=g) < 0.1
        rnd = torch.randint(0, vocab, (self.n, self.seq_len), generator=g)
        for t in range(self.seq_len):
            nxt = (toks[:, t] * a + b) % vocab
            toks[:, t + 1] = torch.where(noise[:, t], rnd[:, t], nxt)
        self.tokens = toks.to(device)

    def inputs(self, start, n):
        return self.tokens[start:start + n, :-1]

    def targets(self, start, n):
        return self.tokens[start:start + n, 1:]


def batch_ranges(n: int, batch_size: int, start_batch: int = 0) -> Iterator[Tuple[int, int, int]]:
    """(batch_idx, start, size) in DataLoader order: sequential, no shuffle, keep the tail."""
    nb = (n + batch_size - 1) // batch_size
    for i in range(start_batch, nb):
        s = i * batch_size
        yield i, s, min(batch_size, n - s)
