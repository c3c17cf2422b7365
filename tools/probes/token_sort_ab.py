"""Embedding backward's stable token sort: int64 stable torch.sort vs the packed int32 key sort (ops/transformer.py)."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())


def _stable_token_sort(tok, vocab: int):  # the rejected variant (was ops/transformer.py), kept here for the record
    n = tok.numel()
    p = max(1, (n - 1).bit_length())
    key = (tok.to(torch.int32) << p) | torch.arange(n, device=tok.device, dtype=torch.int32)
    key = torch.sort(key).values
    return (key >> p).to(tok.dtype), (key & ((1 << p) - 1)).to(torch.int64)


t = torch.randint(0, 50257, (16, 1024), device="cuda").reshape(-1)


def timeit(fn, it=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / it * 1e3, 1)


a, pa = _stable_token_sort(t, 50257)
b, pb = torch.sort(t, stable=True)
assert torch.equal(a, b) and torch.equal(pa, pb)
for r in range(3):
    print({"int64_stable_us": timeit(lambda: torch.sort(t, stable=True)), "packed_int32_us": timeit(lambda: _stable_token_sort(t, 50257))})
