"""Pre-tuned hipBLASLt solutions for the library GEMMs (PyTorch TunableOp).

The GPT-2 stages run their projection GEMMs through hipBLASLt (plain library GEMMs, no
fused epilogues of ours). hipBLASLt's default heuristic choice is not always its fastest
solution at these shapes (M = micro-batch tokens, K/N = 768 / 2304 / 3072 / 50257). TunableOp
benchmarks every candidate solution once. The winners for one MI355X (gfx950, this image's
hipBLASLt) are committed in ``tuning/gemm_gpt2_mi355x.csv``; this module loads them with
tuning disabled, so no benchmarking happens at run time. TunableOp's validators reject the
file on a different PyTorch / hipBLASLt / architecture, and the heuristic choice is used then.
Measured: GPT-2 2-stage step on one GPU +3 % (424K -> 438K tokens/s).

Re-tune: ``PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1
PYTORCH_TUNABLEOP_FILENAME=out.csv python tools/bench_configs.py --config gpt2`` (the device
index is appended to the file name).
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

DEFAULT = Path(__file__).resolve().parent.parent / "tuning" / "gemm_gpt2_mi355x.csv"


def use_tuned_gemms(path=None) -> bool:
    """Enable TunableOp in replay-only mode with the committed results. Returns True when enabled."""
    if os.environ.get("SDML_TUNED_GEMMS", "1") == "0" or not torch.cuda.is_available():
        return False
    if os.environ.get("PYTORCH_TUNABLEOP_ENABLED") is not None:  # the user drives TunableOp
        return False
    p = Path(path) if path else DEFAULT
    if not p.exists():
        return False
    try:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(False)
        torch.cuda.tunable.record_untuned_enable(False)
        return bool(torch.cuda.tunable.read_file(str(p)))
    except Exception:  # noqa: BLE001 - an optional optimisation: never fail the run for it
        torch.cuda.tunable.enable(False)
        return False
