"""Model registry: name -> ModelSpec (a model cut into pipeline stages)."""
from __future__ import annotations

from .base import ModelSpec, PipelineStage, build_stages, stage_seed
from .gpt2 import GPT2Config, gpt2_spec
from .mlp import MLP4X1024_DIMS, MLP_DIMS, MLPStage, mlp_spec
from .ref_cnn import Network1Stage, Network2Stage, ref_cnn_spec
from .resnet import resnet18_spec

MODELS = ("mlp", "mlp4x1024", "ref_cnn", "resnet18", "gpt2", "gpt2_tiny")

DEFAULT_STAGES = {"mlp": 2, "mlp4x1024": 4, "ref_cnn": 2, "resnet18": 8, "gpt2": 2, "gpt2_tiny": 2}


def get_model_spec(name: str, num_stages: int = None, **kw) -> ModelSpec:
    n = num_stages or DEFAULT_STAGES[name]
    if name == "mlp":
        return mlp_spec(MLP_DIMS, n, "mlp")
    if name == "mlp4x1024":
        return mlp_spec(MLP4X1024_DIMS, n, "mlp4x1024")
    if name == "ref_cnn":
        return ref_cnn_spec(n, eval_dropout=kw.get("eval_dropout", True), dropout=kw.get("dropout", 0.5))
    if name == "resnet18":
        return resnet18_spec(n, dtype=kw.get("dtype", None) or __import__("torch").float32)
    if name == "gpt2":
        return gpt2_spec(n, seq_len=kw.get("seq_len"))
    if name == "gpt2_tiny":  # test-sized transformer with the same code path
        cfg = GPT2Config(n_layer=2 * n, n_head=2, n_embd=32, vocab_size=97, block_size=32)
        return gpt2_spec(n, cfg=cfg, seq_len=kw.get("seq_len") or 16,
                         dtype=kw.get("dtype", None) or __import__("torch").float32, name="gpt2_tiny")
    raise ValueError(f"unknown model {name!r}; choose from {MODELS}")


__all__ = ["ModelSpec", "PipelineStage", "build_stages", "stage_seed", "get_model_spec", "MODELS",
           "DEFAULT_STAGES", "MLPStage", "Network1Stage", "Network2Stage", "GPT2Config"]
