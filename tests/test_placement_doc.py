"""README's multi-GPU placement table is the cost model's own output (parallel/placement.py markdown_table), and the
model prices the path the engine runs (the dp split only when SDML_DP_SPLIT says the engine splits)."""
import os

from simple_distributed_machine_learning_amd.parallel import placement as plc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_readme_table_is_the_model_output(monkeypatch):
    monkeypatch.delenv("SDML_DP_SPLIT", raising=False)
    with open(os.path.join(ROOT, "README.md")) as f:
        readme = f.read()
    assert plc.markdown_table() in readme


def test_split_priced_only_when_the_engine_splits(monkeypatch):
    monkeypatch.delenv("SDML_DP_SPLIT", raising=False)
    off = plc.predict("dp", 8, 131072)
    monkeypatch.setenv("SDML_DP_SPLIT", "1")
    on = plc.predict("dp", 8, 131072)
    c = plc.ComputeModel()
    assert off["allreduce_ms"] != on["allreduce_ms"]
    # the default path: the whole all-reduce exposed plus the separate optimizer launch, replayed from a HIP graph
    # (bench.py's dp step at N > 1); eager, the cross-stream hand-offs cost dp_step_us instead
    link = plc.LinkModel()
    ar = 2 * 7 / 8 * c.param_bytes / (2 * link.gbps * 1e3) + link.collective_us
    assert abs(off["allreduce_ms"] - round((ar + c.dp_graph_step_us) / 1e3, 4)) < 1e-4
    monkeypatch.delenv("SDML_DP_SPLIT", raising=False)
    eager = plc.predict("dp", 8, 131072, graph=False)
    assert abs(eager["allreduce_ms"] - round((ar + c.dp_step_us) / 1e3, 4)) < 1e-4


def test_bench_graph_default_matches_the_model():
    """bench.py replays the dp step from a HIP graph at N > 1 over RCCL (not split); the model prices that path."""
    import pathlib
    import re

    src = pathlib.Path(__file__).resolve().parents[1].joinpath("bench.py").read_text()
    assert re.search(r'a\.graph == "auto" and world > 1 and place == "dp" and rccl and not engine\.dp_split', src)


def test_one_gpu_prediction_matches_the_fused_step():
    c = plc.ComputeModel()
    p = plc.predict("dp", 1, 131072)
    assert abs(p["step_ms"] - (131072 * c.fused_ns / 1e3 + c.fixed_us) / 1e3) < 1e-3
