"""bench.py's multi-rank paths (every placement, sharded synthetic data, MAX-over-ranks timing, the
measured boundary bytes, one JSON line from rank 0) rehearsed on Gloo/CPU with 2 and 4 ranks."""
import contextlib
import io
import json
import os
import sys

import pytest

from dist_util import run_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_worker(rank, world, argv):
    sys.path.insert(0, ROOT)
    os.environ["SDML_BENCH_BATCH"] = "256"
    import bench

    sys.argv = ["bench.py"] + list(argv)
    buf = io.StringIO()
    code = 0
    with contextlib.redirect_stdout(buf):
        try:
            bench.main()
        except SystemExit as e:  # bench.py exits non-zero on a failed self-check
            code = e.code
    return buf.getvalue() + (f"\n__EXIT__={code}" if code else "")


def _run(world, extra=()):
    outs = run_ranks(_bench_worker, world, ["--gpus", str(world), "--steps", "2", "--warmup", "1", *extra],
                     timeout=300)
    exits = [o.split("__EXIT__=")[1].strip() for o in outs if "__EXIT__=" in o]
    if exits:
        raise RuntimeError(f"bench exited {exits}")
    lines = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and all(not o.strip() for o in outs[1:])
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == world * 256 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["final_loss"] is not None and d["final_loss"] == d["final_loss"]  # finite
    assert d["config"]["world_size_seen"] == world and d["config"]["backend"] == "gloo"
    # self-checks of a multi-rank run: replicas bit-identical after the timed steps, links measured before the
    # placement was chosen (and the measured model is the one the JSON reports)
    assert d["config"]["replicas_identical"] is True, d["config"]["replica_check"]
    lm = d["config"]["link_measured"]
    assert lm["world_size"] == world and lm["allreduce_us"] > 0 and lm["collective_us"] > 0 and lm["gbps"] > 0
    assert d["config"]["link_model"]["link"]["gbps"] == lm["gbps"]
    assert d["config"]["link_model"]["link"]["allreduce_us"] == lm["allreduce_us"]
    assert d["config"]["link_model_assumed"]["gbps"] == 50.0
    return d


@pytest.mark.parametrize("placement", ["auto", "rotate", "balanced", "pp2dp"])
def test_bench_four_ranks_one_json_line(placement):
    d = _run(4, ["--placement", placement])
    c = d["config"]
    assert set(c["predicted"]) >= {"rotate", "dp", "balanced", "pp2dp"}
    assert c["placement"] == (placement if placement != "auto" else c["placement"])
    rows = 256
    if c["placement"] == "rotate":  # 3/4 of every owner's rows cross: 512 B forward + 40 B back each
        assert c["boundary_bytes_across_gpus_per_step"] == 4 * (rows - rows // 4) * (512 + 40)
    if c["placement"] == "dp":
        assert c["boundary_bytes_across_gpus_per_step"] == 0
    if c["placement"] == "pp2dp":  # every row's activation and its factored gradient (dl, 10 fp32) cross the link
        assert c["boundary_bytes_across_gpus_per_step"] == 4 * rows * (512 + 40)


def test_bench_two_ranks_cross_fraction_override():
    d = _run(2, ["--placement", "rotate", "--cross_fraction", "0.25"])
    assert d["config"]["boundary_bytes_across_gpus_per_step"] == 2 * 64 * (512 + 40)


def test_bench_gpus_flag_spawns_ranks_on_cpu(tmp_path):
    """No launcher: ``bench.py --gpus 2`` starts 2 ranks itself; a WORLD_SIZE/--gpus mismatch exits
    non-zero without printing a result."""
    import subprocess

    env = dict(os.environ, SDML_BENCH_BATCH="256", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["world_size_seen"] == 2
    r = subprocess.run(cmd, env=dict(env, WORLD_SIZE="1", RANK="0"), capture_output=True, text=True, timeout=120,
                       cwd=str(tmp_path))
    assert r.returncode == 2 and not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("world", [2, 4])
def test_bench_measures_the_reference_placement_at_every_even_n(world):
    """At every even N the JSON also carries a measured pp2dp step (stage 0 | stage 1 on the GPUs of each pair,
    Chimera, factored boundary gradient: 512 + 40 B per row over the link), next to the placement the measured
    link model chose."""
    d = _run(world, ["--placement", "dp"])
    alt = d["config"]["measured_alternatives"]["pp2dp"]
    assert "error" not in alt, alt
    assert alt["samples_per_s"] > 0 and alt["boundary_bytes_across_gpus_per_step"] == world * 256 * (512 + 40)


def test_bench_exits_nonzero_when_replicas_diverge():
    """A test hook flips one parameter bit on rank 1 after the timed steps: the replica check must see it, report
    replicas_identical = false and make bench.py exit non-zero (3)."""
    os.environ["SDML_BENCH_PERTURB_RANK"] = "1"
    try:
        with pytest.raises(RuntimeError, match=r"bench exited \['3', '3'\]"):
            _run(2, ["--placement", "dp", "--alternatives", "off"])
    finally:
        os.environ.pop("SDML_BENCH_PERTURB_RANK", None)
