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
    with contextlib.redirect_stdout(buf):
        bench.main()
    return buf.getvalue()


def _run(world, extra=()):
    outs = run_ranks(_bench_worker, world, ["--gpus", str(world), "--steps", "2", "--warmup", "1", *extra],
                     timeout=300)
    lines = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and all(not o.strip() for o in outs[1:])
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == world * 256 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["final_loss"] is not None and d["final_loss"] == d["final_loss"]  # finite
    assert d["config"]["world_size_seen"] == world and d["config"]["backend"] == "gloo"
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


def test_bench_two_ranks_measures_the_reference_placement():
    """At N = 2 (the reference's world size) the JSON also carries a measured pp2dp step (stage 0 | stage 1 on
    the two ranks, Chimera, factored boundary gradient: 512 + 40 B per row over the link)."""
    d = _run(2)
    alt = d["config"]["measured_alternatives"]["pp2dp"]
    assert "error" not in alt, alt
    assert alt["samples_per_s"] > 0 and alt["boundary_bytes_across_gpus_per_step"] == 2 * 256 * (512 + 40)
