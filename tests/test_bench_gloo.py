"""bench.py's multi-rank path (rotate schedule, all-to-all stage boundary, sharded synthetic data,
MAX-over-ranks timing, one JSON line from rank 0) rehearsed on Gloo/CPU with 4 ranks."""
import contextlib
import io
import json
import os
import sys

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


def test_bench_rotate_four_ranks_one_json_line():
    outs = run_ranks(_bench_worker, 4, ["--gpus", "4", "--steps", "2", "--warmup", "1"], timeout=300)
    lines = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and all(not o.strip() for o in outs[1:])
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 4 * 256 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["final_loss"] is not None and d["final_loss"] == d["final_loss"]  # finite
