"""End-to-end: the reference's command line, two processes on 127.0.0.1, reference log format."""
import os
import re
import subprocess
import sys

import pytest

from dist_util import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow

TRAIN_RE = re.compile(r"^Train Epoch: (\d+) \[(\d+)/(\d+) \((\d+)%\)\]\tLoss: (\d+\.\d{6})$")
TEST_RE = re.compile(r"^Test set: Average loss: (\d+\.\d{4}), Accuracy: (\d+)/(\d+) \((\d+)%\)$")


def _launch(extra, world=2):
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    procs = []
    for r in range(world):
        cmd = [sys.executable, os.path.join(ROOT, "simple_distributed.py"), f"--rank={r}", f"--world_size={world}",
               "--interface=lo", "--master_addr=127.0.0.1", f"--master_port={port}", "--device=cpu"] + extra
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=300)
        outs.append(out)
        assert p.returncode == 0, out
    return outs


def test_reference_command_line_two_ranks(tmp_path):
    outs = _launch(["--epochs=2", "--train_size=1200", "--test_size=200", f"--ckpt_dir={tmp_path}",
                    f"--metrics={tmp_path}/m.jsonl"])
    lines = outs[0].splitlines()
    train = [m for m in map(TRAIN_RE.match, lines) if m]
    test = [m for m in map(TEST_RE.match, lines) if m]
    # 1200/60 = 20 batches -> logs at batch 0 and 10, per epoch
    assert [(m.group(1), m.group(2), m.group(3), m.group(4)) for m in train] == [
        ("1", "0", "1200", "0"), ("1", "600", "1200", "50"), ("2", "0", "1200", "0"), ("2", "600", "1200", "50")]
    assert len(test) == 2 and all(m.group(3) == "200" for m in test)
    # the blank lines around the test line, exactly like the reference's '\n...\n'
    i = lines.index(test[0].group(0))
    assert lines[i - 1] == "" and lines[i + 1] == ""
    # rank 1 prints no training lines (master-only logging)
    assert not any(TRAIN_RE.match(l) for l in outs[1].splitlines())
    # checkpoint written by the stage owners with reference key names
    assert (tmp_path / "stage0.pt").exists() and (tmp_path / "stage1.pt").exists()
    assert (tmp_path / "m.jsonl").read_text().count('"event": "train"') == 4
    # resume: continues after the saved epoch (nothing left to do at --epochs=2)
    outs = _launch(["--epochs=3", "--train_size=1200", "--test_size=200", f"--ckpt_dir={tmp_path}", "--resume"])
    assert "resumed from" in outs[0]
    assert sum(1 for l in outs[0].splitlines() if TRAIN_RE.match(l)) == 2  # only epoch 3


def test_timing_metrics_two_ranks(tmp_path):
    # --timing: per-stage/phase times of the logged steps land in the JSONL metrics
    import json

    _launch(["--epochs=1", "--train_size=240", "--test_size=60", "--model=mlp", "--timing", "--no_test",
             f"--metrics={tmp_path}/m.jsonl"])
    recs = [json.loads(l) for l in open(f"{tmp_path}/m.jsonl")]
    t = [r["timing_ms"] for r in recs if r.get("event") == "train"]
    assert t and all(v >= 0 for v in t[0].values())
    # rank 0 holds stage 0 of the 2-stage pipeline: forward, backward, the wait for stage 1's gradient
    assert {"fwd/stage0", "bwd/stage0", "recv_wait/stage1", "optim"} <= set(t[0])
