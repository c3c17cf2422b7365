"""The R > 1 device paths of the engine on ONE MI355X: 2 and 4 processes share ``cuda:0`` and run
every kernel of the real device engine, exchanging boundary tensors and gradients through the
host-staged transport (parallel/p2p.py; RCCL refuses two ranks on one GPU). Only the transport
differs from a multi-GPU run: the orchestration (rotate waves, factored and whole boundary
gradients, the uint8 first layer fed by a received factor, classic neighbour pipelines, dp x pp
gradient all-reduce) is the code the 8-GPU benchmark executes. Each run must train to the weights of
the single-process GPU engine on the same data (reference cut: /root/reference/simple_distributed.py
:47-49, :71, :112)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from dist_util import free_port, run_ranks
from dist_workers import train_worker

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPU = {"device": "cuda:0", "transport": "host"}


def _single(model, M, steps, B, kind, kw=None):
    kw = dict(kw or {}, device="cuda:0")
    return train_worker(0, 1, model, kind, M, 1, steps, B, 3, kw)


def _compare(results, ref, rtol=1e-4, atol=1e-5):
    seen = {}
    for r in results:
        assert r["transport"] == "host"
        for s, sd in r["state"].items():
            for k, v in sd.items():
                if (s, k) in seen:  # replicas agree exactly (same all-reduced gradients)
                    torch.testing.assert_close(v, seen[(s, k)], rtol=0, atol=0)
                seen[(s, k)] = v
                torch.testing.assert_close(v, ref["state"][s][k], rtol=rtol, atol=atol, msg=f"stage {s} {k}")
    for a, b in zip(results[0]["losses"], ref["losses"]):
        assert a == pytest.approx(b, rel=1e-4, abs=1e-6)
    assert results[0]["eval"][2] == ref["eval"][2]


@pytest.mark.parametrize("world,mode", [(2, "factored"), (4, "factored"), (2, "whole_grad"), (2, "u8"),
                                        (4, "u8"), (2, "u8_phi"), (2, "u8_dp"), (4, "u8_dp")])
def test_rotate_multirank_on_device(world, mode, monkeypatch):
    """rotate on the device engine at R = 2, 4: factored boundary gradient (the head's dl crosses),
    the whole gradient (SDML_ROTATE_FACTORED=0), and uint8 pixels where the received factor goes
    straight into the first layer's weight-gradient kernel (4096-row waves: the uint8 kernels'
    shapes); u8_phi: a quarter of each wave crosses (balanced placement); u8_dp: nothing crosses
    (cross_fraction 0, the placement the N > 1 benchmark picks): the fused forward+head kernel, the
    deferred head reduction inside the weight-gradient reduction, the gradient all-reduce and the
    unfused SGD, at the uint8 kernels' shapes."""
    kw = dict(GPU)
    steps, M = 2, 2 * world
    B = 48
    if mode == "whole_grad":
        monkeypatch.setenv("SDML_ROTATE_FACTORED", "0")
    if mode.startswith("u8"):
        kw["pixels"] = "u8"
        B = 8192
    if mode == "u8_phi":
        kw["cross_fraction"] = 0.25
    if mode == "u8_dp":
        kw["cross_fraction"] = 0.0
        kw["dp_split"] = True  # the opt-in split all-reduce (parity of both weight-gradient ranges)
        M = world  # one wave per rank, as bench.py runs dp
    res = run_ranks(train_worker, world, "mlp", "rotate", M, world, steps, B, 3, kw, timeout=400)
    ref = _single("mlp", M, steps, world * B, "rotate", {"pixels": kw.get("pixels", "f32")})
    _compare(res, ref)
    assert all((r["bytes_sent"] > 0) == (mode != "u8_dp") for r in res)
    if mode == "u8_dp":  # the gradient all-reduce split over two weight-gradient ranges (GradSync.issue_span)
        assert all(r["dp_split_steps"] == steps for r in res)
    assert all(r["pool_allocs"] == r["pool_allocs_first"] for r in res)  # persistent boundary buffers


@pytest.mark.parametrize("kind,world,pp,M", [("1f1b", 2, 2, 3), ("chimera", 2, 2, 4), ("1f1b", 4, 2, 2)])
def test_neighbour_pipelines_on_device(kind, world, pp, M):
    """The reference's placement (stage 0 | stage 1 on different ranks, isend/irecv), with 1F1B,
    Chimera, and dp2 x pp2 (gradient all-reduce between the replicas)."""
    B, steps = 64, 2
    dp = world // pp
    res = run_ranks(train_worker, world, "mlp", kind, M, pp, steps, B, 3, dict(GPU), timeout=400)
    ref = _single("mlp", M, steps, dp * B, kind)
    _compare(res, ref)
    assert all(r["bytes_sent"] > 0 for r in res)
    assert all(r["pool_allocs"] == r["pool_allocs_first"] for r in res)


def _bench_json(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_on_one_gpu():
    """bench.py exactly as the driver launches it for N = 2 (torch.distributed.run, one rank per
    process), its ranks sharing the GPU through the host-staged transport: one JSON line, the
    placement's measured boundary bytes, the rank count the process group saw."""
    env = dict(os.environ, SDML_TRANSPORT="host", SDML_BENCH_BATCH="8192", PYTHONPATH=ROOT)
    for place, cross in (("rotate", True), ("auto", None)):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
               "--gpus", "2", "--steps", "3", "--warmup", "1", "--placement", place]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        d = _bench_json(r)
        assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["transport"] == "host"
        assert d["config"]["world_size_seen"] == 2 and d["config"]["backend"] == "gloo"
        if cross:
            assert d["config"]["boundary_bytes_across_gpus_per_step"] == 2 * 4096 * (512 + 40)


def test_bench_spawns_its_ranks_without_a_launcher():
    """``python bench.py --gpus 2`` with no WORLD_SIZE in the environment starts its own two ranks
    (before touching the GPU) instead of silently running one: n_gpus and world_size_seen are 2."""
    env = dict(os.environ, SDML_TRANSPORT="host", SDML_BENCH_BATCH="8192", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = _bench_json(r)
    assert d["n_gpus"] == 2 and d["config"]["world_size_seen"] == 2 and d["value"] > 0
    # a launcher/flag mismatch is fatal, not a relabelled 1-rank run
    env1 = dict(env, WORLD_SIZE="1", RANK="0")
    r = subprocess.run(cmd, env=env1, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode != 0 and not [l for l in r.stdout.splitlines() if l.startswith("{")]
