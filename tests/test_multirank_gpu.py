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


def _compare(results, ref, rtol=1e-4, atol=1e-5, transport="host"):
    seen = {}
    for r in results:
        assert r["transport"] == transport
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


@pytest.mark.parametrize("world", [2, 4])
def test_dp_multirank_ipc_gradient_all_reduce(world):
    """The placement the N > 1 benchmark runs (dp: nothing crosses, the gradient all-reduce is the only collective)
    with the all-reduce device to device between the processes (IpcTransport: every rank sums the members' mapped
    flat-gradient slices in rank order): replicas bit-identical, weights equal to the single-process GPU engine."""
    steps, B = 2, 8192
    kw = dict(GPU, transport="ipc", pixels="u8", cross_fraction=0.0)
    res = run_ranks(train_worker, world, "mlp", "rotate", world, world, steps, B, 3, kw, timeout=400)
    ref = _single("mlp", world, steps, world * B, "rotate", {"pixels": "u8"})
    _compare(res, ref, transport="ipc")
    assert all(r["bytes_sent"] == 0 for r in res)


@pytest.mark.parametrize("world,mode", [(2, "factored"), (4, "u8"), (2, "u8_phi")])
def test_rotate_multirank_ipc_all_to_all(world, mode):
    """The rotate placement with its boundary all-to-alls (and gradient all-reduce) device to device between the
    processes (IpcTransport: one message per peer over the pairwise slot channels, the own part copied locally): the
    same weights as the host-staged run (bit for bit at 2 ranks) and as the single-process GPU engine."""
    runs = {}
    for tr in ("host", "ipc"):
        kw = dict(GPU, transport=tr)
        steps, M, B = 2, 2 * world, 48
        if mode.startswith("u8"):
            kw["pixels"] = "u8"
            B = 8192
        if mode == "u8_phi":
            kw["cross_fraction"] = 0.25
        runs[tr] = run_ranks(train_worker, world, "mlp", "rotate", M, world, steps, B, 3, kw, timeout=400)
    ref = _single("mlp", M, steps, world * B, "rotate", {"pixels": "u8" if mode.startswith("u8") else "f32"})
    _compare(runs["ipc"], ref, transport="ipc")
    assert all(r["bytes_sent"] > 0 for r in runs["ipc"])
    # the boundary bytes are the same bytes; the gradient sum of 2 ranks is one (commutative) add on both transports,
    # of 4 ranks the IPC all-reduce adds in rank order where Gloo's ring adds in its own order (last-bit differences)
    tol = 0 if world == 2 else 1e-6
    for a, b in zip(runs["ipc"], runs["host"]):
        assert a["bytes_sent"] == b["bytes_sent"]
        for s_, sd in a["state"].items():
            for k, v in sd.items():
                torch.testing.assert_close(v, b["state"][s_][k], rtol=tol, atol=tol, msg=f"{s_} {k}")


_NEIGHBOUR = {}


@pytest.mark.parametrize("transport", ["host", "ipc"])
@pytest.mark.parametrize("kind,world,pp,M", [("1f1b", 2, 2, 3), ("chimera", 2, 2, 4), ("1f1b", 4, 2, 2)])
def test_neighbour_pipelines_on_device(kind, world, pp, M, transport):
    """The reference's placement (stage 0 | stage 1 on different ranks, isend/irecv), with 1F1B,
    Chimera, and dp2 x pp2 (gradient all-reduce between the replicas). ``ipc``: the boundary tensors
    go device to device between the processes (hipIPC slots, stream-ordered ready / ack words): the
    trained weights must equal the host-staged run's bit for bit (only the transport differs)."""
    B, steps = 64, 2
    dp = world // pp
    res = run_ranks(train_worker, world, "mlp", kind, M, pp, steps, B, 3, dict(GPU, transport=transport),
                    timeout=400)
    ref = _single("mlp", M, steps, dp * B, kind)
    _compare(res, ref, transport=transport)
    assert all(r["bytes_sent"] > 0 for r in res)
    assert all(r["pool_allocs"] == r["pool_allocs_first"] for r in res)
    _NEIGHBOUR[(kind, world, transport)] = res
    other = _NEIGHBOUR.get((kind, world, "host" if transport == "ipc" else "ipc"))
    if other is not None:  # both transports ran: identical bytes delivered -> identical training
        for a, b in zip(res, other):
            for s, sd in a["state"].items():
                for k, v in sd.items():
                    torch.testing.assert_close(v, b["state"][s][k], rtol=0, atol=0, msg=f"{transport} {s} {k}")


def _bench_json(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_on_one_gpu():
    """bench.py exactly as the driver launches it for N = 2 (torch.distributed.run, one rank per
    process), its ranks sharing the GPU through the host-staged transport: one JSON line, the
    placement's measured boundary bytes, the rank count the process group saw."""
    env = dict(os.environ, SDML_TRANSPORT="host", SDML_BENCH_BATCH="8192", PYTHONPATH=ROOT)
    for place, cross, tr in (("rotate", True, "host"), ("auto", None, "host"), ("rotate", True, "ipc")):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
               "--gpus", "2", "--steps", "3", "--warmup", "1", "--placement", place]
        r = subprocess.run(cmd, env=dict(env, SDML_TRANSPORT=tr), capture_output=True, text=True, timeout=300,
                           cwd=ROOT)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        d = _bench_json(r)
        assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["transport"] == tr
        assert d["config"]["world_size_seen"] == 2 and d["config"]["backend"] == "gloo"
        if cross:
            assert d["config"]["boundary_bytes_across_gpus_per_step"] == 2 * 4096 * (512 + 40)
        else:  # auto: the placement the cost model picks for this N and batch from the MEASURED link constants
            from simple_distributed_machine_learning_amd.parallel import placement as plc

            lm = d["config"]["link_measured"]
            assert lm["allreduce_us"] > 0 and lm["collective_us"] > 0 and lm["gbps"] > 0 and lm["pair_gbps"] > 0
            link = plc.LinkModel(**d["config"]["link_model"]["link"])
            want, phi, table = plc.choose(2, 8192, link=link, graph_dp=False)
            assert d["config"]["placement"] == want, (d["config"]["placement"], want)
            assert d["config"]["predicted"] == table
            if want == "dp":
                assert d["config"]["boundary_bytes_across_gpus_per_step"] == 0
        # self-checks: replicas bit-identical after the timed steps, the reference's cut measured at this even N
        assert d["config"]["replicas_identical"] is True, d["config"]["replica_check"]
        alt = d["config"]["measured_alternatives"]
        if d["config"]["placement"] != "pp2dp":
            assert "error" not in alt["pp2dp"] and alt["pp2dp"]["samples_per_s"] > 0, alt
    # a perturbed replica (test hook: one parameter bit flipped on rank 1 after the timed steps) fails the run
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--placement", "dp", "--alternatives", "off"]
    r = subprocess.run(cmd, env=dict(env, SDML_BENCH_PERTURB_RANK="1"), capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode != 0 and "replicas diverged" in r.stderr, r.stdout[-2000:] + r.stderr[-3000:]
    assert _bench_json(r)["config"]["replicas_identical"] is False


def test_bench_graph_replay_trains_identically():
    """bench.py --graph on (one HIP graph per cycled batch, the data read in place): the same kernels as the eager
    step, so the same final loss bit for bit; every step after the first (eager: momentum init) replays."""
    env = dict(os.environ, SDML_BENCH_BATCH="16384", PYTHONPATH=ROOT)
    out = {}
    for g in ("off", "on"):
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "5", "--graph", g]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        out[g] = _bench_json(r)
    assert out["off"]["config"]["hip_graph"] is None
    hg = out["on"]["config"]["hip_graph"]
    assert hg == {"graphs": 4, "replays": 7, "eager_steps": 0, "disabled": False, "captures_in_timed_region": 0,
                  "dataset_batches_cycled": 4}, hg
    assert out["on"]["final_loss"] == out["off"]["final_loss"]


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


# ---- the reference's own workload and BASELINE configs 3-5 across processes on the device ----
TRAIN_RE = __import__("re").compile(r"^Train Epoch: (\d+) \[(\d+)/(\d+) \((\d+)%\)\]\tLoss: (\d+\.\d{6})$")
TEST_RE = __import__("re").compile(r"^Test set: Average loss: (\d+\.\d{4}), Accuracy: (\d+)/(\d+) \((\d+)%\)$")


def _launch_reference_cli(extra, world=2, timeout=400, transport="host"):
    """``python simple_distributed.py --rank=R --world_size=2 --interface=lo --master_addr=127.0.0.1 ...`` (the
    reference's command line, README.txt:19) as ``world`` processes sharing cuda:0 through the host-staged
    (or the IPC) transport."""
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, SDML_TRANSPORT=transport)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        env.pop(k, None)
    procs = []
    for r in range(world):
        cmd = [sys.executable, os.path.join(ROOT, "simple_distributed.py"), f"--rank={r}", f"--world_size={world}",
               "--interface=lo", "--master_addr=127.0.0.1", f"--master_port={port}", "--device=cuda"] + extra
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env,
                                      cwd=ROOT))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-4000:]
    return outs


@pytest.mark.parametrize("transport", ["ipc", "host"])
def test_reference_command_line_two_ranks_on_device(tmp_path, transport):
    """The reference's CNN split exactly as its README runs it - conv stage on rank 0, fc stage on rank 1
    (/root/reference/simple_distributed.py:33-37, :47-49, :71, :138-186) - as two processes on the MI355X: the
    per-stage fused CNN kernels hand the [60, 320] boundary and its gradient across processes. The log lines keep
    the reference's format; at dropout 0 the trained per-stage weights (reference key names, from the stage
    checkpoints) equal the single-process GPU engine's after the same 12 steps."""
    import torch as _t

    from simple_distributed_machine_learning_amd.data import SyntheticMNIST
    from simple_distributed_machine_learning_amd.models import get_model_spec
    from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

    steps, B = 12, 60
    outs = _launch_reference_cli(["--epochs=1", f"--train_size={steps * B}", "--test_size=120", "--dropout=0",
                                  f"--ckpt_dir={tmp_path}"], transport=transport)
    lines = outs[0].splitlines()
    train = [m for m in map(TRAIN_RE.match, lines) if m]
    test = [m for m in map(TEST_RE.match, lines) if m]
    assert [(m.group(1), m.group(2), m.group(3), m.group(4)) for m in train] == [
        ("1", "0", "720", "0"), ("1", "600", "720", "83")], lines
    assert len(test) == 1 and test[0].group(3) == "120"
    i = lines.index(test[0].group(0))
    assert lines[i - 1] == "" and lines[i + 1] == ""
    assert not any(TRAIN_RE.match(l) for l in outs[1].splitlines())  # master-only logging
    got = {s: _t.load(tmp_path / f"stage{s}.pt", weights_only=True)["model"] for s in (0, 1)}
    assert set(got[0]) == {"conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias"}
    assert set(got[1]) == {"fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"}
    # the same run in one process on the device (default seed 1, data seed 1234, lr 0.1, momentum 0.5)
    mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=_t.device("cuda:0"))
    e = PipelineEngine(get_model_spec("ref_cnn", 2, dropout=0.0), mesh, schedule_kind="1f1b", num_microbatches=1,
                       lr=0.1, momentum=0.5, seed=1)
    ds = SyntheticMNIST(steps * B, seed=1234, device="cuda:0", mode="learnable", offset=0)
    for k in range(steps):
        e.run(ds, k * B, B, train=True, global_batch=B)
    want = e.state_dicts()
    for s in (0, 1):
        for k, v in got[s].items():
            _t.testing.assert_close(v, want[s][k], rtol=1e-4, atol=1e-5, msg=f"stage {s} {k}")


def test_mlp4x1024_gpipe_four_ranks_on_device():
    """BASELINE config 3: the 4-stage 4x1024 MLP, one stage per process, GPipe (fill-drain) on the device
    engine (two-fp16-plane hidden-layer GEMMs), against the single-process GPU engine."""
    B, steps, M = 512, 2, 4
    res = run_ranks(train_worker, 4, "mlp4x1024", "gpipe", M, 4, steps, B, 3, dict(GPU, transport="ipc"),
                    timeout=400)
    ref = _single("mlp4x1024", M, steps, B, "gpipe")
    _compare(res, ref, transport="ipc")
    assert all(r["bytes_sent"] > 0 for r in res)


def test_resnet18_bf16_eight_stages_four_ranks_1f1b_on_device():
    """BASELINE config 4: ResNet-18-style CNN in 8 stages on 4 processes (two stages each), 1F1B, bf16
    channels-last on the hand-written conv / BatchNorm / pooled-head kernels; boundaries [N, H, W, C] bf16 between
    processes. Same kernels in the same order as one process, so the weights agree to bf16 rounding."""
    B, steps, M = 16, 2, 2
    kw = dict(GPU, stages=8, dtype=torch.bfloat16, transport="ipc")
    res = run_ranks(train_worker, 4, "resnet18", "1f1b", M, 4, steps, B, 3, kw, timeout=400)
    ref = _single("resnet18", M, steps, B, "1f1b", {"stages": 8, "dtype": torch.bfloat16})
    _compare(res, ref, rtol=2e-2, atol=2e-3, transport="ipc")
    assert all(r["bytes_sent"] > 0 for r in res)


def test_gpt2_tiny_two_ranks_on_device():
    """BASELINE config 5's code path (the GPT-2 stage modules, flash attention, LayerNorm, fused vocab
    cross-entropy) in two processes on the device: the [B, S, d] boundary and its gradient cross processes."""
    B, steps, M = 4, 2, 2
    kw = dict(GPU, stages=2, seq_len=16)
    res = run_ranks(train_worker, 2, "gpt2_tiny", "1f1b", M, 2, steps, B, 3, kw, timeout=400)
    ref = _single("gpt2_tiny", M, steps, B, "1f1b", {"stages": 2, "seq_len": 16})
    _compare(res, ref)
    assert all(r["bytes_sent"] > 0 for r in res)
