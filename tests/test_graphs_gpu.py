"""hipGraph-captured training step (parallel/graphs.py) == eager engine step (GPU only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402
from simple_distributed_machine_learning_amd.parallel.graphs import GraphedStep  # noqa: E402

DEV = torch.device("cuda", 0)


def _engine(model, kind="1f1b", M=2, **kw):
    mesh = init_mesh(pp=1, schedule_kind=kind, rank=0, world_size=1, device=DEV)
    return PipelineEngine(get_model_spec(model, None, **kw), mesh, schedule_kind=kind, num_microbatches=M, lr=0.1,
                          momentum=0.5, seed=5)


@pytest.mark.parametrize("model,kw,kind,M", [("mlp", {}, "1f1b", 1), ("mlp", {}, "gpipe", 3),
                                             ("mlp4x1024", {}, "1f1b", 2), ("ref_cnn", {"dropout": 0.0}, "1f1b", 1),
                                             ("ref_cnn", {"dropout": 0.0}, "chimera", 2),
                                             ("gpt2_tiny", {"seq_len": 32}, "1f1b", 4)])
def test_graphed_step_matches_eager(model, kw, kind, M):
    if model == "gpt2_tiny":
        from simple_distributed_machine_learning_amd.data import SyntheticTokens

        ds = SyntheticTokens(600, 32, 97, seed=3, device=DEV)
    else:
        ds = SyntheticMNIST(600, seed=3, device=DEV)
    e1, e2 = _engine(model, kind, M, **kw), _engine(model, kind, M, **kw)
    g = GraphedStep(e2)
    sizes = [60, 60, 60, 60, 40, 60]  # the 40 is a ragged last batch: its own graph
    start = 0
    for B in sizes:
        r1 = e1.run(ds, start, B, train=True)
        l1, c1 = float(r1.loss_sum), int(r1.correct)
        r2 = g(ds, start, B)
        l2, c2 = float(r2.loss_sum), int(r2.correct)
        tol = 2e-2 if model == "gpt2_tiny" else 1e-4  # bf16 model: atomics reorder -> bf16 rounding
        assert abs(l1 - l2) <= tol * max(1.0, abs(l1))
        assert (c1 == c2 or model == "gpt2_tiny") and r1.count == r2.count
        start += B
    assert g.replays == len(sizes) - 1 and len(g.graphs) == 2 and not g.disabled
    if model == "gpt2_tiny":
        torch.testing.assert_close(e1.flat.params.float(), e2.flat.params.float(), rtol=2e-2, atol=2e-2)
    else:
        torch.testing.assert_close(e1.flat.params, e2.flat.params, rtol=1e-5, atol=1e-6)
    assert e1.global_step == e2.global_step
    assert int(e1.step_ctr) == int(e2.step_ctr) == (len(sizes) if model == "ref_cnn" else 0)


def test_graphed_dropout_draws_fresh_masks():
    ds = SyntheticMNIST(120, seed=4, device=DEV)
    e = _engine("ref_cnn", "1f1b", 1, dropout=0.5)
    e.optimizer.lr = 0.0  # weights fixed: loss differences come from the masks alone
    g = GraphedStep(e)
    losses = [float(g(ds, 0, 60).loss_sum) for _ in range(4)]
    assert g.replays == 3
    assert len(set(losses[1:])) == 3  # every replay saw different dropout masks
    assert int(e.step_ctr) == 4


def test_graphed_step_with_rccl_allreduce_on_one_rank():
    """A captured step that contains an RCCL collective: a one-rank "nccl" (RCCL) process group, a mesh
    that keeps its gradient all-reduce (force_collectives), GraphedStep(allow_collectives=True); the
    replays must match the eager engine without any process group. Runs in a subprocess (process-group
    state stays out of the test session)."""
    import os
    import subprocess
    import sys
    import textwrap

    from conftest import free_port

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent("""
        import datetime, torch, torch.distributed as dist
        from simple_distributed_machine_learning_amd.data import SyntheticMNIST
        from simple_distributed_machine_learning_amd.models import get_model_spec
        from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh
        from simple_distributed_machine_learning_amd.parallel.graphs import GraphedStep
        dev = torch.device("cuda", 0)
        ds = SyntheticMNIST(8192 * 6, seed=3, device=dev, pixels="u8")
        def engine(mesh):
            return PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="rotate", num_microbatches=1,
                                  lr=0.1, momentum=0.5, seed=5)
        e1 = engine(init_mesh(pp=1, schedule_kind="rotate", rank=0, world_size=1, device=dev))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, timeout=datetime.timedelta(seconds=60))
        m2 = init_mesh(pp=1, schedule_kind="rotate", rank=0, world_size=1, device=dev, force_collectives=True)
        e2 = engine(m2)
        assert e2.grad_sync.enabled and e2.transport is not None
        g = GraphedStep(e2, allow_collectives=True)
        ops0 = e2.transport.ops
        for i in range(6):
            r1 = e1.run(ds, i * 8192, 8192, train=True)
            r2 = g(ds, i * 8192, 8192)
            assert abs(float(r1.loss_sum) - float(r2.loss_sum)) <= 1e-4 * abs(float(r1.loss_sum))
        torch.cuda.synchronize()
        assert g.replays == 5 and not g.disabled, (g.replays, g.disabled)
        assert e2.transport.ops > ops0  # the all-reduce was issued (eager step + capture)
        torch.testing.assert_close(e1.flat.params, e2.flat.params, rtol=1e-5, atol=1e-6)
        dist.destroy_process_group()
        print("graph+rccl ok")
    """)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and "graph+rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_graphed_step_many_waves_ragged_keeps_buffers_alive():
    """more than 16 fused waves evict the engine's per-wave (ReLU bits, gradient) buffers; a captured graph
    keeps their addresses, so evicted buffers must stay alive while the graph can replay. 18 waves (rotate schedule,
    one rank) plus a ragged batch with its own graph: the replays must match an eager engine step for step."""
    ds = SyntheticMNIST(18 * 256 * 8, seed=6, device=DEV, pixels="u8")

    def eng():
        mesh = init_mesh(pp=1, schedule_kind="rotate", rank=0, world_size=1, device=DEV)
        return PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="rotate", num_microbatches=18, lr=0.1,
                              momentum=0.5, seed=7)

    e1, e2 = eng(), eng()
    g = GraphedStep(e2)
    B = 18 * 256
    sizes = [B, B, B - 100, B, B - 100, B, B - 100]
    start = 0
    for n in sizes:
        r1 = e1.run(ds, start, n, train=True)
        r2 = g(ds, start, n)
        assert abs(float(r1.loss_sum) - float(r2.loss_sum)) <= 1e-4 * max(1.0, abs(float(r1.loss_sum)))
        start += n
    torch.cuda.synchronize()
    assert g.replays == len(sizes) - 1 and len(g.graphs) == 2 and not g.disabled
    assert len(e2._wave_bufs) + len(e2._wave_bufs_retired) >= 17  # the eviction path ran with graphs alive
    torch.testing.assert_close(e1.flat.params, e2.flat.params, rtol=1e-5, atol=1e-6)
