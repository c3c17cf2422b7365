"""The reference-size MLP step in two launches (mlp_small.hip) against the multi-kernel engine
step it replaces (SDML_SMALL_STEP=0): same data, same seeds, every SGD option; fp32 agreement (the
summation orders differ), equal correct counts. Reference: /root/reference/simple_distributed.py:18
(B = 60), :100-113 (one training step)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402

DEV = torch.device("cuda", 0)


def _run(kind, B, steps, pixels, opt):
    mesh = init_mesh(pp=1, schedule_kind=kind, rank=0, world_size=1, device=DEV)
    e = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind=kind, num_microbatches=1, lr=0.1,
                       momentum=opt.get("momentum", 0.5), weight_decay=opt.get("wd", 0.0), seed=3)
    e.optimizer.dampening, e.optimizer.nesterov = opt.get("damp", 0.0), opt.get("nesterov", False)
    ds = SyntheticMNIST(B * steps, seed=9, device=DEV, pixels=pixels)
    out = []
    for s in range(steps):
        r = e.run(ds, s * B, B, train=True)
        out.append((float(r.loss_sum), int(r.correct), r.count))
    torch.cuda.synchronize()
    return e, out


@pytest.mark.parametrize("B", [60, 128, 7])
@pytest.mark.parametrize("pixels", ["f32", "u8"])
@pytest.mark.parametrize("opt", [dict(), dict(momentum=0.0), dict(wd=1e-4, damp=0.1), dict(nesterov=True)])
def test_small_step_matches_multi_kernel_step(B, pixels, opt, monkeypatch):
    monkeypatch.setenv("SDML_SMALL_STEP", "0")
    e0, r0 = _run("1f1b", B, 5, pixels, opt)
    monkeypatch.setenv("SDML_SMALL_STEP", "1")
    e1, r1 = _run("1f1b", B, 5, pixels, opt)
    assert e1.fast_steps["mlp_small"] > 0 and e0.fast_steps["mlp_small"] == 0
    for (l0, c0, n0), (l1, c1, n1) in zip(r0, r1):
        assert n0 == n1 == B
        assert l1 == pytest.approx(l0, rel=1e-5, abs=1e-5)
        assert abs(c0 - c1) <= 1  # an argmax tie broken by a last-ulp logit difference at most
    torch.testing.assert_close(e1.flat.params, e0.flat.params, rtol=1e-5, atol=1e-6)
    if e0.optimizer.momentum:
        torch.testing.assert_close(e1.optimizer.momentum_buffer, e0.optimizer.momentum_buffer, rtol=1e-4,
                                   atol=1e-6)
    assert float(e1.flat.grads.abs().max()) == 0.0  # consumed in the kernel: the buffer stays clear


def test_small_step_then_large_batch_uses_fresh_weight_planes():
    """After one-launch steps (which do not write the uint8 forward's weight planes) a large-batch uint8
    step must re-split the planes from the updated weights."""
    e, _ = _run("1f1b", 60, 3, "u8", {})
    cache = e.stages[0].plane_cache
    if cache is not None:
        assert cache.token is None
    ds = SyntheticMNIST(8192, seed=10, device=DEV, pixels="u8")
    r = e.run(ds, 0, 8192, train=True)
    assert torch.isfinite(r.loss_sum)


def _run_cnn(B, steps, opt, dropout=0.5):
    mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=DEV)
    torch.manual_seed(1)  # the host RNG draws the dropout seeds: same stream for both runs
    e = PipelineEngine(get_model_spec("ref_cnn", 2, dropout=dropout), mesh, schedule_kind="1f1b", num_microbatches=1,
                       lr=0.1, momentum=opt.get("momentum", 0.5), weight_decay=opt.get("wd", 0.0), seed=3)
    e.optimizer.dampening, e.optimizer.nesterov = opt.get("damp", 0.0), opt.get("nesterov", False)
    ds = SyntheticMNIST(B * steps, seed=9, device=DEV)
    out = []
    for s in range(steps):
        r = e.run(ds, s * B, B, train=True)
        out.append((float(r.loss_sum), int(r.correct), r.count))
    torch.cuda.synchronize()
    return e, out


@pytest.mark.parametrize("B", [60, 7, 300])
@pytest.mark.parametrize("opt", [dict(), dict(momentum=0.0), dict(wd=1e-4, damp=0.1, nesterov=True)])
def test_cnn_step_matches_per_stage_kernels(B, opt, monkeypatch):
    """The reference CNN's two-launch step (ref_cnn.hip cnn_step_*) against the per-stage kernels + SGD it
    replaces: same dropout masks (same host seeds, same device counter), fp32 agreement (fixed-order sums vs
    atomics), and the dropout counter advanced once per step."""
    monkeypatch.setenv("SDML_SMALL_STEP", "0")
    e0, r0 = _run_cnn(B, 4, opt)
    monkeypatch.setenv("SDML_SMALL_STEP", "1")
    e1, r1 = _run_cnn(B, 4, opt)
    assert e1.fast_steps["cnn"] == 4 and e0.fast_steps["cnn"] == 0
    for (l0, c0, n0), (l1, c1, n1) in zip(r0, r1):
        assert n0 == n1 == B
        assert l1 == pytest.approx(l0, rel=1e-4, abs=1e-4)
        assert abs(c0 - c1) <= 1
    torch.testing.assert_close(e1.flat.params, e0.flat.params, rtol=1e-4, atol=2e-6)
    assert int(e1.step_ctr) == int(e0.step_ctr) == 4
    assert float(e1.flat.grads.abs().max()) == 0.0
