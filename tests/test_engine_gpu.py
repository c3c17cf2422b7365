"""Stage-level and engine-level checks on the GPU: the fused HIP MLP stages reproduce
PyTorch autograd on the same weights, and a full pipeline step on cuda matches the CPU
engine step (same seeds, same data)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402

DEV = torch.device("cuda", 0)


def _engine(model, device, kind="1f1b", M=2, stages=None, **kw):
    mesh = init_mesh(pp=1, schedule_kind=kind, rank=0, world_size=1, device=device)
    spec = get_model_spec(model, stages, **kw)
    return PipelineEngine(spec, mesh, schedule_kind=kind, num_microbatches=M, lr=0.1, momentum=0.5, seed=3)


@pytest.mark.parametrize("model", ["mlp", "mlp4x1024", "ref_cnn"])
@pytest.mark.parametrize("kind,M", [("1f1b", 1), ("1f1b", 3), ("gpipe", 4), ("chimera", 4)])
def test_gpu_engine_matches_cpu(model, kind, M):
    kw = {"dropout": 0.0} if model == "ref_cnn" else {}  # fused CNN kernels vs PyTorch, no RNG
    e_gpu = _engine(model, DEV, kind, M, **kw)
    e_cpu = _engine(model, torch.device("cpu"), kind, M, **kw)
    torch.testing.assert_close(e_gpu.flat.params.cpu(), e_cpu.flat.params)
    ds_g = SyntheticMNIST(600, seed=11, device=DEV)
    ds_c = SyntheticMNIST(600, seed=11, device="cpu")
    for step in range(3):
        rg = e_gpu.run(ds_g, step * 120, 120, train=True)
        rc = e_cpu.run(ds_c, step * 120, 120, train=True)
        torch.testing.assert_close(float(rg.loss_sum), float(rc.loss_sum), rtol=1e-4, atol=1e-3)
        assert int(rg.correct) == int(rc.correct)
    torch.testing.assert_close(e_gpu.flat.params.cpu(), e_cpu.flat.params, rtol=1e-4, atol=2e-5)


def test_gpu_eval_and_ref_cnn_runs():
    e = _engine("ref_cnn", DEV, "1f1b", 2)
    ds = SyntheticMNIST(200, seed=2, device=DEV)
    r = e.run(ds, 0, 60, train=True)
    assert torch.isfinite(r.loss_sum)
    e.eval()
    r = e.run(ds, 60, 40, train=False)
    assert r.count == 40


def test_resnet_fp32_refused_on_gpu():
    """no MIOpen / ATen convolution on a GPU code path. The ResNet's device kernels are bf16
    channels-last; an fp32 ResNet on the GPU raises instead of silently running the library (ops/conv.py)."""
    mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=DEV)
    e = PipelineEngine(get_model_spec("resnet18", None), mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.01,
                       momentum=0.5, seed=3)
    ds = SyntheticMNIST(16, seed=1, device=DEV)
    with pytest.raises(RuntimeError, match="no hand-written gfx950 kernel"):
        e.run(ds, 0, 16, train=True)


@pytest.mark.parametrize("model,B,kw", [("resnet18", 16, {"dtype": torch.bfloat16}),
                                        ("gpt2_tiny", 8, {"seq_len": 16}), ("gpt2", 2, {"seq_len": 64})])
def test_gpu_models_train(model, B, kw):
    from simple_distributed_machine_learning_amd.data import SyntheticTokens

    mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=DEV)
    spec = get_model_spec(model, None, **kw)
    e = PipelineEngine(spec, mesh, schedule_kind="1f1b", num_microbatches=2, lr=0.01, momentum=0.5, seed=3)
    if spec.input_kind == "tokens":
        vocab = 97 if model == "gpt2_tiny" else 50257
        ds = SyntheticTokens(4 * B, kw["seq_len"], vocab, seed=1, device=DEV)
    else:
        ds = SyntheticMNIST(4 * B, seed=1, device=DEV)
    p0 = e.flat.params.clone()
    losses = []
    for i in range(3):
        r = e.run(ds, 0, B, train=True)
        losses.append(float(r.loss_sum) / r.count)
    assert all(l == l for l in losses)  # finite
    assert not torch.equal(p0, e.flat.params)
    assert losses[-1] < losses[0]  # same batch thrice: loss must drop


def test_resnet_bf16_hip_kernels_match_library_path(monkeypatch):
    """8-stage ResNet, bf16 channels-last: the hand-written conv/BatchNorm kernels train like the
    MIOpen/PyTorch path (same init, same data, 3 steps)."""
    from simple_distributed_machine_learning_amd.ops import conv as conv_ops

    def run():
        mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=DEV)
        spec = get_model_spec("resnet18", 8, dtype=torch.bfloat16)
        e = PipelineEngine(spec, mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.05, momentum=0.5, seed=3)
        ds = SyntheticMNIST(64, seed=1, device=DEV)
        out = [float(e.run(ds, 0, 64, train=True).loss_sum) / 64 for _ in range(3)]
        return out, e.flat.params.float().clone()

    fused0 = conv_ops.ResidualLink.fused
    hip_losses, hip_p = run()
    assert conv_ops.ResidualLink.fused - fused0 == 3 * 8  # every block joins its input gradient in an epilogue
    monkeypatch.setattr(conv_ops, "LIBRARY_ON_GPU", True)  # the library path as the reference
    monkeypatch.setattr(conv_ops, "hip_eligible", lambda x, conv: False)
    monkeypatch.setattr(conv_ops, "bn_eligible", lambda x, bn, res=None: False)
    lib_losses, lib_p = run()
    for a, b in zip(hip_losses, lib_losses):
        assert abs(a - b) <= 0.02 * abs(b) + 0.02, (hip_losses, lib_losses)
    rel = (hip_p - lib_p).norm() / lib_p.norm()
    assert rel < 0.02, float(rel)


@pytest.mark.parametrize("model,kind", [("mlp", "1f1b"), ("mlp", "rotate"), ("mlp4x1024", "gpipe"), ("ref_cnn", "1f1b")])
def test_gpu_u8_pixels_match_cpu_float(model, kind):
    """uint8 pixel batches (ToTensor fused into the MLPs' first GEMM on the GPU, converted by the
    engine for other models) train like float32 k/255 images on the CPU engine. 8192-sample
    batches put the MLP's first layer on the uint8 bf16x3 kernels."""
    kw = {"dropout": 0.0} if model == "ref_cnn" else {}
    B = 120 if model == "ref_cnn" else 8192
    e_gpu = _engine(model, DEV, kind, 2, **kw)
    e_cpu = _engine(model, torch.device("cpu"), kind, 2, **kw)
    ds_g = SyntheticMNIST(2 * B, seed=5, device=DEV, pixels="u8")
    ds_c = SyntheticMNIST(2 * B, seed=5, device="cpu")
    assert ds_g.x.dtype == torch.uint8
    ds_c.x = ds_g.x.cpu().float().div_(255.0)
    for step in range(2):
        rg = e_gpu.run(ds_g, step * B, B, train=True)
        rc = e_cpu.run(ds_c, step * B, B, train=True)
        torch.testing.assert_close(float(rg.loss_sum), float(rc.loss_sum), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(e_gpu.flat.params.cpu(), e_cpu.flat.params, rtol=1e-4, atol=5e-5)


def test_gpu_u8_weight_plane_cache_follows_the_weights():
    """fc1's fp16 weight planes are written by the SGD step kernel (no split launch per step) and
    stay current: after steps, after an in-place weight change (a checkpoint load), after more steps,
    the forward equals a forward without the cache."""
    from simple_distributed_machine_learning_amd import ops

    B = 8192
    e = _engine("mlp", DEV, "1f1b", 1)
    s0 = e.stages[0]
    assert s0.plane_cache is not None and e.optimizer.plane_cache is not None
    ds = SyntheticMNIST(3 * B, seed=9, device=DEV, pixels="u8")
    fc1 = s0.fc1
    x = ds.x[:B].reshape(B, -1).contiguous()

    def check():
        got = ops.linear_relu_fwd_u8(x, fc1.weight, fc1.bias, s0.plane_cache, e.flat.param_epoch)
        want = ops.linear_relu_fwd_u8(x, fc1.weight, fc1.bias)  # fresh split
        assert torch.equal(got, want)

    for step in range(2):
        e.run(ds, step * B, B, train=True)
    check()
    assert s0.plane_cache.token == ops.PlaneCache.token_of(fc1.weight, e.flat.param_epoch)
    with torch.no_grad():
        fc1.weight.mul_(0.5)  # e.g. load_state_dict: bumps the version, the cache must re-split
    check()
    e.run(ds, 2 * B, B, train=True)
    check()


@pytest.mark.parametrize("factored", [True, False])
def test_gpu_rotate_one_rank_factored_and_whole_gradient(factored):
    """Rotate on one rank: the head returns its factor dl (stage 0's weight-gradient kernel expands
    it, dz bounded by the head's per-block bounds) or dx (bounds attached to dx); both train like
    the CPU engine on the same images."""
    B = 8192
    e_gpu = _engine("mlp", DEV, "rotate", 1)
    e_gpu.factored_r1 = factored
    e_cpu = _engine("mlp", torch.device("cpu"), "rotate", 1)
    ds_g = SyntheticMNIST(2 * B, seed=7, device=DEV, pixels="u8")
    ds_c = SyntheticMNIST(2 * B, seed=7, device="cpu")
    ds_c.x = ds_g.x.cpu().float().div_(255.0)
    for step in range(2):
        rg = e_gpu.run(ds_g, step * B, B, train=True)
        rc = e_cpu.run(ds_c, step * B, B, train=True)
        torch.testing.assert_close(float(rg.loss_sum), float(rc.loss_sum), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(e_gpu.flat.params.cpu(), e_cpu.flat.params, rtol=1e-4, atol=5e-5)


def test_gpu_u8_headline_training_tracks_cpu_fp32_over_steps():
    """The headline path (rotate on one rank, uint8 pixels, fp16-plane first layer, factored
    boundary gradient) against the CPU fp32 engine over 12 steps of fresh data: the loss curve and
    the weights stay within fp32 rounding drift."""
    B = 16384
    e_gpu = _engine("mlp", DEV, "rotate", 1)
    e_cpu = _engine("mlp", torch.device("cpu"), "rotate", 1)
    ds_g = SyntheticMNIST(12 * B, seed=21, device=DEV, pixels="u8")
    ds_c = SyntheticMNIST(12 * B, seed=21, device="cpu")
    ds_c.x = ds_g.x.cpu().float().div_(255.0)
    lg, lc = [], []
    for step in range(12):
        lg.append(float(e_gpu.run(ds_g, step * B, B, train=True).loss_sum) / B)
        lc.append(float(e_cpu.run(ds_c, step * B, B, train=True).loss_sum) / B)
    assert lg[-1] < lg[0]  # it learns (the synthetic classes are separable)
    for a, b in zip(lg, lc):
        assert abs(a - b) <= 1e-4 * abs(b) + 1e-5, (lg, lc)
    d = (e_gpu.flat.params.cpu() - e_cpu.flat.params).abs().max().item()
    print(f"max |param diff| after 12 steps: {d:.3e}")
    torch.testing.assert_close(e_gpu.flat.params.cpu(), e_cpu.flat.params, rtol=1e-4, atol=1e-4)
