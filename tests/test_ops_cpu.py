"""The PyTorch reference ops (the numerics contract of the HIP kernels) match autograd."""
import torch
import torch.nn.functional as F

from simple_distributed_machine_learning_amd.ops import reference as ref
from simple_distributed_machine_learning_amd.ops.optim import FusedSGD
from simple_distributed_machine_learning_amd.utils.flat import FlatParams


def test_linear_relu_bwd_matches_autograd():
    torch.manual_seed(0)
    x = torch.randn(7, 5, dtype=torch.float64, requires_grad=True)
    w = torch.randn(4, 5, dtype=torch.float64, requires_grad=True)
    b = torch.randn(4, dtype=torch.float64, requires_grad=True)
    y = torch.relu(x @ w.t() + b)
    gy = torch.randn_like(y)
    y.backward(gy)
    gw, gb = torch.zeros_like(w), torch.zeros_like(b)
    dx = ref.linear_relu_bwd(x.detach(), y.detach(), gy, w.detach(), gw, gb, True)
    torch.testing.assert_close(dx, x.grad)
    torch.testing.assert_close(gw, w.grad)
    torch.testing.assert_close(gb, b.grad)


def test_head_matches_autograd():
    torch.manual_seed(1)
    x = torch.randn(9, 6, dtype=torch.float64, requires_grad=True)
    w = torch.randn(3, 6, dtype=torch.float64, requires_grad=True)
    b = torch.randn(3, dtype=torch.float64, requires_grad=True)
    t = torch.randint(0, 3, (9,))
    loss = F.nll_loss(F.log_softmax(x @ w.t() + b, 1), t, reduction="sum")
    (loss * 0.25).backward()
    gw, gb = torch.zeros_like(w), torch.zeros_like(b)
    l, c, dx = ref.linear_logsoftmax_nll(x.detach(), w.detach(), b.detach(), t, gw, gb, 0.25, True)
    torch.testing.assert_close(l, loss.detach())
    torch.testing.assert_close(dx, x.grad)
    torch.testing.assert_close(gw, w.grad)
    torch.testing.assert_close(gb, b.grad)


def test_fused_sgd_matches_torch_sgd():
    torch.manual_seed(2)
    m1 = torch.nn.Sequential(torch.nn.Linear(5, 4), torch.nn.Linear(4, 3))
    m2 = torch.nn.Sequential(torch.nn.Linear(5, 4), torch.nn.Linear(4, 3))
    m2.load_state_dict(m1.state_dict())
    flat = FlatParams([(0, m2)], "cpu")
    opt_ref = torch.optim.SGD(m1.parameters(), lr=0.1, momentum=0.5)
    opt = FusedSGD(flat, lr=0.1, momentum=0.5)
    for _ in range(4):
        x = torch.randn(8, 5)
        opt_ref.zero_grad()
        m1(x).square().sum().backward()
        flat.zero_grad(force=True)
        m2(x).square().sum().backward()
        assert flat.check_bound()
        opt_ref.step()
        opt.step()
        for a, b in zip(m1.parameters(), m2.parameters()):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    assert float(flat.grads.abs().sum()) == 0.0  # step(zero_grad=True) cleared the grads


def test_fused_sgd_bf16_keeps_fp32_master():
    torch.manual_seed(3)
    m = torch.nn.Linear(8, 8).to(torch.bfloat16)
    flat = FlatParams([(0, m)], "cpu", dtype=torch.bfloat16)
    opt = FusedSGD(flat, lr=1e-3, momentum=0.5)
    assert opt.master is not None and opt.master.dtype == torch.float32
    w0 = opt.master.clone()
    for _ in range(3):
        flat.zero_grad(force=True)
        m(torch.randn(4, 8, dtype=torch.bfloat16)).float().square().sum().backward()
        opt.step()
    # tiny updates accumulate in the fp32 master even when they are below bf16 resolution
    assert not torch.equal(opt.master, w0)
    torch.testing.assert_close(flat.params, opt.master.to(torch.bfloat16), rtol=0, atol=0)


def test_ref_cnn_cpu_ops_match_modules_without_dropout():
    from simple_distributed_machine_learning_amd import ops
    from simple_distributed_machine_learning_amd.models.ref_cnn import Network1Stage, Network2Stage

    torch.manual_seed(0)
    s0, s1 = Network1Stage(0.0), Network2Stage(False, 0.0)
    for p in list(s0.parameters()) + list(s1.parameters()):
        p.grad = torch.zeros_like(p)
    x = torch.rand(9, 1, 28, 28)
    t = torch.randint(0, 10, (9,))
    y, _ = ops.ref_cnn_stage0_fwd(x, s0.conv1, s0.conv2, 5, 0.0, False)
    torch.testing.assert_close(y, s0(x))
    st = torch.zeros(2)
    dx = ops.ref_cnn_stage1(y, s1.fc1, s1.fc2, t, 5, 0.0, False, 0.5, st, True)
    yy = y.clone().requires_grad_(True)
    loss = torch.nn.functional.nll_loss(s1(yy), t, reduction="sum")
    torch.testing.assert_close(st[0], loss.detach())
    g = torch.autograd.grad(loss * 0.5, [yy, s1.fc1.weight, s1.fc2.bias])
    torch.testing.assert_close(dx, g[0])
    torch.testing.assert_close(s1.fc1.weight.grad, g[1])
    torch.testing.assert_close(s1.fc2.bias.grad, g[2])


def test_dropout_hash_statistics():
    from simple_distributed_machine_learning_amd.ops import reference as ref

    m = ref.dropout_keep_scale(12345, 0, 2000, 50, 0.5)
    assert set(torch.unique(m).tolist()) == {0.0, 2.0}
    assert abs(float((m == 0).float().mean()) - 0.5) < 0.01
    assert torch.equal(m[10:20], ref.dropout_keep_scale(12345, 10, 10, 50, 0.5))
    assert not torch.equal(m, ref.dropout_keep_scale(12346, 0, 2000, 50, 0.5))


def test_debug_sync_rejects_out_of_range_targets():
    """the fused heads skip rows with a label outside [0, C); under debug_sync the engine
    refuses such a batch up front, as the reference's nll_loss would."""
    import pytest

    from simple_distributed_machine_learning_amd.data import SyntheticMNIST
    from simple_distributed_machine_learning_amd.models import get_model_spec
    from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh

    mesh = init_mesh(pp=1, schedule_kind="1f1b", rank=0, world_size=1, device=torch.device("cpu"))
    e = PipelineEngine(get_model_spec("mlp", 2), mesh, schedule_kind="1f1b", num_microbatches=1, lr=0.01,
                       momentum=0.5, seed=1, debug_sync=True)
    ds = SyntheticMNIST(64, seed=1, device="cpu")
    e.run(ds, 0, 32, train=True)  # valid labels pass
    ds.y[40] = 10
    with pytest.raises(ValueError, match="target out of range"):
        e.run(ds, 32, 32, train=True)
    ds.y[40] = -100
    with pytest.raises(ValueError, match="target out of range"):
        e.run(ds, 32, 32, train=True)


def test_kernel_knobs_pin_timing_probes_in_production_builds():
    """a production build cannot switch on a probe that skips work (the bf16 GEMM
    without its output stores); variant switches between correct kernels are explicit setters."""
    import pytest

    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    assert not K.kernel_experiments_build()
    with pytest.raises(RuntimeError, match="probe"):
        K.set_knob("GEMM_BF16_NOSTORE", 1)
    with pytest.raises(RuntimeError, match="unknown"):
        K.set_knob("NO_SUCH_KNOB", 1)
    K.set_knob("WGRAD_DMA", 0)
    K.reset_knobs()


def test_flat_params_row_padding_stays_zero_under_sgd():
    """FlatParams row padding (a module's ``flat_row_multiple``, GPT-2's lm_head vocabulary): the rows past the
    parameter's own are zero in the parameter and gradient storage, views are unchanged in shape and name, and SGD with
    momentum keeps the pad rows zero (their gradient is zero)."""
    from simple_distributed_machine_learning_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    m = torch.nn.Linear(6, 13, bias=True)
    m.flat_row_multiple = {"weight": 8}
    flat = FlatParams([(0, m)], "cpu")
    w = m.weight
    assert tuple(w.shape) == (13, 6) and w._sdml_rows_padded == 16
    padded = w.as_strided((16, 6), (6, 1))
    assert torch.equal(padded[:13], w) and int((padded[13:] != 0).sum()) == 0
    gpad = w.grad.as_strided((16, 6), (6, 1))
    opt = FusedSGD(flat, lr=0.1, momentum=0.5)
    for _ in range(3):
        flat.zero_grad(force=True)
        x = torch.randn(4, 6)
        m(x).square().sum().backward()
        opt.step()
    assert int((padded[13:] != 0).sum()) == 0 and int((gpad[13:] != 0).sum()) == 0
    assert set(dict(m.named_parameters())) == {"weight", "bias"}
    # the bias segment starts after the padded rows (64-element aligned offsets)
    seg = {s.name: s for s in flat.segments}
    assert seg["bias"].offset >= seg["weight"].offset + 16 * 6
