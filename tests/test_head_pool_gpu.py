"""head_pool.hip (ResNet's last layer: average pool + Linear + log_softmax + NLL + backward in one launch and a
fixed-order reduction) against a float64 PyTorch reference of the same ops."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd import ops  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,C,H,W,ncls", [(64, 512, 4, 4, 10), (7, 64, 1, 1, 3), (130, 256, 2, 3, 16)])
def test_pooled_head_matches_reference(dtype, N, C, H, W, ncls):
    g = torch.Generator().manual_seed(N * C + ncls)
    y = torch.randn(N, C, H, W, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(ncls, C, generator=g) * 0.05).to(DEV, dtype)
    b = (torch.randn(ncls, generator=g) * 0.1).to(DEV, dtype)
    t = torch.randint(0, ncls, (N,), generator=g).to(DEV)
    t[N // 2] = ncls  # out of range: no loss term, no gradient (as the other fused heads)
    gw0 = (torch.randn(ncls, C, generator=g) * 0.01).to(DEV, dtype)
    gb0 = (torch.randn(ncls, generator=g) * 0.01).to(DEV, dtype)
    gw, gb = gw0.clone(), gb0.clone()
    stats = torch.full((2,), 3.0, device=DEV)
    scale = 1.0 / 97
    dy = ops.pooled_head_xent(y, w, b, t, gw, gb, scale, stats)
    torch.cuda.synchronize()
    # reference (float64): rows with a valid label only
    yd = y.double().requires_grad_(True)
    feats = yd.mean(dim=(2, 3))
    z = feats @ w.double().t() + b.double()
    ok = t < ncls
    wd = w.double().requires_grad_(True)
    bd = b.double().requires_grad_(True)
    z = feats @ wd.t() + bd
    loss = F.cross_entropy(z[ok], t[ok], reduction="sum")
    (loss * scale).backward()
    correct = int((z.argmax(1) == t)[ok].sum())
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert float(stats[0]) == pytest.approx(3.0 + float(loss), rel=1e-4)
    assert int(round(float(stats[1]) - 3.0)) == correct
    torch.testing.assert_close(dy.double(), yd.grad, rtol=tol, atol=tol * float(yd.grad.abs().max()))
    assert dy.is_contiguous(memory_format=torch.channels_last) or H * W == 1
    torch.testing.assert_close(gw.double(), gw0.double() + wd.grad, rtol=tol, atol=tol * float(wd.grad.abs().max()))
    torch.testing.assert_close(gb.double(), gb0.double() + bd.grad, rtol=tol, atol=tol * float(bd.grad.abs().max()))


def test_pooled_head_is_deterministic():
    g = torch.Generator().manual_seed(5)
    y = torch.randn(64, 512, 4, 4, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(10, 512, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.zeros(10, device=DEV, dtype=torch.bfloat16)
    t = torch.randint(0, 10, (64,), generator=g).to(DEV)
    outs = []
    for _ in range(2):
        gw, gb = torch.zeros_like(w), torch.zeros_like(b)
        st = torch.zeros(2, device=DEV)
        dy = ops.pooled_head_xent(y, w, b, t, gw, gb, 1 / 64, st)
        outs.append((dy, gw, gb, st))
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
