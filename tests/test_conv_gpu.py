"""Hand-written 3x3 convolution kernels (csrc/kernels/conv_bf16.hip) vs an fp32 PyTorch reference
computed on the same bf16 values: forward, input gradient and weight gradient."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd import _native  # noqa: E402
from simple_distributed_machine_learning_amd.ops import conv as conv_ops  # noqa: E402

DEV = torch.device("cuda", 0)
K = _native.kernels()


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


# W <= 31: halo kernel, 5 halo chunks per thread; W 32..95: 7 chunks; W > 95: im2col kernel
@pytest.mark.parametrize("N,C,Co,H,W", [(4, 64, 128, 14, 14), (3, 128, 64, 7, 7), (2, 64, 64, 28, 28),
                                        (5, 256, 256, 4, 4), (1, 128, 192, 9, 11), (2, 128, 64, 3, 40),
                                        (1, 64, 128, 2, 100)])
def test_conv3x3_fwd_dgrad_wgrad(N, C, Co, H, W):
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + C + Co + H)
    x = torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(Co, C, 3, 3, generator=g) * 0.05).to(DEV, torch.bfloat16)
    dy = torch.randn(N, Co, H, W, generator=g).to(DEV, torch.bfloat16)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, padding=1)
    yr.backward(dy.float())
    # forward; the fused two-layout transform matches the single ones
    wf, wd = K.conv3x3_weights_bf16(w)
    assert torch.equal(wf, K.conv3x3_weight_bf16(w, False)) and torch.equal(wd, K.conv3x3_weight_bf16(w, True))
    # and the batched transform (several weights, one launch; a forward-only entry) into caller buffers
    w2 = (torch.randn(C, Co, 3, 3, generator=g) * 0.05).to(DEV, torch.bfloat16)
    bufs = [torch.empty_like(wf), torch.empty_like(wd), torch.empty(C, 9, Co, device=DEV, dtype=torch.bfloat16)]
    K.conv3x3_weights_batched_bf16([w, w2], [bufs[0], bufs[2]], [bufs[1], None])
    assert torch.equal(bufs[0], wf) and torch.equal(bufs[1], wd)
    assert torch.equal(bufs[2], K.conv3x3_weight_bf16(w2, False))
    y = K.conv3x3_fwd_bf16(cl(x), wf)
    assert y.is_contiguous(memory_format=torch.channels_last)
    scale = F.conv2d(x.float().abs(), w.float().abs(), padding=1) + 1e-3
    assert ((y.float() - yr.detach()).abs() <= 2 ** -7 * scale).all()
    # input gradient: the forward kernel with flipped, transposed weights
    dx = K.conv3x3_fwd_bf16(cl(dy), K.conv3x3_weight_bf16(w, True))
    sdx = F.conv_transpose2d(dy.float().abs(), w.float().abs(), padding=1) + 1e-3
    assert ((dx.float() - xr.grad).abs() <= 2 ** -7 * sdx).all()
    # weight gradient, accumulated into an existing bf16 gradient
    gw0 = (torch.randn(Co, C, 3, 3, generator=g) * 0.1).to(DEV, torch.bfloat16)
    gw = gw0.clone()
    K.conv3x3_wgrad_bf16_(cl(dy), cl(x), gw)
    want = gw0.float() + wr.grad
    sw = torch.nn.grad.conv2d_weight(x.float().abs(), w.shape, dy.float().abs(), padding=1) + gw0.float().abs() + 1e-3
    assert ((gw.float() - want).abs() <= 2 ** -7 * sw).all()


@pytest.mark.parametrize("N,C,Co,H,W,ks,st", [(4, 64, 128, 28, 28, 3, 2), (3, 128, 256, 14, 14, 3, 2),
                                               (2, 256, 512, 7, 7, 3, 2), (4, 64, 128, 28, 28, 1, 2),
                                               (2, 256, 512, 7, 7, 1, 2), (3, 64, 64, 9, 11, 1, 1),
                                               (2, 128, 64, 9, 7, 3, 2), (64, 128, 128, 28, 28, 3, 2),
                                               (5, 128, 256, 15, 8, 1, 2), (3, 64, 128, 10, 12, 3, 1)])
def test_strided_and_pointwise_conv(N, C, Co, H, W, ks, st):
    """All three passes of the general path against fp32 references; stride-2 input gradients run the
    parity-class kernel (conv_dgrad_s2_bf16), including odd sizes (7 -> 4) and the BN 128 tile
    (64 x 28 x 28), so no MIOpen convolution is left in a bf16 ResNet step."""
    g = torch.Generator(device="cpu").manual_seed(N + C + Co + H + ks + st)
    pd = (ks - 1) // 2
    conv = torch.nn.Conv2d(C, Co, ks, st, pd, bias=False).to(DEV, torch.bfloat16)
    x = cl(torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16)).requires_grad_(True)
    assert conv_ops.general_eligible(x, conv)
    y = conv_ops._ConvGeneralFn.apply(x, conv.weight, st, pd)
    yr = F.conv2d(x.detach().float(), conv.weight.detach().float(), stride=st, padding=pd)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    scale = F.conv2d(x.detach().float().abs(), conv.weight.detach().float().abs(), stride=st, padding=pd) + 1e-3
    assert ((y.float() - yr).abs() <= 2 ** -7 * scale).all()
    dy = cl(torch.randn(yr.shape, generator=g).to(DEV, torch.bfloat16))
    y.backward(dy)
    gwr = torch.nn.grad.conv2d_weight(x.detach().float(), conv.weight.shape, dy.float(), stride=st, padding=pd)
    sw = torch.nn.grad.conv2d_weight(x.detach().float().abs(), conv.weight.shape, dy.float().abs(), stride=st,
                                     padding=pd) + 1e-3
    assert ((conv.weight.grad.float() - gwr).abs() <= 2 ** -7 * sw).all()
    dxr = torch.nn.grad.conv2d_input(x.shape, conv.weight.detach().float(), dy.float(), stride=st, padding=pd)
    sdx = torch.nn.grad.conv2d_input(x.shape, conv.weight.detach().float().abs(), dy.float().abs(), stride=st,
                                     padding=pd) + 1e-3
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    assert ((x.grad.float() - dxr).abs() <= 2 ** -7 * sdx).all()


@pytest.mark.parametrize("N,Co,H,W", [(4, 64, 28, 28), (3, 32, 5, 9)])
def test_stem_conv_one_channel(N, Co, H, W):
    g = torch.Generator(device="cpu").manual_seed(N + Co + H)
    x = torch.randn(N, 1, H, W, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(Co, 1, 3, 3, generator=g) * 0.3).to(DEV, torch.bfloat16)
    dy = cl(torch.randn(N, Co, H, W, generator=g).to(DEV, torch.bfloat16))
    y = K.conv_c1_fwd_bf16(x, w)
    assert y.is_contiguous(memory_format=torch.channels_last)
    yr = F.conv2d(x.float(), w.float(), padding=1)
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    gw0 = (torch.randn(Co, 1, 3, 3, generator=g) * 0.1).to(DEV, torch.bfloat16)
    gw = gw0.clone()
    K.conv_c1_wgrad_bf16_(dy, x, gw)
    want = gw0.float() + torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), padding=1)
    sw = torch.nn.grad.conv2d_weight(x.float().abs(), w.shape, dy.float().abs(), padding=1) + gw0.float().abs()
    assert ((gw.float() - want).abs() <= 2 ** -7 * sw + 1e-3).all()
    conv = torch.nn.Conv2d(1, Co, 3, 1, 1, bias=False).to(DEV, torch.bfloat16)
    assert conv_ops.stem_eligible(x, conv)


def test_conv_autograd_function_matches_torch():
    conv = torch.nn.Conv2d(64, 128, 3, 1, 1, bias=False).to(DEV, torch.bfloat16)
    x = cl(torch.randn(2, 64, 8, 8, device=DEV, dtype=torch.bfloat16)).requires_grad_(True)
    assert conv_ops.hip_eligible(x, conv)
    y = conv_ops.conv2d(conv, x)
    y.float().square().sum().backward()
    gx, gw = x.grad.clone(), conv.weight.grad.clone()
    x2 = x.detach().float().requires_grad_(True)
    w2 = conv.weight.detach().float().requires_grad_(True)
    F.conv2d(x2, w2, padding=1).square().sum().backward()
    torch.testing.assert_close(gx.float(), x2.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(gw.float(), w2.grad, rtol=3e-2, atol=5e-1)


@pytest.mark.parametrize("relu,res", [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize("N,C,H,W", [(8, 64, 14, 14), (4, 512, 4, 4), (3, 24, 5, 7)])
def test_batchnorm_nhwc_train_matches_torch(N, C, H, W, relu, res):
    g = torch.Generator(device="cpu").manual_seed(N + C + H)
    x = cl(torch.randn(N, C, H, W, generator=g).mul(2).add(0.5).to(DEV, torch.bfloat16))
    r = cl(torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16)) if res else None
    dy = cl(torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16))
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
    ref = torch.nn.BatchNorm2d(C).to(DEV)
    ref.load_state_dict(bn.state_dict())
    bn = bn.to(torch.bfloat16)
    ref_w = ref.weight.detach().to(torch.bfloat16).float()  # same (bf16-rounded) parameters
    with torch.no_grad():
        ref.weight.copy_(ref_w)
        ref.bias.copy_(ref.bias.detach().to(torch.bfloat16).float())
    xr = x.float().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    yr = ref(xr)
    if res:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    yr.backward(dy.float())
    xx = x.clone().requires_grad_(True)
    rx = r.clone().requires_grad_(True) if res else None
    y = conv_ops.batch_norm(bn, xx, res=rx, relu=relu)
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yr.detach(), rtol=2e-2, atol=3e-2)
    y.backward(dy)
    torch.testing.assert_close(xx.grad.float(), xr.grad, rtol=3e-2, atol=3e-2)
    if res:
        torch.testing.assert_close(rx.grad.float(), rr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(bn.weight.grad.float(), ref.weight.grad, rtol=2e-2, atol=0.5)
    torch.testing.assert_close(bn.bias.grad.float(), ref.bias.grad, rtol=2e-2, atol=0.5)
    torch.testing.assert_close(bn.running_mean.float(), ref.running_mean, rtol=2e-2, atol=1e-2)
    torch.testing.assert_close(bn.running_var.float(), ref.running_var, rtol=2e-2, atol=1e-2)
    assert int(bn.num_batches_tracked) == 1
    # eval mode: running statistics
    bn.eval()
    ref.eval()
    with torch.no_grad():
        ye = conv_ops.batch_norm(bn, x, res=r, relu=relu)
        yre = ref(x.float()) + (r.float() if res else 0)
        if relu:
            yre = torch.relu(yre)
    torch.testing.assert_close(ye.float(), yre, rtol=2e-2, atol=3e-2)


def _tile_sums(y, rows=256):
    """per-256-pixel-tile channel sums of y and y^2 (the conv epilogue's BatchNorm partials), fp64"""
    Co = y.shape[1]
    f = y.permute(0, 2, 3, 1).reshape(-1, Co).double()
    pad = (-f.shape[0]) % rows
    f = torch.cat([f, f.new_zeros(pad, Co)])
    return f.view(-1, rows, Co).sum(1), f.square().view(-1, rows, Co).sum(1)


@pytest.mark.parametrize("N,C,Co,H,W,ks,st", [(4, 64, 128, 14, 14, 3, 1), (3, 128, 64, 7, 7, 3, 1),
                                               (2, 64, 64, 28, 28, 3, 1), (4, 64, 128, 28, 28, 3, 2),
                                               (2, 256, 512, 7, 7, 1, 2), (3, 64, 64, 9, 11, 1, 1)])
def test_conv_epilogue_addend_and_bn_partials(N, C, Co, H, W, ks, st):
    """The fused epilogue: y = bf16(conv + add) and the BatchNorm partials (per 256-pixel tile, sums of
    the stored y and y^2) equal the same sums taken over y afterwards; BatchNorm fed those partials
    equals BatchNorm running its own statistics pass."""
    g = torch.Generator(device="cpu").manual_seed(N * C + Co + H + ks + st)
    pd = (ks - 1) // 2
    x = cl(torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16))
    w = (torch.randn(Co, C, ks, ks, generator=g) * 0.05).to(DEV, torch.bfloat16)
    OH, OW = (H + 2 * pd - ks) // st + 1, (W + 2 * pd - ks) // st + 1
    add = cl(torch.randn(N, Co, OH, OW, generator=g).to(DEV, torch.bfloat16))
    part = torch.empty(K.conv_part_rows(N, OH, OW) * 2 * Co, device=DEV)
    if ks == 3 and st == 1:
        wt = K.conv3x3_weight_bf16(w, False)
        y0 = K.conv3x3_fwd_bf16(x, wt)
        y = K.conv3x3_fwd_bf16(x, wt, add=add, part=part)
    else:
        wt = K.conv3x3_weight_bf16(w, False) if ks == 3 else w
        y0 = K.conv_fwd_bf16(x, wt, ks, st, pd)
        y = K.conv_fwd_bf16(x, wt, ks, st, pd, add=add, part=part)
    # one rounding of (conv + add) vs bf16(conv) + add: two half-ulp (2^-8 relative) roundings apart
    want = y0.float() + add.float()
    assert ((y.float() - want).abs() <= 2 ** -7 * (y0.float().abs() + add.float().abs()) + 1e-6).all()
    s1, s2 = _tile_sums(y)
    p = part.view(-1, 2, Co).double()
    torch.testing.assert_close(p[:, 0], s1, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(p[:, 1], s2, rtol=1e-5, atol=1e-3)
    bn = torch.nn.BatchNorm2d(Co).to(DEV, torch.bfloat16)
    bn2 = torch.nn.BatchNorm2d(Co).to(DEV, torch.bfloat16)
    a = conv_ops.batch_norm(bn, y, relu=True, part=part)
    b = conv_ops.batch_norm(bn2, y, relu=True)
    torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(bn.running_var.float(), bn2.running_var.float(), rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("stride,cin,cout", [(1, 64, 64), (2, 64, 128), (2, 256, 512)])
def test_basic_block_fused_residual_gradient(stride, cin, cout):
    """ResNet BasicBlock on the HIP path (conv epilogue BatchNorm partials, residual input gradient
    added in conv1's dgrad epilogue through ResidualLink) against the same block in fp32 PyTorch."""
    from simple_distributed_machine_learning_amd.models.resnet import BasicBlock

    torch.manual_seed(stride + cin)
    blk = BasicBlock(cin, cout, stride).to(DEV)
    ref = BasicBlock(cin, cout, stride).to(DEV)
    ref.load_state_dict(blk.state_dict())
    blk = blk.to(torch.bfloat16)
    with torch.no_grad():  # same bf16-rounded parameters in the reference
        for pr, pb in zip(ref.parameters(), blk.parameters()):
            pr.copy_(pb.float())
    hw = 14 if cin == 64 else 7
    x0 = cl(torch.randn(8, cin, hw, hw, device=DEV).to(torch.bfloat16))
    xr = x0.float().requires_grad_(True)
    yr = F.relu(ref.bn2(ref.conv2(F.relu(ref.bn1(ref.conv1(xr))))) + (xr if ref.shortcut is None else ref.shortcut(xr)))
    dy = cl(torch.randn(yr.shape, device=DEV).to(torch.bfloat16))
    yr.backward(dy.float())
    grads = {}
    for fuse in (True, False):  # fused join vs autograd's add of the two gradients
        conv_ops.FUSE_RESIDUAL = fuse
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            fused0 = conv_ops.ResidualLink.fused
            y = blk(x)
            torch.testing.assert_close(y.float(), yr.detach(), rtol=5e-2, atol=5e-2)
            y.backward(dy)
            assert conv_ops.ResidualLink.fused == fused0 + (1 if fuse else 0)  # joined in the epilogue
        finally:
            conv_ops.FUSE_RESIDUAL = True
        grads[fuse] = (x.grad.float(), [p.grad.float().clone() for p in blk.parameters()])
    gf, gu = grads[True][0], grads[False][0]
    assert (gf - gu).norm() / gu.norm() < 1e-2  # one rounding of the sum instead of two
    err_f = float((gf - xr.grad).norm() / xr.grad.norm())
    err_u = float((gu - xr.grad).norm() / xr.grad.norm())
    assert err_f < 6e-2 and err_f <= 1.2 * err_u + 1e-3, (err_f, err_u)
    for (n, _), pf, pr in zip(blk.named_parameters(), grads[True][1], ref.parameters()):
        e = (pf - pr.grad).norm() / (pr.grad.norm() + 1e-6)
        assert e < 8e-2, (n, float(e))


@pytest.mark.parametrize("N,C,Co,H,W,ks,st", [(4, 64, 128, 28, 28, 3, 2), (3, 64, 64, 9, 11, 1, 1),
                                               (2, 256, 512, 7, 7, 3, 2), (3, 64, 128, 10, 12, 3, 1),
                                               (8, 64, 64, 14, 14, 3, 1)])
def test_wgrad_dma_loops_match_staged_loop(N, C, Co, H, W, ks, st, monkeypatch):
    """The opt-in LDS-DMA weight-gradient loops (2- and 3-stage rings; zero page for padding taps and pixels
    past a split) and the register-staged default run the same MFMA sequence: bit-identical gradients."""
    g = torch.Generator(device="cpu").manual_seed(N * C + Co + H + ks)
    pd = (ks - 1) // 2
    conv = torch.nn.Conv2d(C, Co, ks, st, pd, bias=False).to(DEV, torch.bfloat16)
    x = cl(torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16))
    y = F.conv2d(x.float(), conv.weight.float(), stride=st, padding=pd)
    dy = cl(torch.randn(y.shape, generator=g).to(DEV, torch.bfloat16))
    out = []
    try:
        for dma, stages in ((0, 2), (1, 2), (1, 3)):
            K.set_knob("CONV_WGRAD_DMA", dma)
            K.set_knob("CONV_WGRAD_STAGES", stages)
            conv.weight.grad = None
            xx = x.clone().requires_grad_(True)
            conv_ops._ConvGeneralFn.apply(xx, conv.weight, st, pd).backward(dy)
            out.append(conv.weight.grad.clone())
    finally:
        K.reset_knobs()
    assert torch.equal(out[0], out[1]) and torch.equal(out[0], out[2])


def test_resnet_last_stage_fused_head_matches_autograd_head(monkeypatch):
    """ResNetStage.head_fwd on ROCm (pool + fc + loss + backward in head_pool.hip) against the autograd head
    (SDML_RESNET_HEAD=aten): same loss, same stage gradients within bf16 tolerance."""
    from simple_distributed_machine_learning_amd.models import get_model_spec

    spec = get_model_spec("resnet18", 8, dtype=torch.bfloat16)
    res = []
    for mode in ("aten", "fused"):
        monkeypatch.setenv("SDML_RESNET_HEAD", mode)
        torch.manual_seed(0)
        m = spec.build_stage(7)
        m.stage_id, m.num_stages = 7, 8
        m = m.to(DEV, torch.bfloat16)
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        g = torch.Generator().manual_seed(1)
        x = torch.randn(64, 4, 4, 512, generator=g).to(DEV, torch.bfloat16)  # [N, H, W, C] boundary
        t = torch.randint(0, 10, (64,), generator=g).to(DEV)
        stats = torch.zeros(2, device=DEV)
        ctx = {}
        l, c, n = m.head_fwd(x, t, ctx, True, 1 / 64, stats=stats)
        if l is not None:
            stats[0] += l.float()
            stats[1] += c.float()
        dx = m.head_bwd(ctx)
        torch.cuda.synchronize()
        res.append((stats.clone(), dx.float(), [p.grad.float().clone() for p in m.parameters()]))
    (s0, d0, g0), (s1, d1, g1) = res
    assert float(s1[0]) == pytest.approx(float(s0[0]), rel=2e-2)
    torch.testing.assert_close(d1, d0, rtol=5e-2, atol=5e-2 * float(d0.abs().max()))
    for a, b in zip(g1, g0):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2 * float(b.abs().max()) + 1e-6)


def test_resnet_weight_layout_cache_is_exact_across_steps():
    """ops/conv.py caches the kernels' weight layouts within an optimizer step (keyed on the weight's storage,
    version and the optimizer's WEIGHT_GEN): 3 training steps of an 8-stage ResNet-18 with M = 4 micro-batches
    give bit-identical parameters with and without the cache (run in subprocesses: the switch is read at
    import)."""
    import os
    import subprocess
    import sys
    import textwrap

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent("""
        import sys, torch
        from simple_distributed_machine_learning_amd.data import SyntheticMNIST
        from simple_distributed_machine_learning_amd.models import get_model_spec
        from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh
        dev = torch.device("cuda", 0)
        mesh = init_mesh(pp=1, schedule_kind="gpipe", rank=0, world_size=1, device=dev)
        e = PipelineEngine(get_model_spec("resnet18", 8, dtype=torch.bfloat16), mesh, schedule_kind="gpipe",
                           num_microbatches=4, lr=0.05, momentum=0.9, seed=2)
        ds = SyntheticMNIST(64 * 3, seed=4, device=dev)
        for i in range(3):
            e.run(ds, 64 * i, 64, train=True)
        torch.cuda.synchronize()
        torch.save(e.flat.params.cpu(), sys.argv[1])
    """)
    outs = []
    for on in ("1", "0"):
        path = f"/tmp/sdml_wcache_{on}.pt"
        env = dict(os.environ, SDML_CONV_WCACHE=on, PYTHONPATH=root)
        r = subprocess.run([sys.executable, "-c", code, path], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(torch.load(path, weights_only=True))
    assert torch.equal(outs[0], outs[1])


def _bn_back_sums(dx, x, y, mean, rstd, gamma, beta, relu, rows=None):
    """fp64 per-channel sums of g = dx * mask and g * (x - mean) * rstd over rows of 256 pixels (rows=None: one sum
    over every pixel), the mask as batchnorm_nhwc.hip forms it (relu 1: y > 0; 2: x * sc + sh > 0, sc = gamma rstd)."""
    C = x.shape[1]
    f = lambda t: t.permute(0, 2, 3, 1).reshape(-1, C).double()  # noqa: E731
    g, xf = f(dx.float()), f(x.float())
    if relu == 1:
        g = torch.where(f(y.float()) > 0, g, torch.zeros_like(g))
    elif relu == 2:
        sc = gamma.float() * rstd
        sh = beta.float() - mean * sc
        g = torch.where(f(x.float() * sc.view(1, C, 1, 1) + sh.view(1, C, 1, 1)) > 0, g, torch.zeros_like(g))
    gx = g * (xf - mean.double()) * rstd.double()
    if rows is None:
        return g.sum(0), gx.sum(0)
    pad = (-g.shape[0]) % rows
    g, gx = torch.cat([g, g.new_zeros(pad, C)]), torch.cat([gx, gx.new_zeros(pad, C)])
    return g.view(-1, rows, C).sum(1), gx.view(-1, rows, C).sum(1)


@pytest.mark.parametrize("relu", [0, 1, 2])
@pytest.mark.parametrize("N,C,Co,H,W,ks,st", [(4, 64, 128, 14, 14, 3, 1), (2, 128, 64, 28, 28, 3, 1),
                                               (4, 64, 128, 28, 28, 3, 2), (3, 128, 256, 7, 7, 3, 2),
                                               (2, 64, 128, 9, 11, 3, 2)])
def test_dgrad_epilogue_bn_backward_partials(N, C, Co, H, W, ks, st, relu):
    """The input-gradient epilogue's BatchNorm backward statistics (conv_bf16.hip BnBack): dx is unchanged, the
    partial rows are the sums of g = dx * mask and g * xhat (per 256-pixel tile for the stride-1 kernel; in total
    for the stride-2 parity classes), and the BatchNorm backward fed them matches the one running its own pass."""
    g = torch.Generator(device="cpu").manual_seed(N * C + Co + H + st + relu)
    pd = (ks - 1) // 2
    x = cl(torch.randn(N, C, H, W, generator=g).mul(1.5).add(0.3).to(DEV, torch.bfloat16))  # the BatchNorm's input
    res = cl(torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16)) if relu == 1 else None
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV, torch.bfloat16)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV, torch.bfloat16)
    yb, mean, rstd = K.bn_nhwc_fwd(x, res, gamma, beta, None, None, 1e-5, 0.1, relu != 0)
    w = (torch.randn(Co, C, ks, ks, generator=g) * 0.05).to(DEV, torch.bfloat16)
    OH, OW = (H + 2 * pd - ks) // st + 1, (W + 2 * pd - ks) // st + 1
    dyc = cl(torch.randn(N, Co, OH, OW, generator=g).to(DEV, torch.bfloat16))  # the convolution's output gradient
    bnk = dict(bn_x=x, bn_y=yb if relu == 1 else None, bn_mean=mean, bn_rstd=rstd, bn_gamma=gamma, bn_beta=beta,
               bn_relu=relu)
    if st == 1:
        wd = K.conv3x3_weight_bf16(w, True)
        rows = K.conv_part_rows(N, H, W)
        part = torch.full((rows * 2 * C,), float("nan"), device=DEV)
        dx0 = K.conv3x3_fwd_bf16(dyc, wd)
        dx = K.conv3x3_fwd_bf16(dyc, wd, part=part, **bnk)
    else:
        rows = K.conv_dgrad_s2_part_rows(N, H, W, ks, pd)
        part = torch.full((rows * 2 * C,), float("nan"), device=DEV)
        dx0 = K.conv_dgrad_s2_bf16(dyc, w, H, W, pd)
        dx = K.conv_dgrad_s2_bf16(dyc, w, H, W, pd, part=part, **bnk)
    assert torch.equal(dx, dx0)
    p = part.view(rows, 2, C).double()
    assert torch.isfinite(p).all()  # every row written
    s1, s2 = _bn_back_sums(dx, x, yb, mean, rstd, gamma, beta, relu, rows=256 if st == 1 else None)
    if st == 1:
        torch.testing.assert_close(p[:, 0], s1, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(p[:, 1], s2, rtol=1e-4, atol=1e-3)
    else:
        torch.testing.assert_close(p[:, 0].sum(0), s1, rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(p[:, 1].sum(0), s2, rtol=1e-4, atol=1e-2)
    # BatchNorm backward from these partials vs its own statistics pass
    outs = []
    for pp in (part, None):
        gg = torch.zeros(C, device=DEV, dtype=torch.bfloat16)
        gb = torch.zeros(C, device=DEV, dtype=torch.bfloat16)
        d, dr = K.bn_nhwc_bwd(x, dx, yb if relu == 1 else None, mean, rstd, gamma, relu != 0, relu == 1, gg, gb, beta,
                              part=pp, part_rows=rows if pp is not None else 0)
        outs.append((d.float(), None if dr is None else dr.float(), gg.float(), gb.float()))
    (d1, r1, g1, b1), (d0, r0, g0, b0) = outs
    torch.testing.assert_close(d1, d0, rtol=1e-2, atol=1e-2 * float(d0.abs().max()))
    if relu == 1:
        assert torch.equal(r1, r0)
    torch.testing.assert_close(g1, g0, rtol=1e-2, atol=1e-2 * float(g0.abs().max()) + 1e-3)
    torch.testing.assert_close(b1, b0, rtol=1e-2, atol=1e-2 * float(b0.abs().max()) + 1e-3)


def test_resnet_stage_bn_backward_statistics_from_dgrad_epilogues():
    """A one-stage bf16 ResNet-18 forward + backward with BNBackLink (every bn1 from conv2's input-gradient epilogue,
    every BatchNorm closing a block or the stem from the next conv1's when the residual gradient was fused there)
    against the same step with the BatchNorm backward running its own statistics passes: same loss, gradients within
    bf16 tolerance."""
    from simple_distributed_machine_learning_amd.models import get_model_spec

    spec = get_model_spec("resnet18", 1, dtype=torch.bfloat16)
    res, fused = [], []
    try:
        for on in (True, False):
            conv_ops.FUSE_BN_BACK = on
            torch.manual_seed(0)
            m = spec.build_stage(0).to(DEV, torch.bfloat16)
            g = torch.Generator().manual_seed(3)
            x = torch.randn(32, 1, 28, 28, generator=g).to(DEV, torch.bfloat16)
            t = torch.randint(0, 10, (32,), generator=g).to(DEV)
            f0 = conv_ops.BNBackLink.fused
            out = m(x)
            loss = F.cross_entropy(out.float(), t)
            loss.backward()
            torch.cuda.synchronize()
            fused.append(conv_ops.BNBackLink.fused - f0)
            res.append((float(loss), [(n, p.grad.float().clone()) for n, p in m.named_parameters()]))
    finally:
        conv_ops.FUSE_BN_BACK = True
    # 8 bn1 (conv2's epilogue) + the stem's and the closing BatchNorms of blocks 0-6 whose next conv1 fused the
    # residual gradient (the downsampling blocks' taps may run after their conv1: then that one is not fused)
    assert fused[1] == 0 and 8 + 5 <= fused[0] <= 16, fused
    assert res[0][0] == pytest.approx(res[1][0], rel=1e-3)
    for (n, a), (_, b) in zip(res[0][1], res[1][1]):
        e = float((a - b).norm() / (b.norm() + 1e-6))
        assert e < 3e-2, (n, e)
