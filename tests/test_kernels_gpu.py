"""Numerics of every HIP kernel against a plain PyTorch fp32 reference (GPU only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd import _native, ops  # noqa: E402
from simple_distributed_machine_learning_amd.ops import reference as ref  # noqa: E402

DEV = torch.device("cuda", 0)
K = _native.kernels()


def rnd(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.empty(shape).uniform_(-1, 1, generator=g).to(DEV)


def close(a, b, rtol=2e-5, atol=2e-5):
    torch.testing.assert_close(a, b, rtol=rtol, atol=atol)


def test_mfma_layout_identity_asymmetric():
    # A = I, asymmetric B: catches a transposed C/D map (guide §3)
    n = 128
    A = torch.eye(n, device=DEV)
    B = torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) / (n * n)
    C = torch.empty(n, n, device=DEV)
    K.gemm_f32(A, B, C, False, False, 0)  # C = A @ B^T  (B given as [N,K])
    close(C, B.t().contiguous(), rtol=0, atol=0)
    K.gemm_f32(B, A, C, False, False, 0)
    close(C, B, rtol=0, atol=0)


@pytest.mark.parametrize("a_km,b_km", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,Kd", [(128, 128, 128), (60, 128, 784), (300, 50, 320), (1, 10, 4), (257, 129, 100)])
def test_gemm_layouts(a_km, b_km, M, N, Kd):
    A = rnd(M, Kd, seed=1)
    B = rnd(N, Kd, seed=2)
    A_in = A.t().contiguous() if a_km else A
    B_in = B.t().contiguous() if b_km else B
    C = torch.empty(M, N, device=DEV)
    K.gemm_f32(A_in, B_in, C, a_km, b_km, 0)
    close(C, A @ B.t(), rtol=1e-5, atol=1e-4)


def test_gemm_epilogues_and_splitk():
    M, N, Kd = 200, 130, 1000
    A, B, bias = rnd(M, Kd, seed=3), rnd(N, Kd, seed=4), rnd(N, seed=5)
    C = torch.empty(M, N, device=DEV)
    K.gemm_f32(A, B, C, False, False, 2, 1, bias)
    close(C, torch.relu(A @ B.t() + bias), atol=1e-4, rtol=1e-5)
    K.gemm_f32(A, B, C, False, False, 1, 1, bias)
    close(C, A @ B.t() + bias, atol=1e-4, rtol=1e-5)
    C0 = rnd(M, N, seed=6)
    C = C0.clone()
    K.gemm_f32(A, B, C, False, False, 3)
    close(C, C0 + A @ B.t(), atol=1e-4, rtol=1e-5)
    for splits in (1, 3, 8):
        C = C0.clone()
        rs = torch.zeros(M, device=DEV)
        K.gemm_f32(A, B, C, False, False, 4, splits, None, rs)
        close(C, C0 + A @ B.t(), atol=2e-4, rtol=1e-5)
        close(rs, A.sum(1), atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("M", [1, 7, 60, 128, 129, 1000, 4096])
@pytest.mark.parametrize("N,Kd", [(128, 784), (1024, 1024), (50, 320), (50, 322)])
def test_linear_relu_fwd_bwd(M, N, Kd):
    x, w, b = rnd(M, Kd, seed=7), rnd(N, Kd, seed=8) * 0.05, rnd(N, seed=9) * 0.1
    y = ops.linear_relu_fwd(x, w, b)
    yr = ref.linear_relu_fwd(x, w, b)
    close(y, yr, atol=1e-4, rtol=1e-5)
    gy = rnd(M, N, seed=10)
    gw, gb = rnd(N, Kd, seed=11), rnd(N, seed=12)
    gw_r, gb_r = gw.clone(), gb.clone()
    dx = ops.linear_relu_bwd(x, yr, gy, w, gw, gb, True)
    dx_r = ref.linear_relu_bwd(x, yr, gy, w, gw_r, gb_r, True)
    close(dx, dx_r, atol=2e-4, rtol=1e-5)
    close(gw, gw_r, atol=5e-4 * max(1, M / 1000), rtol=1e-5)
    close(gb, gb_r, atol=5e-4 * max(1, M / 1000), rtol=1e-5)


@pytest.mark.parametrize("M,N,Kd", [(60, 1024, 1024), (1, 1024, 1024), (60, 784, 1024), (200, 512, 2048)])
def test_skinny_split_k_epilogues(M, N, Kd):
    # few output tiles + long K: split-K (bias init / atomics / ReLU-or-mask pass) path
    x, w, b = rnd(M, Kd, seed=31).relu(), rnd(N, Kd, seed=32) * 0.05, rnd(N, seed=33) * 0.1
    close(ops.linear_relu_fwd(x, w, b), torch.relu(x @ w.t() + b), atol=1e-4, rtol=1e-5)
    close(ops.linear_fwd(x, w, b), x @ w.t() + b, atol=1e-4, rtol=1e-5)
    gz = rnd(M, N, seed=34)
    dx = ops.linear_relu_bwd(x, None, gz, w, None, None, True, gy_masked=True, mask_dx=True)
    close(dx, (gz @ w) * (x > 0), atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("M", [1, 60, 64, 1000, 70001])
@pytest.mark.parametrize("Kd,C", [(128, 10), (1024, 10), (50, 10), (128, 3)])
def test_head_logsoftmax_nll(M, Kd, C):
    x, w, b = rnd(M, Kd, seed=13), rnd(C, Kd, seed=14) * 0.1, rnd(C, seed=15)
    t = torch.randint(0, C, (M,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(0))
    scale = 1.0 / M
    gw, gb = torch.zeros(C, Kd, device=DEV), torch.zeros(C, device=DEV)
    gw_r, gb_r = gw.clone(), gb.clone()
    loss, correct, dx = ops.linear_logsoftmax_nll(x, w, b, t, gw, gb, scale, True)
    loss_r, correct_r, dx_r = ref.linear_logsoftmax_nll(x, w, b, t, gw_r, gb_r, scale, True)
    close(loss, loss_r, rtol=2e-5, atol=1e-3)
    assert int(correct) == int(correct_r)
    close(dx, dx_r, atol=2e-6, rtol=1e-4)
    close(gw, gw_r, atol=2e-5, rtol=1e-4)
    close(gb, gb_r, atol=2e-5, rtol=1e-4)
    # eval mode: no grads
    loss_e, correct_e, dx_e = ops.linear_logsoftmax_nll(x, w, b, t, None, None, 1.0, False)
    assert dx_e is None
    close(loss_e, loss_r, rtol=2e-5, atol=1e-3)


@pytest.mark.parametrize("M", [60, 3000, 131072])
@pytest.mark.parametrize("C", [10, 2])
def test_head_factored_boundary_grad_bit_identical(M, C):
    """The factored head (dlogits out) + head_dx_from_dl rebuild the masked boundary gradient bit for
    bit, with the same loss/correct/dW/db as the fused head that writes dx itself."""
    Kd = 128
    x, w, b = rnd(M, Kd, seed=41).relu(), rnd(C, Kd, seed=42) * 0.1, rnd(C, seed=43)
    t = torch.randint(0, C, (M,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    scale = 1.0 / M
    gw, gb, st = torch.zeros(C, Kd, device=DEV), torch.zeros(C, device=DEV), torch.zeros(2, device=DEV)
    gw2, gb2, st2 = gw.clone(), gb.clone(), st.clone()
    _, _, dx = ops.linear_logsoftmax_nll(x, w, b, t, gw, gb, scale, True, stats=st, mask_dx=True)
    dl = ops.linear_logsoftmax_nll_dl(x, w, b, t, gw2, gb2, scale, st2)
    assert dl.shape == (M, C)
    dx2 = ops.head_dx_from_dlogits(dl, w, x, mask=True)
    assert torch.equal(dx, dx2)
    assert torch.equal(gw, gw2) and torch.equal(gb, gb2) and torch.equal(st, st2)
    # and the factor is the reference dlogits
    _, _, dl_r = ref.linear_logsoftmax_nll_dl(x, w, b, t, torch.zeros_like(gw), torch.zeros_like(gb), scale)
    close(dl, dl_r, atol=1e-7, rtol=1e-4)


@pytest.mark.parametrize("first", [True, False])
@pytest.mark.parametrize("wd,damp,nest", [(0.0, 0.0, False), (1e-4, 0.1, False), (0.0, 0.0, True)])
def test_sgd_momentum(first, wd, damp, nest):
    n = 4096 + 64
    p, g, buf = rnd(n, seed=16), rnd(n, seed=17), rnd(n, seed=18)
    p_r, buf_r = p.clone(), buf.clone()
    if nest:
        damp = 0.0
    ops.sgd_momentum_(p, g, buf, 0.1, 0.5, damp, wd, nest, first)
    ref.sgd_momentum_(p_r, g, buf_r, 0.1, 0.5, damp, wd, nest, first)
    close(p, p_r, atol=1e-6, rtol=1e-6)
    close(buf, buf_r, atol=1e-6, rtol=1e-6)


def test_synth_device_matches_host():
    from simple_distributed_machine_learning_amd.data import SyntheticMNIST

    for mode in ("learnable", "random"):
        a = SyntheticMNIST(777, seed=5, device=DEV, mode=mode, offset=123)
        b = SyntheticMNIST(777, seed=5, device="cpu", mode=mode, offset=123)
        assert torch.equal(a.y.cpu(), b.y)
        assert torch.equal(a.x.cpu(), b.x), (a.x.cpu() - b.x).abs().max()


@pytest.mark.parametrize("first", [True, False])
def test_sgd_mixed_bf16(first):
    n = 8192 + 64
    master = rnd(n, seed=20)
    p = master.to(torch.bfloat16)
    g = rnd(n, seed=21).to(torch.bfloat16)
    buf = rnd(n, seed=22)
    m_r, b_r, g_r = master.clone(), buf.clone(), g.float()
    ops.sgd_momentum_mixed_(master, p, g, buf, 0.1, 0.5, 0.0, 0.0, False, first, True)
    ref.sgd_momentum_(m_r, g_r, b_r, 0.1, 0.5, 0.0, 0.0, False, first)
    close(master, m_r, atol=1e-6, rtol=1e-6)
    close(buf, b_r, atol=1e-6, rtol=1e-6)
    assert torch.equal(p, m_r.to(torch.bfloat16))
    assert float(g.float().abs().sum()) == 0.0


@pytest.mark.parametrize("first", [True, False])
def test_sgd_mixed_two_chunk_variant_bit_identical(first):
    """Knob SGD_MIXED_V: the two-chunks-per-trip form and the nontemporal-store form of the mixed SGD write the same
    bits as the one-chunk form (n spans several grid strides plus a partial one, so both loops and the tail run)."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    n = 8192 * 256 * 8 * 2 + 8 * 1000 + 64  # > 2 strides of the 8192-block grid, odd remainder
    outs = []
    try:
        for v in (0, 1, 2):
            K.set_knob("SGD_MIXED_V", v)
            master = rnd(n, seed=40)
            p = master.to(torch.bfloat16)
            g = rnd(n, seed=41).to(torch.bfloat16)
            buf = rnd(n, seed=42)
            ops.sgd_momentum_mixed_(master, p, g, buf, 0.1, 0.5, 0.0, 1e-4, False, first, True)
            assert float(g.float().abs().sum()) == 0.0
            outs.append((master, p, buf))
    finally:
        K.reset_knobs()
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("rows,V", [(7, 97), (64, 50257), (33, 1000), (5, 4096), (3, 131073), (2, 7), (9, 50257 * 2)])
def test_cross_entropy_bf16(rows, V):
    from simple_distributed_machine_learning_amd.ops.transformer import cross_entropy_sum

    z = (rnd(rows, V, seed=30) * 4).to(torch.bfloat16)
    t = torch.randint(0, V, (rows,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    l, c, n, g = cross_entropy_sum(z, t, 0.5, True)
    zf = z.float().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(zf, t, reduction="sum")
    (lr_ * 0.5).backward()
    close(l, lr_.detach(), rtol=1e-4, atol=1e-3)
    assert int(c) == int((zf.argmax(1) == t).sum()) and n == rows
    close(g.float(), zf.grad, rtol=2e-2, atol=2e-3)  # bf16 output rounding


@pytest.mark.parametrize("rows,D", [(1, 768), (1000, 768), (37, 64), (8, 3072)])
def test_layernorm_bf16(rows, D):
    from simple_distributed_machine_learning_amd.ops.transformer import layer_norm

    x = (rnd(rows, D, seed=31) * 3 + 0.5).to(torch.bfloat16).requires_grad_(True)
    w = (1 + 0.1 * rnd(D, seed=32)).to(torch.bfloat16).requires_grad_(True)
    b = (0.1 * rnd(D, seed=33)).to(torch.bfloat16).requires_grad_(True)
    y = layer_norm(x, w, b)
    gy = rnd(rows, D, seed=34).to(torch.bfloat16)
    y.backward(gy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
    yr.backward(gy.float())
    close(y.float(), yr, rtol=2e-2, atol=2e-2)
    close(x.grad.float(), xr.grad, rtol=2e-2, atol=3e-2)
    close(w.grad.float(), wr.grad, rtol=2e-2, atol=max(3e-2, 1e-3 * rows))
    close(b.grad.float(), br.grad, rtol=2e-2, atol=max(3e-2, 1e-3 * rows))


@pytest.mark.parametrize("B,S,H", [(1, 64, 1), (2, 128, 2), (1, 200, 3), (2, 1024, 12), (1, 33, 1)])
def test_flash_attention_fwd_bwd(B, S, H):
    from simple_distributed_machine_learning_amd.ops.transformer import causal_attention

    C = 64 * H
    qkv = (rnd(B, S, 3 * C, seed=40) * 1.5).to(torch.bfloat16).requires_grad_(True)
    y = causal_attention(qkv, H)
    gy = rnd(B, S, C, seed=41).to(torch.bfloat16)
    y.backward(gy)
    # fp32 reference (math path) on the same bf16 inputs
    x = qkv.detach().float().requires_grad_(True)
    q, k, v = x.split(C, dim=2)
    q, k, v = (t.view(B, S, H, 64).transpose(1, 2) for t in (q, k, v))
    att = (q @ k.transpose(-1, -2)) / 8.0
    mask = torch.ones(S, S, device=DEV, dtype=torch.bool).tril()
    att = att.masked_fill(~mask, float("-inf")).softmax(-1)
    yr = (att @ v).transpose(1, 2).reshape(B, S, C)
    yr.backward(gy.float())
    close(y.float(), yr, rtol=2e-2, atol=2e-2)
    close(qkv.grad.float(), x.grad, rtol=5e-2, atol=5e-2)


@pytest.mark.parametrize("B,S,H", [(1, 64, 1), (1, 200, 3), (2, 1024, 12), (1, 33, 1), (1, 300, 2)])
def test_flash_attention_dkdv_two_key_tiles_per_wave_bit_identical(B, S, H):
    """The dK/dV kernel with two 32-key tiles per wave (256 keys per workgroup, one wave per SIMD; knob ATTN_DKDV_KT=2)
    runs every key tile's MFMA chains in the same order as one tile per wave: bit-identical gradients (ragged S
    included: the last workgroup's second tile may hold no valid key)."""
    from simple_distributed_machine_learning_amd import _native
    from simple_distributed_machine_learning_amd.ops.transformer import causal_attention

    K = _native.kernels()
    C = 64 * H
    qkv0 = (rnd(B, S, 3 * C, seed=42) * 1.5).to(torch.bfloat16)
    gy = rnd(B, S, C, seed=43).to(torch.bfloat16)
    grads = []
    try:
        for kt in (1, 2):
            K.set_knob("ATTN_DKDV_KT", kt)
            qkv = qkv0.clone().requires_grad_(True)
            causal_attention(qkv, H).backward(gy)
            torch.cuda.synchronize()
            grads.append(qkv.grad.clone())
    finally:
        K.reset_knobs()
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("B,S,H", [(2, 1024, 3), (1, 333, 2), (2, 97, 1)])
def test_flash_attention_forward_two_query_subblocks_bit_identical(B, S, H):
    """The forward with two 32-query sub-blocks per wave (256 queries per workgroup; knob ATTN_FWD_QS=2) runs each
    sub-block's score, softmax and PV chain in the same order as one sub-block per wave: bit-identical outputs and
    gradients (the backward reads the forward's LSE), ragged S included."""
    from simple_distributed_machine_learning_amd import _native
    from simple_distributed_machine_learning_amd.ops.transformer import causal_attention

    K = _native.kernels()
    C = 64 * H
    qkv0 = (rnd(B, S, 3 * C, seed=44) * 1.5).to(torch.bfloat16)
    gy = rnd(B, S, C, seed=45).to(torch.bfloat16)
    res = []
    try:
        for qs in (1, 2, 3):  # 3: two sub-blocks per wave in 2-wave workgroups
            K.set_knob("ATTN_FWD_QS", qs)
            qkv = qkv0.clone().requires_grad_(True)
            y = causal_attention(qkv, H)
            y.backward(gy)
            torch.cuda.synchronize()
            res.append((y.detach().clone(), qkv.grad.clone()))
    finally:
        K.reset_knobs()
    for y, g in res[1:]:
        assert torch.equal(res[0][0], y) and torch.equal(res[0][1], g)


def test_fused_relu_mask_protocol():
    # head: dx *= (x > 0); linear bwd: skip the gy mask, mask dx by (x > 0)
    M, Kd, C = 1000, 128, 10
    x = torch.relu(rnd(M, Kd, seed=50))
    w, b = rnd(C, Kd, seed=51) * 0.1, rnd(C, seed=52)
    t = torch.randint(0, C, (M,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    gw, gb = torch.zeros(C, Kd, device=DEV), torch.zeros(C, device=DEV)
    _, _, dx = ops.linear_logsoftmax_nll(x, w, b, t, gw, gb, 1.0 / M, True, mask_dx=True)
    _, _, dx_r = ref.linear_logsoftmax_nll(x, w, b, t, gw.clone(), gb.clone(), 1.0 / M, True)
    close(dx, dx_r * (x > 0), atol=2e-6, rtol=1e-4)
    N, K2 = 256, 512
    x2 = torch.relu(rnd(M, K2, seed=53))
    w2 = rnd(N, K2, seed=54) * 0.05
    y2 = ref.linear_relu_fwd(x2, w2, torch.zeros(N, device=DEV))
    gz = rnd(M, N, seed=55) * (y2 > 0)
    gw2, gb2 = torch.zeros_like(w2), torch.zeros(N, device=DEV)
    dx2 = ops.linear_relu_bwd(x2, y2, gz, w2, gw2, gb2, True, gy_masked=True, mask_dx=True)
    gw2r, gb2r = torch.zeros_like(w2), torch.zeros(N, device=DEV)
    dx2r = ref.linear_relu_bwd(x2, y2, gz, w2, gw2r, gb2r, True) * (x2 > 0)
    close(dx2, dx2r, atol=2e-4, rtol=1e-5)
    close(gw2, gw2r, atol=5e-4, rtol=1e-5)
    close(gb2, gb2r, atol=5e-4, rtol=1e-5)


# ---- reference CNN fused stages (ref_cnn.hip) vs PyTorch fp32 with the same dropout masks ----
def _cnn_params(seed=0):
    torch.manual_seed(seed)
    c1, c2 = torch.nn.Conv2d(1, 10, 5), torch.nn.Conv2d(10, 20, 5)
    f1, f2 = torch.nn.Linear(320, 50), torch.nn.Linear(50, 10)
    mods = [m.to(DEV) for m in (c1, c2, f1, f2)]
    for m in mods:
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
    return mods


@pytest.mark.parametrize("B,drop", [(60, False), (60, True), (7, True), (130, True)])
def test_ref_cnn_stage0(B, drop):
    c1, c2, _, _ = _cnn_params(1)
    x = rnd(B, 1, 28, 28, seed=2).abs()
    seed, p = 123456789, 0.5
    y, saved = ops.ref_cnn_stage0_fwd(x, c1, c2, seed, p, drop, save=True)
    y_eval, none = ops.ref_cnn_stage0_fwd(x, c1, c2, seed, p, drop)
    assert none is None and torch.equal(y, y_eval)
    ps = [t.detach().clone().requires_grad_(True) for t in (c1.weight, c1.bias, c2.weight, c2.bias)]
    y_ref = ref.ref_cnn_stage0(x, *ps, seed, 0, p, drop)
    close(y, y_ref.detach(), rtol=1e-5, atol=1e-5)
    gout = rnd(B, 320, seed=3)
    ops.ref_cnn_stage0_bwd(x, c1, c2, y, gout, saved, seed, p, drop)
    gs = torch.autograd.grad(y_ref, ps, gout)
    for got, want in zip((c1.weight.grad, c1.bias.grad, c2.weight.grad, c2.bias.grad), gs):
        close(got, want, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("B,drop,train", [(60, True, True), (60, False, True), (200, True, True),
                                          (33, True, False)])
def test_ref_cnn_stage1(B, drop, train):
    _, _, f1, f2 = _cnn_params(4)
    x = rnd(B, 320, seed=5).relu()
    tgt = torch.randint(0, 10, (B,), generator=torch.Generator().manual_seed(6)).to(DEV)
    seed, p, scale = 987654321, 0.5, 1.0 / B
    stats = torch.zeros(2, device=DEV)
    dx = ops.ref_cnn_stage1(x, f1, f2, tgt, seed, p, drop, scale, stats, train)
    xx = x.clone().requires_grad_(True)
    ps = [t.detach().clone().requires_grad_(True) for t in (f1.weight, f1.bias, f2.weight, f2.bias)]
    logp = ref.ref_cnn_stage1_logp(xx, *ps, seed, 0, p, drop)
    loss = torch.nn.functional.nll_loss(logp, tgt, reduction="sum")
    close(stats[0], loss.detach(), rtol=1e-5, atol=1e-4)
    assert int(stats[1]) == int((logp.argmax(1) == tgt).sum())
    if not train:
        assert dx is None
        return
    gs = torch.autograd.grad(loss * scale, [xx] + ps)
    close(dx, gs[0], rtol=1e-4, atol=1e-6)
    for got, want in zip((f1.weight.grad, f1.bias.grad, f2.weight.grad, f2.bias.grad), gs[1:]):
        close(got, want, rtol=1e-4, atol=1e-5)


def test_ref_cnn_dropout_mask_statistics():
    # the kernel's masks: ~p dropped, whole channels in stage 0 (Dropout2d semantics)
    c1, c2, _, _ = _cnn_params(7)
    x = rnd(512, 1, 28, 28, seed=8).abs()
    y0, _ = ops.ref_cnn_stage0_fwd(x, c1, c2, 1, 0.5, False)
    y1, _ = ops.ref_cnn_stage0_fwd(x, c1, c2, 1, 0.5, True)
    ch0 = y0.view(512, 20, 16)
    ch1 = y1.view(512, 20, 16)
    dropped = (ch1.abs().sum(-1) == 0) & (ch0.abs().sum(-1) > 0)
    frac = dropped.float().sum() / (ch0.abs().sum(-1) > 0).float().sum()
    assert 0.45 < float(frac) < 0.55
    kept = ~dropped & (ch0.abs().sum(-1) > 0)
    close(ch1[kept], 2 * ch0[kept], rtol=1e-5, atol=1e-5)


# ---- gradient-accumulating Linear / LayerNorm (ops/linear.py, transformer.hip) -------------
@pytest.mark.parametrize("M,N", [(4096, 768), (5, 50), (1000, 3072), (64, 50257)])
def test_bias_grad_bf16(M, N):
    gy = rnd(M, N, seed=41).to(torch.bfloat16)
    gb = rnd(N, seed=42).to(torch.bfloat16)
    want = gb.float() + gy.float().sum(0)
    K.bias_grad_bf16_(gy, gb)
    close(gb.float(), want, rtol=1e-2, atol=2e-2 * max(1.0, (M / 1000) ** 0.5))


@pytest.mark.parametrize("with_bias", [True, False])
def test_fused_linear_accumulates_into_grad(with_bias):
    from simple_distributed_machine_learning_amd.ops.linear import Linear

    torch.manual_seed(3)
    lin = Linear(96, 200, bias=with_bias).to(DEV, torch.bfloat16)
    ref_lin = torch.nn.Linear(96, 200, bias=with_bias).to(DEV, torch.float32)
    ref_lin.load_state_dict({k: v.float() for k, v in lin.state_dict().items()})
    for p in lin.parameters():  # pre-existing (flat-buffer style) grads get ADDED to
        p.grad = torch.full_like(p, 0.25)
    for mb in range(2):  # two micro-batches accumulate
        x = rnd(3, 40, 96, seed=50 + mb).to(torch.bfloat16).requires_grad_(True)
        gy = rnd(3, 40, 200, seed=60 + mb).to(torch.bfloat16)
        y = lin(x)
        y.backward(gy)
        xr = x.detach().float().requires_grad_(True)
        yr = ref_lin(xr)
        yr.backward(gy.float())
        close(y.float(), yr.detach(), rtol=2e-2, atol=3e-2)
        close(x.grad.float(), xr.grad, rtol=2e-2, atol=3e-2)
    close(lin.weight.grad.float(), 0.25 + ref_lin.weight.grad, rtol=2e-2, atol=1e-1)
    if with_bias:
        close(lin.bias.grad.float(), 0.25 + ref_lin.bias.grad, rtol=2e-2, atol=1e-1)
    # no pre-existing grads: ordinary autograd accumulation
    lin2 = Linear(96, 200, bias=with_bias).to(DEV, torch.bfloat16)
    x = rnd(7, 96, seed=70).to(torch.bfloat16)
    lin2(x).float().sum().backward()
    assert lin2.weight.grad is not None and torch.isfinite(lin2.weight.grad.float()).all()


def test_layernorm_accumulates_into_grad():
    from simple_distributed_machine_learning_amd.ops.transformer import LayerNorm

    ln = LayerNorm(768).to(DEV, torch.bfloat16)
    with torch.no_grad():
        ln.weight.copy_(rnd(768, seed=80).to(torch.bfloat16))
        ln.bias.copy_(rnd(768, seed=81).to(torch.bfloat16))
    ln.weight.grad = torch.full_like(ln.weight, 0.5)
    ln.bias.grad = torch.full_like(ln.bias, -0.5)
    x = rnd(4, 64, 768, seed=82).to(torch.bfloat16).requires_grad_(True)
    gy = rnd(4, 64, 768, seed=83).to(torch.bfloat16)
    ln(x).backward(gy)
    xr = x.detach().float().requires_grad_(True)
    wr = ln.weight.detach().float().requires_grad_(True)
    br = ln.bias.detach().float().requires_grad_(True)
    torch.nn.functional.layer_norm(xr, (768,), wr, br, 1e-5).backward(gy.float())
    close(x.grad.float(), xr.grad, rtol=3e-2, atol=5e-2)
    close(ln.weight.grad.float(), 0.5 + wr.grad, rtol=2e-2, atol=2e-1)
    close(ln.bias.grad.float(), -0.5 + br.grad, rtol=2e-2, atol=2e-1)


@pytest.mark.parametrize("flat_grads", [True, False])
def test_add_layernorm_fused_matches_unfused(flat_grads):
    """(x + h, LN(x + h)) in one pass; backward adds the residual-path gradient inside the LN kernel."""
    from simple_distributed_machine_learning_amd.ops.transformer import LayerNorm, add_layer_norm

    ln = LayerNorm(768).to(DEV, torch.bfloat16)
    with torch.no_grad():
        ln.weight.copy_(rnd(768, seed=84).to(torch.bfloat16))
        ln.bias.copy_(rnd(768, seed=85).to(torch.bfloat16))
    if flat_grads:
        ln.weight.grad = torch.zeros_like(ln.weight)
        ln.bias.grad = torch.zeros_like(ln.bias)
    x = rnd(3, 50, 768, seed=86).to(torch.bfloat16).requires_grad_(True)
    h = rnd(3, 50, 768, seed=87).to(torch.bfloat16).requires_grad_(True)
    g_xs = rnd(3, 50, 768, seed=88).to(torch.bfloat16)
    g_y = rnd(3, 50, 768, seed=89).to(torch.bfloat16)
    xs, y = add_layer_norm(x, h, ln)
    assert torch.equal(xs, x.detach() + h.detach())  # the unfused bf16 add, bit for bit
    torch.autograd.backward([xs, y], [g_xs, g_y])
    xr = (x.detach().float() + h.detach().float()).to(torch.bfloat16).float().requires_grad_(True)
    wr = ln.weight.detach().float().requires_grad_(True)
    br = ln.bias.detach().float().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (768,), wr, br, 1e-5)
    torch.autograd.backward([xr, yr], [g_xs.float(), g_y.float()])
    close(y.float(), yr.detach(), rtol=2e-2, atol=3e-2)
    close(x.grad.float(), xr.grad, rtol=3e-2, atol=5e-2)
    assert torch.equal(x.grad, h.grad)
    gw = ln.weight.grad
    close(gw.float(), wr.grad, rtol=2e-2, atol=2e-1)


@pytest.mark.parametrize("T,M,N", [(16384, 3072, 768), (4096, 768, 768), (1000, 2304, 776), (64, 8, 16), (300, 520, 136)])
def test_wgrad_bf16(T, M, N):
    """gw (bf16) += gy^T x, split-token MFMA GEMM vs an fp64 reference of the same bf16 inputs."""
    g = torch.Generator(device="cpu").manual_seed(T + M)
    gy = torch.randn(T, M, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(T, N, generator=g).to(DEV, torch.bfloat16)
    gw0 = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    gw = gw0.clone()
    K.wgrad_bf16_(gy, x, gw)
    want = gw0.double() + gy.double().t() @ x.double()
    scale = (gy.double().abs().t() @ x.double().abs()) + gw0.double().abs()
    err = (gw.double() - want).abs()
    assert (err <= 2 ** -7 * scale + 1e-6).all(), float((err / scale).max())
    gw2 = gw0.clone()
    K.wgrad_bf16_(gy, x, gw2)
    assert torch.equal(gw, gw2)  # deterministic (fixed-order slab reduction, no atomics)
    # fused bias gradient: gb += column sums of gy
    gb0 = torch.randn(M, generator=g).to(DEV, torch.bfloat16)
    gw3, gb = gw0.clone(), gb0.clone()
    K.wgrad_bf16_(gy, x, gw3, gb)
    assert torch.equal(gw3, gw)
    want_b = gb0.double() + gy.double().sum(0)
    scale_b = gy.double().abs().sum(0) + gb0.double().abs()
    assert ((gb.double() - want_b).abs() <= 2 ** -7 * scale_b + 1e-6).all()


@pytest.mark.parametrize("T,M,N", [(16384, 2304, 768), (4096, 768, 3072), (2368, 520, 136), (64, 8, 16)])
def test_wgrad_bf16_dma_loop_matches_staged_loop(T, M, N, monkeypatch):
    """The LDS-DMA main loop (T % 64 == 0, the default) and the register-staged one run the same MFMA
    sequence per split and the same slab order: bit-identical gw. The bias sums are split differently
    (the DMA loop spreads them over the column tiles), so gb is checked against fp64."""
    g = torch.Generator(device="cpu").manual_seed(T + N)
    gy = torch.randn(T, M, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(T, N, generator=g).to(DEV, torch.bfloat16)
    gw0 = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    gb0 = torch.randn(M, generator=g).to(DEV, torch.bfloat16)
    K = _native.kernels()
    out = []
    try:
        for mode in (1, 0):
            K.set_knob("WGRAD_DMA", mode)
            gw, gb = gw0.clone(), gb0.clone()
            K.wgrad_bf16_(gy, x, gw, gb)
            gw2 = gw0.clone()
            K.wgrad_bf16_(gy, x, gw2)
            out.append((gw, gb, gw2))
    finally:
        K.reset_knobs()
    assert torch.equal(out[0][0], out[1][0])
    want_b = gb0.double() + gy.double().sum(0)
    scale_b = gy.double().abs().sum(0) + gb0.double().abs()
    for o in out:
        assert ((o[1].double() - want_b).abs() <= 2 ** -7 * scale_b + 1e-6).all()
    assert torch.equal(out[0][2], out[1][2]) and torch.equal(out[0][0], out[0][2])
    want = gw0.double() + gy.double().t() @ x.double()
    scale = (gy.double().abs().t() @ x.double().abs()) + gw0.double().abs()
    assert ((out[0][0].double() - want).abs() <= 2 ** -7 * scale + 1e-6).all()


@pytest.mark.parametrize("M", [60, 70001])
def test_head_stats_init_overwrites(M):
    """stats_init: the head overwrites a garbage-filled stats tensor with its own totals (the engine's
    per-step stats then need no zero-fill launch), on both the dx and the factored head."""
    Kd, C = 128, 10
    x, w, b = rnd(M, Kd, seed=51).relu(), rnd(C, Kd, seed=52) * 0.1, rnd(C, seed=53)
    t = torch.randint(0, C, (M,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
    want = torch.zeros(2, device=DEV)
    ops.linear_logsoftmax_nll(x, w, b, t, torch.zeros(C, Kd, device=DEV), torch.zeros(C, device=DEV), 1.0 / M, True,
                              stats=want, mask_dx=True)
    got = torch.full((2,), float("nan"), device=DEV)
    ops.linear_logsoftmax_nll(x, w, b, t, torch.zeros(C, Kd, device=DEV), torch.zeros(C, device=DEV), 1.0 / M, True,
                              stats=got, mask_dx=True, stats_init=True)
    assert torch.equal(got, want)
    got2 = torch.full((2,), float("nan"), device=DEV)
    ops.linear_logsoftmax_nll_dl(x, w, b, t, torch.zeros(C, Kd, device=DEV), torch.zeros(C, device=DEV), 1.0 / M,
                                 got2, stats_init=True)
    assert torch.equal(got2, want)
