"""GPT-2 elementwise / embedding HIP kernels (gpt2_ops.hip) against PyTorch fp32 references: tanh-GELU
forward and backward, the token + position embedding gather, and its deterministic backward (bitwise
repeatable, equal to an fp64 scatter-add within bf16 rounding of the accumulation)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd import _native  # noqa: E402
from simple_distributed_machine_learning_amd.ops.transformer import embedding, gelu  # noqa: E402

DEV = torch.device("cuda", 0)
K = _native.kernels()


@pytest.mark.parametrize("n", [8, 4096 * 3072, 1000 * 8])
def test_gelu_fwd_bwd_match_torch(n):
    g = torch.Generator(device="cpu").manual_seed(n % 97)
    x = (torch.randn(n, generator=g) * 3).to(DEV, torch.bfloat16)
    gy = torch.randn(n, generator=g).to(DEV, torch.bfloat16)
    y = K.gelu_fwd_bf16(x)
    ref = F.gelu(x.float(), approximate="tanh")
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    # the same formula as PyTorch's bf16 kernels: at most one bf16 ulp apart
    yt = F.gelu(x, approximate="tanh")
    assert float((y.float() - yt.float()).abs().max()) <= float(yt.float().abs().max()) * 2 ** -7 + 1e-6
    xr = x.float().requires_grad_(True)
    F.gelu(xr, approximate="tanh").backward(gy.float())
    gx = K.gelu_bwd_bf16(gy, x, False)
    torch.testing.assert_close(gx.float(), xr.grad, rtol=1e-2, atol=1e-2)
    gx2 = gy.clone()
    K.gelu_bwd_bf16(gx2, x, True)
    assert torch.equal(gx2, gx)


def test_gelu_autograd_wrapper():
    x = torch.randn(64, 3072, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = gelu(x)
    y.sum().backward()
    xr = x.detach().float().requires_grad_(True)
    F.gelu(xr, approximate="tanh").sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,S,C,V", [(16, 1024, 768, 50257), (4, 16, 32, 97), (3, 7, 64, 5)])
def test_embedding_fwd_bwd(B, S, C, V):
    g = torch.Generator(device="cpu").manual_seed(B * S)
    tok = torch.randint(0, V, (B, S), generator=g).to(DEV)
    if V > 50:  # a heavily repeated token: one long segment
        tok[:, ::3] = 11
    wte = (torch.randn(V, C, generator=g) * 0.02).to(DEV, torch.bfloat16).requires_grad_(True)
    wpe = (torch.randn(S + 5, C, generator=g) * 0.02).to(DEV, torch.bfloat16).requires_grad_(True)
    out = embedding(tok, wte, wpe)
    want = F.embedding(tok, wte.detach()) + wpe.detach()[:S][None]
    assert torch.equal(out, want)
    gout = torch.randn(B, S, C, generator=g).to(DEV, torch.bfloat16)
    # flat-buffer style: the backward adds into preset bf16 grads in place
    wte.grad = torch.zeros_like(wte)
    wpe.grad = torch.zeros_like(wpe)
    out.backward(gout)
    gw1, gp1 = wte.grad.clone(), wpe.grad.clone()
    wte.grad.zero_()
    wpe.grad.zero_()
    embedding(tok, wte, wpe).backward(gout)
    assert torch.equal(wte.grad, gw1) and torch.equal(wpe.grad, gp1)  # deterministic
    ref_w = torch.zeros(V, C, dtype=torch.float64, device=DEV).index_add_(0, tok.reshape(-1),
                                                                        gout.reshape(-1, C).double())
    ref_p = gout.double().sum(0)
    torch.testing.assert_close(gw1.double(), ref_w, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(gp1[:S].double(), ref_p, rtol=2e-2, atol=2e-2)
    assert float(gp1[S:].abs().max()) == 0.0


def _ref_gelu(u):
    return F.gelu(u.float(), approximate="tanh")


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 64), (300, 776, 192), (4096, 2304, 768), (1000, 768, 3072)])
@pytest.mark.parametrize("b_kn", [False, True])
def test_gemm_bf16_layouts_match_fp32(M, N, Kd, b_kn):
    g = torch.Generator(device="cpu").manual_seed(M + N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(Kd, N, generator=g) if b_kn else torch.randn(N, Kd, generator=g)).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    Wf = W.float() if b_kn else W.float().t()
    ref = A.float() @ Wf
    C, _ = K.gemm_bf16(A, W, None, b_kn, 0)
    torch.testing.assert_close(C.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    if not b_kn:
        C, _ = K.gemm_bf16(A, W, bias, False, 1)
        torch.testing.assert_close(C.float(), ref + bias.float(), rtol=1e-2, atol=1e-2 * float(ref.abs().max()))


def test_gemm_bf16_identity_asymmetric():
    """A = I and an asymmetric B catch a transposed fragment or C map (guide §3)."""
    n = 256
    A = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    B = (torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) % 251 / 8).to(torch.bfloat16)
    C, _ = K.gemm_bf16(A, B, None, False, 0)  # A B^T
    assert torch.equal(C, B.t().contiguous())
    C, _ = K.gemm_bf16(A, B, None, True, 0)  # A B
    assert torch.equal(C, B)


def test_gemm_bf16_gelu_epilogues_match_unfused():
    g = torch.Generator(device="cpu").manual_seed(5)
    M, N, Kd = 512, 3072, 768
    x = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    y, u = K.gemm_bf16(x, w, b, False, 5)
    ub, _ = K.gemm_bf16(x, w, b, False, 1)
    assert torch.equal(u, ub)  # the pre-activation is the plain bias GEMM's output
    assert torch.equal(y, K.gelu_fwd_bf16(ub))  # and the activation is the standalone GELU kernel's
    # backward: dU = (dY W2) * gelu'(U), exactly the unfused GEMM + gelu_bwd pair
    w2 = (torch.randn(768, N, generator=g) * 0.05).to(DEV, torch.bfloat16)  # c_proj [768, 3072]
    gy = torch.randn(M, 768, generator=g).to(DEV, torch.bfloat16)
    du, _ = K.gemm_bf16(gy, w2, None, True, 6, u)
    da, _ = K.gemm_bf16(gy, w2, None, True, 0)
    assert torch.equal(du, K.gelu_bwd_bf16(da, u, False))
    # the gelu'-saving pair (7, 8): the same activation bits; aux = bf16(gelu'(U)); dU = bf16(aux * bf16(dY W2))
    ones = torch.ones_like(u)
    for t2 in (0, 1):
        K.set_knob("GEMM_BF16_T2", t2)
        try:
            y7, d7 = K.gemm_bf16(x, w, b, False, 7)
        finally:
            K.set_knob("GEMM_BF16_T2", 0)
        assert torch.equal(y7, y)
        assert torch.equal(d7, K.gelu_bwd_bf16(ones, u, False))
    for b_kn, w2x in ((True, w2), (False, w2.t().contiguous())):
        du8, _ = K.gemm_bf16(gy, w2x, None, b_kn, 8, d7)
        assert torch.equal(du8, (d7.float() * da.float()).to(torch.bfloat16))
    torch.testing.assert_close(du8.float(), K.gelu_bwd_bf16(da, u, False).float(), rtol=1.6e-2, atol=1e-2)


@pytest.mark.parametrize("save", ["grad", "u"])
def test_mlp_gelu_fused_matches_composed(save, monkeypatch):
    """GPT-2's MLP with the GELU fused into the GEMM epilogues (ops.linear._MLPFn) against
    c_proj(gelu(c_fc(x))) composed from separate kernels: forward and every gradient; the forward saving
    gelu'(U) (SDML_GELU_SAVE=grad, the default) or U."""
    from simple_distributed_machine_learning_amd.ops import linear as L
    from simple_distributed_machine_learning_amd.ops.linear import _MLPFn, linear

    monkeypatch.setattr(L, "_GELU_EPI", (7, 8) if save == "grad" else (5, 6))

    g = torch.Generator(device="cpu").manual_seed(9)
    T, C = 1024, 768
    x0 = torch.randn(2, T // 2, C, generator=g).to(DEV, torch.bfloat16)
    ps = [(torch.randn(4 * C, C, generator=g) * 0.02), (torch.randn(4 * C, generator=g) * 0.02),
          (torch.randn(C, 4 * C, generator=g) * 0.02), (torch.randn(C, generator=g) * 0.02)]
    ps = [p.to(DEV, torch.bfloat16) for p in ps]
    gy = torch.randn(2, T // 2, C, generator=g).to(DEV, torch.bfloat16)

    def run(fused):
        x = x0.clone().requires_grad_(True)
        w = [p.clone().requires_grad_(True) for p in ps]
        y = _MLPFn.apply(x, *w) if fused else linear(gelu(linear(x, w[0], w[1])), w[2], w[3])
        y.backward(gy)
        return [y] + [x.grad] + [t.grad for t in w]

    for a, b in zip(run(True), run(False)):
        scale = float(b.float().abs().max())
        torch.testing.assert_close(a.float(), b.float(), rtol=3e-2, atol=3e-2 * scale)


@pytest.mark.parametrize("M,N,Kd", [(256, 128, 64), (300, 776, 192), (4096, 2304, 768), (1000, 768, 3072)])
def test_gemm_bf16_t2_tiles_match_fp32_and_the_256_tile(M, N, Kd):
    """Knob GEMM_BF16_T2: the NT GEMM on 256 x 128 tiles of 4 waves (two workgroups per CU). Same products over
    the same 32-deep MFMAs as the 256 x 256 kernel's substeps: equal to it bit for bit, and to fp32 within bf16
    rounding; every epilogue (store, bias, bias + GELU) and the identity / asymmetric-B check."""
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    ref = A.float() @ W.float().t()
    outs = {}
    try:
        for t2 in (0, 1):
            K.set_knob("GEMM_BF16_T2", t2)
            C0, _ = K.gemm_bf16(A, W, None, False, 0)
            C1, _ = K.gemm_bf16(A, W, bias, False, 1)
            y, u = K.gemm_bf16(A, W, bias, False, 5)
            outs[t2] = (C0, C1, y, u)
            torch.testing.assert_close(C0.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
            torch.testing.assert_close(C1.float(), ref + bias.float(), rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
            assert torch.equal(u, C1) and torch.equal(y, K.gelu_fwd_bf16(C1))
        n = 256
        K.set_knob("GEMM_BF16_T2", 1)
        I = torch.eye(n, device=DEV, dtype=torch.bfloat16)
        B = (torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) % 251 / 8).to(torch.bfloat16)
        Ci, _ = K.gemm_bf16(I, B, None, False, 0)
        assert torch.equal(Ci, B.t().contiguous())
    finally:
        K.reset_knobs()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,Kd", [(256, 192, 64), (300, 776, 192), (4096, 768, 768), (1000, 2304, 3072)])
def test_gemm_bf16_192_wide_tiles_bit_identical_to_256(M, N, Kd):
    """Knob GEMM_BF16_N192: the 4-phase NT GEMM on 256 x 192 tiles (wave tile 128 x 48, chosen automatically where it
    fills the CUs' rounds better, e.g. N = 768 at 16384 rows). Every output element sums the same 32-deep MFMA products
    in the same k order as on 256 x 256 tiles: bit-identical for each epilogue, and equal to fp32 within bf16."""
    g = torch.Generator(device="cpu").manual_seed(M + 5 * N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    u_in = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    ref = A.float() @ W.float().t()
    outs = {}
    try:
        for n192 in (0, 1):
            K.set_knob("GEMM_BF16_N192", n192)
            C0, _ = K.gemm_bf16(A, W, None, False, 0)
            C1, _ = K.gemm_bf16(A, W, bias, False, 1)
            y, u = K.gemm_bf16(A, W, bias, False, 5)
            du, _ = K.gemm_bf16(A, W, None, False, 6, u_in)
            outs[n192] = (C0, C1, y, u, du)
            torch.testing.assert_close(C0.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    finally:
        K.reset_knobs()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,Kd", [(256, 192, 64), (3000, 776, 192), (4096, 768, 768), (1000, 2304, 3072),
                                    (5000, 3072, 128)])
def test_gemm_bf16_grouped_tile_order_bit_identical(M, N, Kd):
    """Knob GEMM_GROUP_M: the NT / NN GEMMs visit their tiles in groups of g m-tiles x every n-tile (ragged last
    group included) instead of M fastest. Only the order in which workgroups take tiles changes: bit-identical
    outputs for every epilogue, both tile widths and the NN layout."""
    g = torch.Generator(device="cpu").manual_seed(M + 11 * N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    Wkn = W.t().contiguous()
    bias = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    u_in = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    outs = {}
    try:
        for gm in (0, 3, 8):
            for n192 in (0, 1):
                K.set_knob("GEMM_GROUP_M", gm)
                K.set_knob("GEMM_BF16_N192", n192)
                C0, _ = K.gemm_bf16(A, W, None, False, 0)
                C1, _ = K.gemm_bf16(A, W, bias, False, 1)
                y, u = K.gemm_bf16(A, W, bias, False, 5)
                du, _ = K.gemm_bf16(A, W, None, False, 6, u_in)
                Cn, _ = K.gemm_bf16(A, Wkn, None, True, 0)
                outs[(gm, n192)] = (C0, C1, y, u, du, Cn)
    finally:
        K.reset_knobs()
    for key, o in outs.items():
        for a, b in zip(outs[(0, key[1])], o):
            assert torch.equal(a, b), key


@pytest.mark.parametrize("M,N,Kd", [(256, 192, 128), (3000, 776, 192), (4096, 768, 768), (16384, 3072, 768),
                                    (20000, 2304, 256), (2048, 50304, 128)])
def test_gemm_bf16_persistent_kernel_bit_identical(M, N, Kd):
    """Knob GEMM_BF16_PERSIST: one workgroup per CU walks its tiles with the half-tile stream running on into the
    next tile, and stores its epilogue from registers (8-B pieces). Same MFMAs in the same order and the same
    elementwise math as the one-tile-per-workgroup kernel: bit-identical for every epilogue (incl. the gelu'-saving
    pair), both tile widths, fewer tiles than CUs, several tiles per CU and a ragged last round."""
    g = torch.Generator(device="cpu").manual_seed(M + 17 * N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    u_in = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    outs = {}
    try:
        for pers in (0, 1):
            for n192 in (0, 1):
                K.set_knob("GEMM_BF16_PERSIST", pers)
                K.set_knob("GEMM_BF16_N192", n192)
                C0, _ = K.gemm_bf16(A, W, None, False, 0)
                C1, _ = K.gemm_bf16(A, W, bias, False, 1)
                y, u = K.gemm_bf16(A, W, bias, False, 5)
                ys, us = K.gemm_bf16(A, W, bias, False, 7)
                du, _ = K.gemm_bf16(A, W, None, False, 6, u_in)
                dm, _ = K.gemm_bf16(A, W, None, False, 8, u_in)
                outs[(pers, n192)] = (C0, C1, y, u, ys, us, du, dm)
    finally:
        K.reset_knobs()
    ref = A.float() @ W.float().t()
    torch.testing.assert_close(outs[(1, 0)][0].float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()) / 8)
    for key, o in outs.items():
        for i, (a, b) in enumerate(zip(outs[(0, key[1])], o)):
            assert torch.equal(a, b), (key, i)


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 64), (300, 776, 192), (4096, 768, 768), (1000, 2304, 3072),
                                    (16384, 3072, 768)])
def test_gemm_bf16_four_wave_kernel_matches_fp32(M, N, Kd):
    """Knob GEMM_BF16_W4: the NT GEMM on 4 waves of 128 x 128 (32x32x16 MFMAs, one barrier per K-step) against fp32 and
    against the 8-wave kernel, for every epilogue (a different MFMA shape sums each dot product in another internal
    order: equal within one bf16 rounding)."""
    g = torch.Generator(device="cpu").manual_seed(M + 13 * N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    u_in = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    ref = A.float() @ W.float().t()
    outs = {}
    try:
        for w4 in (0, 1):
            K.set_knob("GEMM_BF16_W4", w4)
            C0, _ = K.gemm_bf16(A, W, None, False, 0)
            C1, _ = K.gemm_bf16(A, W, bias, False, 1)
            y, u = K.gemm_bf16(A, W, bias, False, 5)
            du, _ = K.gemm_bf16(A, W, None, False, 6, u_in)
            outs[w4] = (C0, C1, y, u, du)
            torch.testing.assert_close(C0.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
            torch.testing.assert_close(C1.float(), ref + bias.float(), rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    finally:
        K.reset_knobs()
    for a, b in zip(outs[0], outs[1]):
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-2 * float(a.float().abs().max()) + 1e-3)


@pytest.mark.parametrize("M,N,Kd", [(256, 192, 64), (300, 776, 192), (4096, 768, 768), (1000, 2304, 3072)])
def test_gemm_bf16_transposed_accumulators(M, N, Kd):
    """Knob GEMM_BF16_TR: the 4-phase NT GEMM with the MFMA operands swapped, so each lane accumulates 4 consecutive
    columns of one output row (8-byte epilogue writes) - on both tile widths and every epilogue. The same products
    summed per output element; equal to the untransposed kernel within one bf16 rounding and to fp32 within bf16."""
    g = torch.Generator(device="cpu").manual_seed(M + 7 * N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV, torch.bfloat16)
    u_in = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    ref = A.float() @ W.float().t()
    outs = {}
    try:
        for n192 in (0, 1):
            for tr in (0, 1):
                K.set_knob("GEMM_BF16_N192", n192)
                K.set_knob("GEMM_BF16_TR", tr)
                C0, _ = K.gemm_bf16(A, W, None, False, 0)
                C1, _ = K.gemm_bf16(A, W, bias, False, 1)
                y, u = K.gemm_bf16(A, W, bias, False, 5)
                du, _ = K.gemm_bf16(A, W, None, False, 6, u_in)
                outs[(n192, tr)] = (C0, C1, y, u, du)
                torch.testing.assert_close(C0.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
                torch.testing.assert_close(C1.float(), ref + bias.float(), rtol=1e-2,
                                           atol=1e-2 * float(ref.abs().max()))
    finally:
        K.reset_knobs()
    for n192 in (0, 1):
        for a, b in zip(outs[(n192, 0)], outs[(n192, 1)]):
            # (one bf16 rounding apart at most: the MFMA may sum a dot product in another internal order)
            torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-2 * float(a.float().abs().max()))
    for a, b in zip(outs[(0, 1)], outs[(1, 1)]):
        assert torch.equal(a, b)


def test_transpose_batched_bf16():
    """transpose_batched_bf16: the hand GEMMs' W^T operands, every stale weight in one launch - exact transposes for
    shapes with partial 64 x 64 tiles, across more matrices than one launch descriptor holds."""
    g = torch.Generator(device="cpu").manual_seed(11)
    shapes = [(2304, 768), (768, 768), (776, 200), (8, 8), (3072, 768), (64, 136)] * 12  # 72 > kTransposeBatchMax
    src = [torch.randn(r, c, generator=g).to(DEV, torch.bfloat16) for r, c in shapes]
    dst = [torch.empty(c, r, device=DEV, dtype=torch.bfloat16) for r, c in shapes]
    K.transpose_batched_bf16(src, dst)
    torch.cuda.synchronize()
    for s_, d_ in zip(src, dst):
        assert torch.equal(d_, s_.t())


def test_hand_linear_wt_cache_batches_and_refreshes():
    """ops.linear._w_t: after a weight generation bump every known weight's W^T is re-derived (one batched launch) and
    equals the new transpose."""
    from simple_distributed_machine_learning_amd.ops import conv as conv_ops
    from simple_distributed_machine_learning_amd.ops import linear as lin

    ws = [torch.randn(r, c, device=DEV).to(torch.bfloat16) for r, c in [(2304, 768), (768, 3072), (768, 768)]]
    for w in ws:
        assert torch.equal(lin._w_t(w), w.t())
    conv_ops.bump_weight_generation()
    with torch.no_grad():
        for w in ws:
            w.mul_(2)  # (bumps the version too)
    t0 = lin._w_t(ws[0])
    assert torch.equal(t0, ws[0].t())
    for w in ws[1:]:  # refreshed by the same batched launch: cache hits now
        hit = conv_ops._cache_get(lin._WT, w)
        assert hit is not None and torch.equal(hit[1], w.t())


@pytest.mark.parametrize("T,C,V", [(2048, 768, 50257), (512, 64, 97)])
def test_lm_head_padded_vocabulary_matches_fp32(T, C, V):
    """GPT-2's lm_head on the hand-written kernels with the vocabulary padded in place (ops/linear.py _LMHeadFn;
    FlatParams row padding): logits, the cross-entropy's dlogits, the input gradient and the weight gradient against
    a PyTorch fp32 reference of the same op on the same bf16 operands; the pad rows of the weight gradient stay
    exactly zero."""
    from simple_distributed_machine_learning_amd.ops.linear import _LMHeadFn, lm_head
    from simple_distributed_machine_learning_amd.ops.transformer import cross_entropy_sum
    from simple_distributed_machine_learning_amd.utils.flat import FlatParams

    g = torch.Generator(device="cpu").manual_seed(V)
    head = torch.nn.Linear(C, V, bias=False)
    head.flat_row_multiple = {"weight": 64}
    with torch.no_grad():
        head.weight.copy_(torch.randn(V, C, generator=g) * 0.02)
    flat = FlatParams([(0, head)], DEV, torch.bfloat16)
    w = head.weight
    Vp = -(-V // 64) * 64
    assert w._sdml_rows_padded == Vp and w.grad is not None
    x = (torch.randn(T, C, generator=g)).to(DEV, torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, V, (T,), generator=g).to(DEV)
    logits = lm_head(x, w)
    assert logits.grad_fn is not None and type(logits.grad_fn).__name__.startswith("_LMHeadFn")
    assert logits.shape == (T, V) and logits.stride() == (Vp, 1)
    ref = x.detach().float() @ w.detach().float().t()
    torch.testing.assert_close(logits.float(), ref, rtol=2e-2, atol=2e-2)
    l, c, n, gl = cross_entropy_sum(logits.detach(), tgt, 1.0 / T, True)
    assert gl.stride() == (Vp, 1)
    pad = gl.as_strided((T, Vp), (Vp, 1))[:, V:]
    assert int((pad != 0).sum()) == 0  # the CE kernel zeroed the pad columns
    torch.autograd.backward(logits, gl)
    gref = gl.float()
    torch.testing.assert_close(x.grad.float(), gref @ w.detach().float(), rtol=2e-2, atol=2e-3)
    gw = flat.grads[:Vp * C].view(Vp, C)
    torch.testing.assert_close(gw[:V].float(), gref.t() @ x.detach().float(), rtol=2e-2, atol=2e-3)
    assert int((gw[V:] != 0).sum()) == 0 and int((flat.params[V * C:Vp * C] != 0).sum()) == 0


def test_side_stream_weight_gradients_are_joined_after_backward():
    """ops/side_stream.py: with the weight gradients on the side stream, a plain loss.backward() returns with the
    compute stream already waiting for them (the autograd-engine callback), so reading .grad right after it on the
    compute stream - no synchronise, no engine join - gives the same bits as the one-stream order. Three layers, so
    several side launches queue behind each other in one pass; the long first layer keeps the side stream busy."""
    from simple_distributed_machine_learning_amd.ops import linear as lin
    from simple_distributed_machine_learning_amd.ops import side_stream

    g = torch.Generator(device="cpu").manual_seed(5)
    dims = [(768, 3072), (3072, 768), (768, 768)]
    ws = [(torch.randn(o, i, generator=g) * 0.02).to(DEV, torch.bfloat16).requires_grad_(True) for i, o in dims]
    bs = [torch.zeros(o, device=DEV, dtype=torch.bfloat16).requires_grad_(True) for _, o in dims]
    x0 = torch.randn(16384, 768, generator=g).to(DEV, torch.bfloat16)
    grads = {}
    saved = side_stream.WGRAD_STREAM
    try:
        for on in (False, True):
            side_stream.WGRAD_STREAM = on
            for p in ws + bs:  # the flat-buffer form: .grad exists, the kernels accumulate into it in place
                p.grad = torch.zeros_like(p)
            torch.cuda.synchronize()
            y = x0
            for w, b in zip(ws, bs):
                y = lin.linear(y, w, b)
            y.float().square().mean().backward()
            grads[on] = [p.grad.clone() for p in ws + bs]  # on the compute stream, straight after backward
            torch.cuda.synchronize()
    finally:
        side_stream.WGRAD_STREAM = saved
        side_stream.join_side_streams()
    for a, b in zip(grads[False], grads[True]):
        assert torch.equal(a, b)
