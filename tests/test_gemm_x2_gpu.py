"""The two-fp16-plane fp32 GEMM engine (csrc/kernels/gemm_f16x2.hip) against fp64 references: the
split's representation bound, the forward (NT: bias + ReLU, per-wave maxima), the input gradient (NN:
ReLU mask of the layer input), the weight + bias gradient, and the documented error bound on operands
that span many binades (per-tensor scale: elements far below the tensor's maximum keep an absolute
error, not a relative one)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd import _native  # noqa: E402

DEV = torch.device("cuda", 0)
K = _native.kernels()


def rnd(*shape, seed=0, lo=-1.0, hi=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.empty(shape).uniform_(lo, hi, generator=g).to(DEV)


def inf_norm(x):
    return torch.linalg.vector_norm(x, float("inf")).reshape(1)


def split(x):
    return K.x2_split(x.contiguous(), inf_norm(x))


def unsplit(p, s):
    return (p[0].view(torch.float16).float() + p[1].view(torch.float16).float()) * s


def bound(A, B, Kd):
    """|C - AB^T| bound of the engine (gemm_f16x2.hip header): fp32 accumulation + the 2-plane
    representation (2^-23 relative per operand, 2^(E-39) absolute floor) + the dropped lo*lo term."""
    Ad, Bd = A.abs().double(), B.abs().double()
    ea = torch.frexp(A.abs().max().double())[1].item()
    eb = torch.frexp(B.abs().max().double())[1].item()
    rel = (Kd * 2.0 ** -24 + 2.0 ** -20) * (Ad @ Bd.t())
    absf = 2.0 ** (ea - 38) * Bd.sum(1)[None, :] + 2.0 ** (eb - 38) * Ad.sum(1)[:, None]
    return 2 * (rel + absf) + 1e-30


def test_x2_split_represents_x():
    x = rnd(333, 96, seed=1) * 7.0
    p, s = split(x)
    assert p.shape == (2, 333, 96) and p.dtype == torch.int16
    E = torch.frexp(x.abs().max())[1].item()
    assert float(s) == 2.0 ** (E - 14)
    back = unsplit(p, s)
    big = x.abs() >= 2.0 ** (E - 17)
    rel = ((back - x).abs() / x.abs().clamp_min(1e-30))[big]
    assert rel.max() <= 2.0 ** -22
    assert ((back - x).abs()[~big] <= 2.0 ** (E - 38)).all()


@pytest.mark.parametrize("M,N,Kd", [(1000, 512, 320), (4096, 1024, 1024)])
def test_x2_gemm_nt_bias_relu(M, N, Kd):
    A, B, bias = rnd(M, Kd, seed=2), rnd(N, Kd, seed=3), rnd(N, seed=4)
    pa, sa = split(A)
    pb, sb = split(B)
    C, wm = K.x2_gemm(pa, sa, pb, sb, False, None, False, None, True)
    want = A.double() @ B.double().t()
    err = (C.double() - want).abs()
    assert (err <= bound(A, B, Kd)).all()
    ef = ((A @ B.t()).double() - want).abs()  # the fp32 GEMM on the same data
    assert err.max() <= 4 * ef.max() + 1e-6, (float(err.max()), float(ef.max()))
    assert float(wm.max()) == float(C.abs().max())
    C2, _ = K.x2_gemm(pa, sa, pb, sb, False, bias, True)
    torch.testing.assert_close(C2, torch.relu(C + bias), rtol=0, atol=1e-6)


@pytest.mark.parametrize("M,N,Kd", [(700, 320, 256), (4096, 1024, 1024)])
def test_x2_gemm_nn_mask(M, N, Kd):
    # input gradient: dx[M, N] = dz[M, Kd] @ W[Kd, N], times (x > 0) of the layer input
    dz, W, x = rnd(M, Kd, seed=5), rnd(Kd, N, seed=6), rnd(M, N, seed=7)
    pd, sd = split(dz)
    pw, sw = split(W)
    C, wm = K.x2_gemm(pd, sd, pw, sw, True, None, False, x, True)
    want = (dz.double() @ W.double()) * (x > 0)
    err = (C.double() - want).abs()
    assert (err <= bound(dz, W.t(), Kd)).all()
    assert (C[x <= 0] == 0).all()
    assert float(wm.max()) == float(C.abs().max())


def test_x2_wide_dynamic_range():
    M, N, Kd = 512, 256, 512
    A = rnd(M, Kd, seed=8) * torch.exp2(rnd(M, Kd, seed=9, lo=-20, hi=20).round())
    B = rnd(N, Kd, seed=10) * torch.exp2(rnd(N, Kd, seed=11, lo=-20, hi=20).round())
    pa, sa = split(A)
    pb, sb = split(B)
    C, _ = K.x2_gemm(pa, sa, pb, sb, False)
    want = A.double() @ B.double().t()
    assert ((C.double() - want).abs() <= bound(A, B, Kd)).all()


@pytest.mark.parametrize("T,M,N", [(20000, 256, 512), (65536, 1024, 1024)])
def test_x2_wgrad_bias(T, M, N):
    dz, x = rnd(T, M, seed=12), rnd(T, N, seed=13)
    gw0, gb0 = rnd(M, N, seed=14), rnd(M, seed=15)
    gw, gb = gw0.clone(), gb0.clone()
    pd, sd = split(dz)
    px, sx = split(x)
    K.x2_wgrad_(pd, sd, px, sx, gw, gb)
    want = dz.double().t() @ x.double()
    err = (gw.double() - gw0.double() - want).abs()
    assert (err <= bound(dz.t(), x.t(), T) + 2.0 ** -23 * gw0.abs().double()).all()
    ef = ((dz.t() @ x).double() - want).abs()
    assert err.max() <= 4 * ef.max() + 1e-5, (float(err.max()), float(ef.max()))
    torch.testing.assert_close(gb.double(), gb0.double() + dz.double().sum(0), rtol=1e-5, atol=1e-4)


def test_x2_zero_operand():
    # an all-zero operand (bound 0) must give exact zeros, not NaN
    A, B = torch.zeros(256, 128, device=DEV), rnd(256, 128, seed=16)
    pa, sa = split(A)
    pb, sb = split(B)
    C, _ = K.x2_gemm(pa, sa, pb, sb, False)
    assert (C == 0).all()


def test_x2_split_t_is_the_split_of_the_transpose():
    w = rnd(320, 192, seed=17) * 3.0
    pt, st = K.x2_split_t(w, inf_norm(w))
    p, s = K.x2_split(w.t().contiguous(), inf_norm(w))
    assert torch.equal(pt, p) and torch.equal(st, s)


def test_x2_input_gradient_nt_matches_nn():
    # dx = dz @ W (W [N_out, K_in] = nn.Linear's weight) as NT against W^T's planes and as NN against W's
    M, Nout, Kin = 1024, 512, 384
    dz, W, x = rnd(M, Nout, seed=18), rnd(Nout, Kin, seed=19), rnd(M, Kin, seed=20)
    pd, sd = split(dz)
    pw, sw = split(W)
    pt, st = K.x2_split_t(W, inf_norm(W))
    c_nn, _ = K.x2_gemm(pd, sd, pw, sw, True, None, False, x)
    c_nt, _ = K.x2_gemm(pd, sd, pt, st, False, None, False, x)
    want = (dz.double() @ W.double()) * (x > 0)
    b = bound(dz, W.t(), Nout)
    assert ((c_nn.double() - want).abs() <= b).all()
    assert ((c_nt.double() - want).abs() <= b).all()


@pytest.mark.parametrize("T,M,N", [(16384, 1024, 1024), (4096, 520, 136)])
def test_x2_wgrad_dma_loop_matches_staged_loop(T, M, N, monkeypatch):
    # the LDS-DMA main loop (T % 64 == 0, default) vs the register-staged one: the same MFMA sequence and
    # slab order (bit-identical gw); the bias sums are split differently, so gb is checked against fp64
    dz, x = rnd(T, M, seed=21), rnd(T, N, seed=22)
    gw0, gb0 = rnd(M, N, seed=23), rnd(M, seed=24)
    pd, sd = split(dz)
    px, sx = split(x)
    out = []
    try:
        for mode in (1, 0):
            K.set_knob("WGRAD_DMA", mode)
            gw, gb = gw0.clone(), gb0.clone()
            K.x2_wgrad_(pd, sd, px, sx, gw, gb)
            out.append((gw, gb))
    finally:
        K.reset_knobs()
    assert torch.equal(out[0][0], out[1][0])
    for _, gb in out:
        torch.testing.assert_close(gb.double(), gb0.double() + dz.double().sum(0), rtol=1e-5, atol=1e-4)
