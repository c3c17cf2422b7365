"""The bf16x3-split fp32 GEMM engine (csrc/kernels/gemm_f32x3.hip) against fp32/fp64 PyTorch
references: every operand layout, every epilogue, the fused bias-gradient row sums and ReLU
masks, and an accuracy comparison with the exact-fp32 MFMA engine (gemm_f32.hip)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd import _native, ops  # noqa: E402

DEV = torch.device("cuda", 0)
K = _native.kernels()


def rnd(*shape, seed=0, lo=-1.0, hi=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.empty(shape).uniform_(lo, hi, generator=g).to(DEV)


def ref64(A, B):
    return (A.double() @ B.double().t())


def layout(A, km):
    return A.t().contiguous() if km else A


def test_x3_identity_asymmetric():
    # A = I with an asymmetric B: a transposed C/D map or a wrong fragment k order fails
    n = 256
    A = torch.eye(n, device=DEV)
    B = torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) / (n * n)
    for a_km in (False, True):
        for b_km in (False, True):
            C = torch.empty(n, n, device=DEV)
            K.gemm_f32x3(layout(A, a_km), layout(B, b_km), C, a_km, b_km, 0)
            torch.testing.assert_close(C, B.t().contiguous(), rtol=0, atol=0)


@pytest.mark.parametrize("a_km,b_km", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,Kd", [(256, 128, 784), (300, 132, 100), (1000, 260, 68), (64, 784, 2048), (8, 4, 4)])
def test_x3_layouts_fp32_accuracy(a_km, b_km, M, N, Kd):
    A, B = rnd(M, Kd, seed=1), rnd(N, Kd, seed=2)
    C = torch.full((M, N), float("nan"), device=DEV)
    K.gemm_f32x3(layout(A, a_km), layout(B, b_km), C, a_km, b_km, 0)
    want = ref64(A, B)
    err = (C.double() - want).abs()
    # fp32-level accuracy: bounded like an fp32 dot product, |err| <~ K * 2^-24 * sum|a||b|
    bound = Kd * 2.0 ** -24 * (A.abs().double() @ B.abs().double().t()) + 1e-30
    assert torch.isfinite(C).all()
    assert (err <= bound).all(), float((err / bound).max())


@pytest.mark.parametrize("Kd", [784, 4096])
def test_x3_error_matches_fp32_mfma(Kd):
    """Error vs fp64 of the split engine is within 2x of the exact fp32-input MFMA engine."""
    M, N = 512, 256
    A, B = rnd(M, Kd, seed=3), rnd(N, Kd, seed=4)
    C3 = torch.empty(M, N, device=DEV)
    Cf = torch.empty(M, N, device=DEV)
    K.gemm_f32x3(A, B, C3, False, False, 0)
    mode = K.gemm_f32_mode()
    try:
        K.gemm_f32_set_mode(0)
        K.gemm_f32(A, B, Cf, False, False, 0)
    finally:
        K.gemm_f32_set_mode(mode)
    want = ref64(A, B)
    e3 = (C3.double() - want).abs()
    ef = (Cf.double() - want).abs()
    assert e3.max() <= 2.0 * ef.max() + 1e-7, (float(e3.max()), float(ef.max()))
    assert e3.mean() <= 2.0 * ef.mean() + 1e-8, (float(e3.mean()), float(ef.mean()))


def test_x3_wide_dynamic_range():
    # terms spanning many binades: the split is exact for any normal-range value
    M, N, Kd = 256, 128, 512
    A = rnd(M, Kd, seed=5) * torch.exp2(rnd(M, Kd, seed=6, lo=-30, hi=30).round())
    B = rnd(N, Kd, seed=7) * torch.exp2(rnd(N, Kd, seed=8, lo=-30, hi=30).round())
    C = torch.empty(M, N, device=DEV)
    K.gemm_f32x3(A, B, C, False, False, 0)
    want = ref64(A, B)
    bound = Kd * 2.0 ** -24 * (A.abs().double() @ B.abs().double().t()) + 1e-30
    assert ((C.double() - want).abs() <= bound).all()


def test_x3_epilogues():
    M, N, Kd = 512, 256, 320
    A, B, bias = rnd(M, Kd, seed=9), rnd(N, Kd, seed=10), rnd(N, seed=11)
    want = (A.double() @ B.double().t()).float()
    C = torch.empty(M, N, device=DEV)
    K.gemm_f32x3(A, B, C, False, False, 1, bias)
    torch.testing.assert_close(C, want + bias, rtol=1e-5, atol=1e-5)
    K.gemm_f32x3(A, B, C, False, False, 2, bias)
    torch.testing.assert_close(C, torch.relu(want + bias), rtol=1e-5, atol=1e-5)
    C0 = rnd(M, N, seed=12)
    C = C0.clone()
    K.gemm_f32x3(A, B, C, False, False, 3)
    torch.testing.assert_close(C, C0 + want, rtol=1e-5, atol=1e-5)
    cm = rnd(M, N, seed=13)
    K.gemm_f32x3(A, B, C, False, False, 0, None, None, None, cm)
    torch.testing.assert_close(C, want * (cm > 0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("a_km", [False, True])
def test_x3_splitk_atomic_rowsum_amask(a_km):
    # the weight-gradient shape: gW[N, K] += (gy*mask)^T x, gb += colsum(gy*mask), split over M
    Mb, N, Kd = 20000, 128, 784
    gy, x, mask = rnd(Mb, N, seed=14), rnd(Mb, Kd, seed=15), rnd(Mb, N, seed=16)
    gz = gy * (mask > 0)
    gw0, gb0 = rnd(N, Kd, seed=17), rnd(N, seed=18)
    gw, gb = gw0.clone(), gb0.clone()
    if a_km:  # A(n, m) = gy[m][n] (k-major), B(k, m) = x[m][k] (k-major)
        K.gemm_f32x3(gy, x, gw, True, True, 4, None, gb, mask)
    else:
        K.gemm_f32x3(gy.t().contiguous(), x, gw, False, True, 4, None, gb, mask.t().contiguous())
    want_w = (gz.double().t() @ x.double()).float() + gw0
    want_b = gz.double().sum(0).float() + gb0
    torch.testing.assert_close(gw, want_w, rtol=1e-5, atol=2e-4)
    torch.testing.assert_close(gb, want_b, rtol=1e-5, atol=2e-4)


def test_linear_ops_route_to_x3_at_bench_shape():
    """ops.linear_relu_fwd / linear_relu_bwd at the headline shape run on the split engine and
    agree with an fp64 reference to fp32 accuracy."""
    assert K.gemm_f32_mode() == 1
    M, Kd, N = 16384, 784, 128
    x, w, b = rnd(M, Kd, seed=19, lo=0, hi=1), rnd(N, Kd, seed=20) * 0.05, rnd(N, seed=21) * 0.1
    y = ops.linear_relu_fwd(x, w, b)
    want = torch.relu(x.double() @ w.double().t() + b.double())
    assert ((y.double() - want).abs() <= 1e-5 * (1 + want.abs())).all()
    gy = rnd(M, N, seed=22) * 1e-3 * (y > 0)
    gw, gb = torch.zeros_like(w), torch.zeros_like(b)
    dx = ops.linear_relu_bwd(x, y, gy, w, gw, gb, need_dx=True, gy_masked=True, mask_dx=False)
    torch.testing.assert_close(gw, (gy.double().t() @ x.double()).float(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gb, gy.double().sum(0).float(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dx, (gy.double() @ w.double()).float(), rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("M,N", [(20000, 100), (4096, 128), (70000, 1024)])
def test_linear_fwd_presplit_weight(M, N):
    """x @ W^T with W pre-split into bf16 planes once per call (ragged row/column tiles)."""
    Kd = 784 if N != 1024 else 1024
    x, w, b = rnd(M, Kd, seed=23), rnd(N, Kd, seed=24) * 0.05, rnd(N, seed=25)
    y = ops.linear_relu_fwd(x, w, b)
    want = torch.relu(x.double() @ w.double().t() + b.double())
    bound = Kd * 2.0 ** -24 * (x.abs().double() @ w.abs().double().t() + b.double().abs()) + 1e-30
    assert ((y.double() - want).abs() <= bound).all()
    y2 = ops.linear_fwd(x, w, b)
    assert ((y2.double() - (x.double() @ w.double().t() + b.double())).abs() <= bound).all()


@pytest.mark.parametrize("M,N,Kd", [(70000, 1024, 1024), (20000, 136, 520)])
def test_linear_bwd_dx_presplit_transposed_weight(M, N, Kd):
    """dX = gz @ W with W^T pre-split into bf16 planes by the transposed split (ragged 64-tiles)."""
    x, w = rnd(M, Kd, seed=26), rnd(N, Kd, seed=27) * 0.05
    gy = rnd(M, N, seed=28) * 1e-2
    dx = ops.linear_relu_bwd(x, None, gy, w, None, None, need_dx=True, gy_masked=True, mask_dx=False)
    want = gy.double() @ w.double()
    bound = N * 2.0 ** -24 * (gy.abs().double() @ w.abs().double()) + 1e-30
    assert ((dx.double() - want).abs() <= bound).all()


# ---- uint8-pixel first layer (ToTensor fused into the GEMM) ----------------------------------

def pixels(M, Kd, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(0, 256, (M, Kd), generator=g, dtype=torch.uint8).to(DEV)


@pytest.mark.parametrize("M,N,Kd", [(131072, 128, 784), (4096 + 77, 128, 784), (5000, 1024, 784), (8192, 36, 96),
                                    (4096 + 77, 256, 816), (5000, 128, 96), (300, 128, 784)])
def test_linear_fwd_u8_matches_fp32_reference(M, N, Kd):
    x8 = pixels(M, Kd, 3)
    w, b = rnd(N, Kd, seed=4, lo=-0.05, hi=0.05), rnd(N, seed=5)
    y = K.linear_fwd_u8(x8, w, b, True, 1.0 / 255.0)
    xf = x8.double() / 255.0
    want = torch.relu(xf @ w.double().t() + b.double())
    bound = Kd * 2.0 ** -24 * (xf @ w.double().abs().t() + b.double().abs()) + 1e-30
    assert ((y.double() - want).abs() <= 2 * bound).all()
    # the fp32 ToTensor path (x.float() / 255 through the fp32 GEMM) agrees to fp32 rounding
    torch.testing.assert_close(y, ops.linear_relu_fwd(x8.float().div(255.0), w, b), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("flat", [False, True])
@pytest.mark.parametrize("M,N,Kd", [(131072, 128, 784), (4096 + 33, 128, 784), (6000, 1024, 784), (8192, 36, 96),
                                    (4096, 128, 784), (65536, 64, 784)])
def test_linear_wgrad_u8_matches_fp32_reference(M, N, Kd, flat):
    """flat: gw and gb adjacent in one buffer (the flat gradient layout), which selects mlp_u8.hip's
    one-split-per-dz-element kernel when M % 32 == 0; otherwise the bf16x3 engine kernel."""
    x8 = pixels(M, Kd, 6)
    gz = rnd(M, N, seed=7) * (rnd(M, N, seed=8) > 0).float()
    gw0, gb0 = rnd(N, Kd, seed=9), rnd(N, seed=10)
    if flat:
        buf = torch.cat([gw0.reshape(-1), gb0])
        gw, gb = buf[:N * Kd].view(N, Kd), buf[N * Kd:]
    else:
        gw, gb = gw0.clone(), gb0.clone()
    K.linear_wgrad_u8(x8, gz, gw, gb, 1.0 / 255.0)
    xf = x8.double() / 255.0
    want_w = gw0.double() + gz.double().t() @ xf
    want_b = gb0.double() + gz.double().sum(0)
    bound = M * 2.0 ** -24 * (gz.double().abs().t() @ xf + gw0.double().abs()) + 1e-30
    assert ((gw.double() - want_w).abs() <= 2 * bound).all(), float(((gw.double() - want_w).abs() / bound).max())
    torch.testing.assert_close(gb.double(), want_b, rtol=1e-5, atol=1e-3)


def test_u8_fwd_weight_planes_reproduce_w():
    """The forward's two fp16 planes of W * 2^8 (csrc/kernels/u8_planes.h) give W back to within one
    fp32 ulp for |W| >= 2^-9, to 2^-33 absolute below that, and overflow to inf (loudly) past
    the fp16 range; the SGD step's plane writer agrees with the split kernel."""
    N, Kd = 128, 784
    g = torch.Generator(device="cpu").manual_seed(31)
    mag = torch.pow(2.0, torch.empty(N, Kd).uniform_(-20, 7, generator=g))
    sign = torch.where(torch.rand(N, Kd, generator=g) < 0.5, -1.0, 1.0)
    w = (mag * sign).float().to(DEV)
    w[0, :4] = torch.tensor([0.0, -0.0, 255.0, -2.0 ** -9])
    kp = int(K.u8_fwd_kpad(Kd))
    planes = torch.zeros(int(K.u8_fwd_planes()), N, kp, dtype=torch.int16, device=DEV)
    x8 = pixels(4096, Kd, 32)
    K.linear_fwd_u8(x8, w, torch.zeros(N, device=DEV), False, 1.0 / 255.0, planes, False)
    hi = planes[0].view(torch.float16).double()
    lo = planes[1].view(torch.float16).double()
    assert torch.all(hi[:, Kd:] == 0) and torch.all(lo[:, Kd:] == 0)
    back = (hi + lo)[:, :Kd] / 256.0
    wd = w.double()
    err = (back - wd).abs()
    big = wd.abs() >= 2.0 ** -9
    assert torch.all(err[big] <= 2.0 ** -23 * wd.abs()[big])
    assert torch.all(err[~big] <= 2.0 ** -33)
    # the fused SGD step writes the same bits (lr = 0: the weights stay as they are)
    flat = torch.cat([w.reshape(-1), torch.zeros(4, device=DEV)])
    grad, buf = torch.zeros_like(flat), torch.zeros_like(flat)
    planes2 = torch.zeros_like(planes)
    ops.sgd_momentum_(flat, grad, buf, 0.0, 0.5, first=True, planes=(planes2, 0, N, Kd))
    assert torch.equal(planes.view(torch.float16), planes2.view(torch.float16))  # (the sign of a zero lo may differ)
    # past the fp16 range: a non-finite output, not a silent error
    w[3, 5] = 300.0
    y = K.linear_fwd_u8(x8, w, torch.zeros(N, device=DEV), False, 1.0 / 255.0)
    assert not torch.isfinite(y[:, 3]).all()


def test_u8_small_batch_falls_back_to_fp32():
    x8 = pixels(60, 784, 11)
    w, b = rnd(128, 784, seed=12, lo=-0.05, hi=0.05), rnd(128, seed=13)
    y = K.linear_fwd_u8(x8, w, b, True, 1.0 / 255.0)
    torch.testing.assert_close(y, ops.linear_relu_fwd(x8.float().div(255.0), w, b), rtol=1e-5, atol=1e-5)
    gz = rnd(60, 128, seed=14)
    gw, gb = torch.zeros(128, 784, device=DEV), torch.zeros(128, device=DEV)
    K.linear_wgrad_u8(x8, gz, gw, gb, 1.0 / 255.0)
    torch.testing.assert_close(gw, gz.t() @ (x8.float() / 255.0), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gb, gz.sum(0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M", [4096, 65536, 131072])
@pytest.mark.parametrize("C", [10, 2])
def test_wgrad_u8_from_factor_bit_identical(M, C):
    """The factored boundary gradient expanded inside the weight-gradient kernel (rotate placement,
    R > 1) gives bit for bit the gw/gb of head_dx_from_dl followed by linear_wgrad_u8 (same dz bound)."""
    N, Kd = 128, 784
    x8 = pixels(M, Kd, 21)
    h = rnd(M, N, seed=22).relu()
    dl = rnd(M, C, seed=23) * 1e-3
    w2 = rnd(C, N, seed=24) * 0.1
    g0 = rnd(N * Kd + N, seed=25)

    def flat():
        buf = g0.clone()
        return buf, buf[:N * Kd].view(N, Kd), buf[N * Kd:]

    dz_dev = ops.head_dx_from_dlogits(dl, w2, h, mask=True)
    amax = dz_dev.abs().amax().reshape(1)
    b1, gw1, gb1 = flat()
    ops.linear_wgrad_u8_dl(x8, dl, w2, h, gw1, gb1, amax=amax)
    b2, gw2, gb2 = flat()
    ops.linear_wgrad_u8(x8, dz_dev, gw2, gb2, amax=amax)
    assert torch.equal(b1, b2)
    # the workgroup-local bound (rotate placement: no amax) agrees with the fp64 reference as well
    b3, gw3, gb3 = flat()
    ops.linear_wgrad_u8_dl(x8, dl, w2, h, gw3, gb3)
    # and against the fp64 reference
    dz = (dl.double() @ w2.double()) * (h > 0).double()
    want = g0.double()[:N * Kd].view(N, Kd) + dz.t() @ (x8.double() / 255.0)
    for gwi, gbi in ((gw1, gb1), (gw3, gb3)):
        torch.testing.assert_close(gwi.double(), want, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(gbi.double(), g0.double()[N * Kd:] + dz.sum(0), rtol=1e-4, atol=1e-6)
