"""The uint8 first layer and the classifier head fused into one kernel (mlp_u8.hip u8_fwd_head) and the
weight gradient reading ReLU bits instead of h: bit-identity with the unfused kernels where the
arithmetic is the same (dl, the mask, gW1/gb1), fp32 agreement where only the summation blocking
differs (gW2/gb2, loss), engine-level agreement of the fused and unfused steps, the fused optimizer step
against optimizer.step() (bitwise, every SGD option), and the documented error bound of the weight
gradient's fp16 dz planes on adversarial data (one row dominating its block). Reference ops:
/root/reference/simple_distributed.py:63-64, :75-79 (fc1, relu, fc2, log_softmax), :111 (nll_loss),
:100-104 (SGD)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from simple_distributed_machine_learning_amd import ops  # noqa: E402
from simple_distributed_machine_learning_amd.data import SyntheticMNIST  # noqa: E402
from simple_distributed_machine_learning_amd.models import get_model_spec  # noqa: E402
from simple_distributed_machine_learning_amd.parallel import PipelineEngine, init_mesh  # noqa: E402

DEV = torch.device("cuda", 0)
N, KD = 128, 784


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1).mul_(scale).to(DEV)


def pixels(M, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(0, 256, (M, KD), generator=g, dtype=torch.uint8).to(DEV)


def _problem(M, C, seed=0):
    x8 = pixels(M, seed)
    w1, b1 = rnd(N, KD, seed=seed + 1, scale=0.05), rnd(N, seed=seed + 2, scale=0.1)
    w2, b2 = rnd(C, N, seed=seed + 3, scale=0.2), rnd(C, seed=seed + 4, scale=0.1)
    g = torch.Generator(device="cpu").manual_seed(seed + 5)
    tgt = torch.randint(0, C, (M,), generator=g).to(DEV)
    return x8, w1, b1, w2, b2, tgt


@pytest.mark.parametrize("M", [4096, 4096 + 100, 131072])
@pytest.mark.parametrize("C", [10, 2])
@pytest.mark.parametrize("defer", [False, True])
def test_fused_forward_head_matches_unfused(M, C, defer):
    x8, w1, b1, w2, b2, tgt = _problem(M, C)
    scale = 1.0 / M
    # unfused: forward (h + its bits) -> standalone MFMA head returning dl
    mask_u = torch.empty(M, N // 32, dtype=torch.int32, device=DEV)
    h = ops.linear_relu_fwd_u8(x8, w1, b1, None, 0, mask_out=mask_u)
    gw_u, gb_u = torch.zeros(C, N, device=DEV), torch.zeros(C, device=DEV)
    st_u = torch.empty(2, device=DEV)
    dl_u = ops.linear_logsoftmax_nll_dl(h, w2, b2, tgt, gw_u, gb_u, scale, st_u, stats_init=True)
    # fused
    cache = ops.PlaneCache(w1)
    dl_f = torch.full((M, C), float("nan"), device=DEV)
    mask_f = torch.zeros(M, N // 32, dtype=torch.int32, device=DEV)
    gw_f, gb_f = torch.zeros(C, N, device=DEV), torch.zeros(C, device=DEV)
    st_f = torch.full((2,), 123.0, device=DEV)
    bound, pend = ops.linear_relu_head_u8(x8, w1, b1, cache, 0, w2, b2, tgt, gw_f, gb_f, scale, st_f, True, dl_f,
                                          mask_f, defer=defer)
    if defer:
        assert pend is not None and pend.pending
        pend.run()
    torch.cuda.synchronize()
    assert torch.equal(mask_u, ops.relu_bits(h))
    assert torch.equal(mask_f, mask_u)
    assert torch.equal(dl_f, dl_u)  # same h, same MFMA sequence (head_tile.h)
    torch.testing.assert_close(gw_f, gw_u, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(gb_f, gb_u, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(st_f[0], st_u[0], rtol=1e-5, atol=1e-3)
    assert float(st_f[1]) == float(st_u[1])
    assert float(bound.max()) >= float((dl_f.double() @ w2.double()).abs().max())
    # and against an fp64 reference of the whole head
    z = (x8.double() / 255.0) @ w1.double().t() + b1.double()
    hr = z.clamp_min(0)
    logits = hr @ w2.double().t() + b2.double()
    p = torch.softmax(logits, 1)
    want = (p - torch.nn.functional.one_hot(tgt, C).double()) * scale
    torch.testing.assert_close(dl_f.double(), want, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(gw_f.double(), want.t() @ hr, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("M", [4096, 65536])
def test_wgrad_from_relu_bits_bit_identical_to_h(M):
    C = 10
    x8 = pixels(M, 31)
    h = rnd(M, N, seed=32).relu()
    dl = rnd(M, C, seed=33, scale=1e-3)
    w2 = rnd(C, N, seed=34, scale=0.1)
    g0 = rnd(N * KD + N, seed=35)
    bits = ops.relu_bits(h)
    for amax in (None, (dl.abs().sum(1).max() * w2.abs().max() * 2).reshape(1)):
        bufs = []
        for act in (h, bits):
            b = g0.clone()
            ops.linear_wgrad_u8_dl(x8, dl, w2, act, b[:N * KD].view(N, KD), b[N * KD:], amax=amax)
            bufs.append(b)
        assert torch.equal(bufs[0], bufs[1])


def test_wgrad_dz_planes_error_bound_with_a_dominating_row():
    """One row's |dl| is 2^20 times its neighbours': the block's dz bound (hence the fp16 plane scale)
    is set by that row, and the small rows' dz fall to the planes' absolute floor. The documented bound
    (README "Two fp16 planes"): each dz element keeps one fp32 ulp above 2^(E-15) and an absolute error
    below 2^(E-39) otherwise, |dz| < 2^E. The weight gradient must stay within that, plus fp32
    accumulation."""
    M, C = 8192, 10
    x8 = pixels(M, 41)
    h = rnd(M, N, seed=42).relu()
    dl = rnd(M, C, seed=43, scale=2.0 ** -20)
    dl[1234] = rnd(C, seed=44)  # ~2^20 x the others
    w2 = rnd(C, N, seed=45, scale=0.5)
    g = torch.zeros(N * KD + N, device=DEV)
    ops.linear_wgrad_u8_dl(x8, dl, w2, ops.relu_bits(h), g[:N * KD].view(N, KD), g[N * KD:])
    dz = (dl.double() @ w2.double()) * (h > 0).double()
    xf = x8.double() / 255.0
    want = dz.t() @ xf
    E = torch.ceil(torch.log2(2 * dl.abs().sum(1).max().double() * w2.abs().max().double())) + 1
    per_elem = torch.maximum(dz.abs() * 2.0 ** -23, torch.full_like(dz, float(2.0 ** (E - 39))))
    bound = per_elem.t() @ xf + 1e-5 * (dz.abs().t() @ xf) + 1e-30
    err = (g[:N * KD].view(N, KD).double() - want).abs()
    assert bool((err <= bound).all()), float((err / bound).max())
    # the small rows' contribution survives: the error is far below what they add
    only_big = dz[1234:1235].t() @ xf[1234:1235]
    assert float(err.max()) < 0.05 * float((want - only_big).abs().max())


def _engine(M, lr=0.1, momentum=0.5, wd=0.0, damp=0.0, nesterov=False):
    mesh = init_mesh(pp=1, schedule_kind="rotate", rank=0, world_size=1, device=DEV)
    spec = get_model_spec("mlp", 2)
    e = PipelineEngine(spec, mesh, schedule_kind="rotate", num_microbatches=M, lr=lr, momentum=momentum,
                       weight_decay=wd, seed=3)
    e.optimizer.dampening, e.optimizer.nesterov = damp, nesterov
    return e


def _train(e, steps=3, B=16384):
    ds = SyntheticMNIST(B * steps, seed=5, device=DEV, pixels="u8")
    losses = []
    for s in range(steps):
        r = e.run(ds, s * B, B, train=True)
        losses.append(float(r.loss_sum) / r.count)
    torch.cuda.synchronize()
    return losses


@pytest.mark.parametrize("M", [1, 2])
def test_engine_fused_head_step_matches_unfused(M, monkeypatch):
    monkeypatch.setenv("SDML_FUSE_HEAD", "0")
    e0 = _engine(M)
    l0 = _train(e0)
    monkeypatch.setenv("SDML_FUSE_HEAD", "1")
    e1 = _engine(M)
    l1 = _train(e1)
    assert getattr(e1.stages[0], "fused_head_calls", 0) == 3 * M  # every wave went through the fused kernel
    assert getattr(e0.stages[0], "fused_head_calls", 0) == 0
    assert l1 == pytest.approx(l0, rel=1e-5)
    torch.testing.assert_close(e1.flat.params, e0.flat.params, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("M", [1, 2])
def test_slab_reduce_geometries_bitwise_equal(M):
    """Knob U8_SLAB_COLS: the weight-gradient slab reduction (+ head reduction + fused SGD) with one lane per float4
    column (64 per block) or two (32 per block, each lane half of a wave's split partial) adds the same numbers in
    the same order: bitwise equal parameters, momentum and weight planes after 3 engine steps."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    runs = []
    try:
        for cols in (64, 32):
            K.set_knob("U8_SLAB_COLS", cols)
            e = _engine(M)
            losses = _train(e)
            runs.append((losses, e.flat.params.clone(), e.optimizer.momentum_buffer.clone(),
                         e.stages[0].plane_cache.planes.clone()))
    finally:
        K.reset_knobs()
    (l0, p0, b0, c0), (l1, p1, b1, c1) = runs
    assert l0 == l1
    assert torch.equal(p0, p1) and torch.equal(b0, b1) and torch.equal(c0, c1)


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("opt", [dict(), dict(momentum=0.0), dict(wd=1e-4), dict(damp=0.1), dict(nesterov=True)])
def test_fused_optimizer_step_bitwise_equals_optimizer_step(M, opt, monkeypatch):
    """the SGD update applied inside the last reduction launch (FusedSGD.fused_args) against
    the separate optimizer.step() launch - same fp32 operations in the same order, so bitwise equal
    parameters, momentum buffers and uint8 forward weight planes."""
    runs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("SDML_FUSED_STEP", fused)
        e = _engine(M, **opt)
        _train(e)
        cache = e.stages[0].plane_cache
        runs.append((e.flat.params.clone(), e.optimizer.momentum_buffer.clone() if e.optimizer.momentum else None,
                     cache.planes.clone()))
    (p0, b0, c0), (p1, b1, c1) = runs
    assert torch.equal(p0, p1)
    assert (b0 is None and b1 is None) or torch.equal(b0, b1)
    assert torch.equal(c0, c1)


def test_small_batch_forward_keeps_the_plane_cache_current():
    """A uint8 forward on a batch the uint8 kernel does not take (< 4096 rows: ToTensor + fp32 GEMM) still
    refreshes a stale weight-plane cache, because ops.linear_relu_fwd_u8 marks it current afterwards and
    a later fused forward+head reads it (the rotate placement runs the cross rows of a wave that way)."""
    g = torch.Generator(device="cpu").manual_seed(4)
    w = (torch.rand(128, 784, generator=g) - 0.5).mul_(0.1).to(DEV)
    b = torch.rand(128, generator=g).to(DEV)
    x = torch.randint(0, 256, (2048, 784), generator=g, dtype=torch.uint8).to(DEV)
    cache, ref = ops.PlaneCache(w), ops.PlaneCache(w)
    ops.linear_relu_fwd_u8(x, w, b, cache, 0)
    ops.linear_relu_fwd_u8(torch.cat([x, x]), w, b, ref, 0)  # 4096 rows: the kernel path splits into its cache
    assert cache.token == ops.PlaneCache.token_of(w, 0)
    assert torch.equal(cache.planes, ref.planes)


@pytest.mark.parametrize("M", [4096 + 100, 131072])
def test_fused_forward_head_three_stage_ring_is_bit_identical(M):
    """The fused uint8 forward + head with a 3-stage LDS ring (knob U8_FH_STAGES=3: two K-steps of DMA in
    flight) runs the same MFMA / epilogue arithmetic as the 2-stage ring: bit-identical outputs."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    x8, w1, b1, w2, b2, tgt = _problem(M, 10, seed=7)
    outs = []
    try:
        for stages in (2, 3):
            K.set_knob("U8_FH_STAGES", stages)
            cache = ops.PlaneCache(w1)
            dl = torch.empty(M, 10, device=DEV)
            mask = torch.empty(M, N // 32, dtype=torch.int32, device=DEV)
            gw, gb = torch.zeros(10, N, device=DEV), torch.zeros(10, device=DEV)
            st = torch.empty(2, device=DEV)
            bound, pend = ops.linear_relu_head_u8(x8, w1, b1, cache, 0, w2, b2, tgt, gw, gb, 1.0 / M, st, True, dl,
                                                  mask, defer=False)
            torch.cuda.synchronize()
            outs.append((dl, mask, gw, gb, st, bound))
    finally:
        K.reset_knobs()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


def test_ds_read_tr8_lane_map():
    """ds_read_b64_tr_b8 (the ring weight gradient's pixel-fragment read, mlp_u8.hip frag_x8): per 16-lane group,
    lane 2q + p addresses row q, bytes 8p .. 8p + 7 of an 8-row x 16-byte block; lane i of the group receives byte
    column i of the 8 rows, row q in byte q. Checked on an 800-byte-pitch image as frag_x8 addresses it."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    g = torch.Generator(device="cpu").manual_seed(3)
    img = torch.randint(0, 256, (1024,), generator=g, dtype=torch.uint8)
    pitch = 64  # rows of the probe image (any multiple of 8 works for the map)
    lane = torch.arange(64)
    grp, i = lane // 16, lane % 16
    row0 = 8 * (grp // 2)  # groups 2, 3: the next 8 rows (frag_x8's lane half h)
    col0 = 16 * (grp % 2) + 32  # groups 1, 3: the next 16 columns
    addr = (row0 + i // 2) * pitch + col0 + 8 * (i % 2)
    out = K.u8_tr8_probe(img.to(DEV), addr.to(torch.int32).to(DEV)).cpu()
    got = out.contiguous().view(torch.uint8).view(64, 8)
    want = torch.empty(64, 8, dtype=torch.uint8)
    for l in range(64):
        for q in range(8):
            want[l, q] = img[(int(row0[l]) + q) * pitch + int(col0[l]) + int(i[l])]
    assert torch.equal(got, want), (got[:4], want[:4])


@pytest.mark.parametrize("M,C,Nh", [(4096, 10, 128), (4096 + 96, 10, 128), (131072, 10, 128), (8192, 2, 64),
                                    (8192, 16, 256)])
def test_wgrad_dma_ring_bit_identical_to_register_staged(M, C, Nh):
    """Knob U8_WGRAD_RING: the weight gradient from dl + ReLU bits with its operands on a 4-stage LDS-DMA ring
    (pixel fragments by transposed byte reads, widened in registers) against the register-staged kernel: the same
    dz planes, k order and MFMA sequence, so bit-identical gW / gb, with and without the head's bound."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    x8 = pixels(M, 51)
    h = rnd(M, Nh, seed=52).relu()
    dl = rnd(M, C, seed=53, scale=1e-3)
    w2 = rnd(C, Nh, seed=54, scale=0.1)
    g0 = rnd(Nh * KD + Nh, seed=55)
    bits = ops.relu_bits(h)
    try:
        for amax in (None, (dl.abs().sum(1).max() * w2.abs().max() * 2).reshape(1)):
            bufs = []
            for ring in (0, 1):
                K.set_knob("U8_WGRAD_RING", ring)
                b = g0.clone()
                ops.linear_wgrad_u8_dl(x8, dl, w2, bits, b[:Nh * KD].view(Nh, KD), b[Nh * KD:], amax=amax)
                torch.cuda.synchronize()
                bufs.append(b)
            assert torch.equal(bufs[0], bufs[1])
    finally:
        K.reset_knobs()
    # and against fp64
    dz = (dl.double() @ w2.double()) * (h > 0).double()
    want = dz.t() @ (x8.double() / 255.0)
    got = bufs[1][:Nh * KD].view(Nh, KD).double() - g0[:Nh * KD].view(Nh, KD).double()
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("M,C,Nh", [(4096 + 96, 10, 128), (131072, 10, 128), (8192, 16, 256)])
def test_wgrad_ring_balanced_tiles(M, C, Nh):
    """Knob U8_WGRAD_BAL: 3 full column tiles per wave and the last 16 columns on 16x16x32 MFMAs (waves 4..7). Columns
    0..767 and the bias keep the unbalanced ring kernel's MFMA sequence (bit-identical); columns 768..783 sum in a
    different MFMA order (fp32-equal)."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    x8 = pixels(M, 61)
    h = rnd(M, Nh, seed=62).relu()
    dl = rnd(M, C, seed=63, scale=1e-3)
    w2 = rnd(C, Nh, seed=64, scale=0.1)
    bits = ops.relu_bits(h)
    outs = []
    try:
        for bal in (0, 1):
            K.set_knob("U8_WGRAD_BAL", bal)
            b = torch.zeros(Nh * KD + Nh, device=DEV)
            ops.linear_wgrad_u8_dl(x8, dl, w2, bits, b[:Nh * KD].view(Nh, KD), b[Nh * KD:])
            torch.cuda.synchronize()
            outs.append(b)
    finally:
        K.reset_knobs()
    g0, g1 = (o[:Nh * KD].view(Nh, KD) for o in outs)
    assert torch.equal(g0[:, :768], g1[:, :768])
    assert torch.equal(outs[0][Nh * KD:], outs[1][Nh * KD:])
    # (a sum over M rows with cancellation: compare at the scale of the gradient's largest entries)
    torch.testing.assert_close(g1[:, 768:], g0[:, 768:], rtol=1e-4, atol=1e-6 * float(g0.abs().max()))
    dz = (dl.double() @ w2.double()) * (h > 0).double()
    want = dz.t() @ (x8.double() / 255.0)
    torch.testing.assert_close(g1.double(), want, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("M,C,Nh", [(131072, 10, 128), (65536, 10, 128), (131072 + 256, 10, 128), (8192, 16, 256)])
def test_wgrad_ring_pairwise_combine(M, C, Nh):
    """Knob U8_WGRAD_PAIR: splits s and s + S/2 of the ring weight gradient add their partials in-kernel (ticket, the
    first arriver publishes, the second adds and stores into row s) and the reduction reads S/2 rows. Equal to the
    unpaired gradient to fp32 summation order, repeatable bit for bit over launches (the pair sum is one commutative
    add, whoever arrives first; the ticket words reset themselves), and within the fp64 bound. Shapes whose split
    count is not a multiple of 16 run unpaired."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    x8 = pixels(M, 81)
    h = rnd(M, Nh, seed=82).relu()
    dl = rnd(M, C, seed=83, scale=1e-3)
    w2 = rnd(C, Nh, seed=84, scale=0.1)
    bits = ops.relu_bits(h)
    outs = []
    try:
        for pair in (0, 1, 1, 1):
            K.set_knob("U8_WGRAD_PAIR", pair)
            b = torch.zeros(Nh * KD + Nh, device=DEV)
            ops.linear_wgrad_u8_dl(x8, dl, w2, bits, b[:Nh * KD].view(Nh, KD), b[Nh * KD:])
            torch.cuda.synchronize()
            outs.append(b)
    finally:
        K.reset_knobs()
    assert torch.equal(outs[1], outs[2]) and torch.equal(outs[1], outs[3])
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=1e-6 * float(outs[0].abs().max()))
    dz = (dl.double() @ w2.double()) * (h > 0).double()
    want = dz.t() @ (x8.double() / 255.0)
    torch.testing.assert_close(outs[1][:Nh * KD].view(Nh, KD).double(), want, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("ring,cols", [(0, 64), (1, 64), (1, 32)])
def test_wgrad_hidden_group_ranges_match_the_whole_gradient(ring, cols):
    """linear_wgrad_u8_dl(groups=(g_first, g_count, blocks)) - the data-parallel step's two hidden-unit ranges
    (SDML_DP_SPLIT) - on both kernel forms: each range writes only its rows of gW / entries of gb, and the two ranges
    together equal the one-launch gradient to fp32 summation order (the row splits differ)."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    M, C, Nh = 16384, 10, 128
    x8 = pixels(M, 71)
    h = rnd(M, Nh, seed=72).relu()
    dl = rnd(M, C, seed=73, scale=1e-3)
    w2 = rnd(C, Nh, seed=74, scale=0.1)
    bits = ops.relu_bits(h)
    try:
        K.set_knob("U8_WGRAD_RING", ring)
        K.set_knob("U8_SLAB_COLS", cols)
        full = torch.zeros(Nh * KD + Nh, device=DEV)
        ops.linear_wgrad_u8_dl(x8, dl, w2, bits, full[:Nh * KD].view(Nh, KD), full[Nh * KD:])
        part = torch.zeros(Nh * KD + Nh, device=DEV)
        gw, gb = part[:Nh * KD].view(Nh, KD), part[Nh * KD:]
        ops.linear_wgrad_u8_dl(x8, dl, w2, bits, gw, gb, groups=(0, 1, 128))
        torch.cuda.synchronize()
        # (gW += ...: range 1's gradient is nonzero, so a touch would show)
        assert bool((gw[64:] == 0).all()) and bool((gb[64:] == 0).all()) and bool((gb[:64] != 0).all())
        ops.linear_wgrad_u8_dl(x8, dl, w2, bits, gw, gb, groups=(1, 1, 128))
        torch.cuda.synchronize()
    finally:
        K.reset_knobs()
    torch.testing.assert_close(part, full, rtol=1e-5, atol=1e-6 * float(full.abs().max()))


@pytest.mark.parametrize("M", [4096 + 100, 4096 + 300, 131072])
def test_fused_forward_head_512_row_blocks_are_bit_identical(M):
    """512-row blocks (knob U8_FH_ROWS512: every wave holds 4 row tiles, two per 256-row half, and the head runs once
    per half) against the 256-row blocks: the same K order per element and the same head per 256 rows, so every
    output is bit-identical; the ragged cases end in a block whose second half is partly empty (+300) or empty
    (+100, that pass is skipped)."""
    from simple_distributed_machine_learning_amd import _native

    K = _native.kernels()
    x8, w1, b1, w2, b2, tgt = _problem(M, 10, seed=11)
    outs = []
    try:
        for r512 in (0, 1):
            K.set_knob("U8_FH_ROWS512", r512)
            cache = ops.PlaneCache(w1)
            dl = torch.full((M, 10), float("nan"), device=DEV)
            mask = torch.zeros(M, N // 32, dtype=torch.int32, device=DEV)
            gw, gb = torch.zeros(10, N, device=DEV), torch.zeros(10, device=DEV)
            st = torch.empty(2, device=DEV)
            bound, pend = ops.linear_relu_head_u8(x8, w1, b1, cache, 0, w2, b2, tgt, gw, gb, 1.0 / M, st, True, dl,
                                                  mask, defer=False)
            torch.cuda.synchronize()
            outs.append((dl, mask, gw, gb, st, bound))
    finally:
        K.reset_knobs()
    assert not torch.isnan(outs[1][0]).any()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
