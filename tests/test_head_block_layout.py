"""Bank-conflict freedom of head_block.h's LDS images, by enumeration of every lane's address (no GPU).

The fused uint8 forward + head (mlp_u8.hip) and the standalone block head (head_xent.hip) stage h as fp16 planes
in an image of 8-byte granules (4 rows of one hidden unit), granule q of hidden unit h at q ^ gswz(h); the dl^T
image uses the same swizzle per class. This replays the kernel's address arithmetic for each access and checks,
per LDS lane group, that no bank is hit by two different addresses (MI355X_MICROARCH.md, LDS table):
ds_write_b64 in 4 groups of 16 lanes (bank = dword mod 32), ds_read_b64 / ds_read_b64_tr_b16 in 2 groups of 32
lanes (bank = dword mod 64).
"""
ROWS = 256
PLANE_B = 128 * ROWS * 2


def gswz(h):
    return ((h >> 2) & 1) | (((h >> 3) & 1) << 1) | ((h & 1) << 2) | (((h >> 1) & 1) << 3) | (((h >> 3) & 1) << 4)


def hoff(p, h, q):  # the two planes of a hidden unit are adjacent 512-B rows
    return h * (4 * ROWS) + p * (2 * ROWS) + 8 * (q ^ gswz(h))


def _conflicts(addrs, groups, banks):
    """max over groups and banks of the number of DISTINCT dwords hitting one bank (1 = conflict-free);
    addrs: lane -> byte address of its 8-byte access"""
    worst = 1
    for grp in groups:
        per_bank = {}
        for lane in grp:
            for d in (addrs[lane] // 4, addrs[lane] // 4 + 1):
                per_bank.setdefault(d % banks, set()).add(d)
        worst = max(worst, max(len(v) for v in per_bank.values()))
    return worst


W16 = [list(range(16 * k, 16 * k + 16)) for k in range(4)]   # ds_write_b64
R32 = [list(range(32)), list(range(32, 64))]                  # ds_read_b64, ds_read_b64_tr_b16


def test_h_image_writes_conflict_free():
    # wave (wm, wn), tile (i, j), register quad rq: lane -> hidden 64 wn + 32 j + (lane & 31),
    # granule 16 wm + 8 i + 2 rq + (lane >> 5)
    for wm in range(4):
        for wn in range(2):
            for i in range(2):
                for j in range(2):
                    for rq in range(4):
                        for p in range(2):
                            addrs = [hoff(p, 64 * wn + 32 * j + (l & 31), 16 * wm + 8 * i + 2 * rq + (l >> 5))
                                     for l in range(64)]
                            assert _conflicts(addrs, W16, 32) == 1


def test_logits_transposed_reads_conflict_free():
    # B operand of the 16x16x32 logits MFMA: lane (r = l & 15, g = l >> 4) reads image row (hidden)
    # 32 kk + 8 g + (r >> 2) (+ 4), granule 4 T + (r & 3)
    for T in range(16):
        for kk in range(4):
            for plus in (0, 4):
                addrs = [hoff(0, 32 * kk + 8 * (l >> 4) + ((l & 15) >> 2) + plus, 4 * T + (l & 3)) for l in range(64)]
                assert _conflicts(addrs, R32, 64) == 1


def test_dw2_reads_conflict_free():
    # B operand of the dW2 MFMA: lane (r, g) reads hidden 16 w + r, granules 8 ks + 2 g (+ 1); the dl^T image the
    # same with the class r
    for w in range(8):
        for ks in range(8):
            for e in (0, 1):
                addrs = [hoff(1, 16 * w + (l & 15), 8 * ks + 2 * (l >> 4) + e) for l in range(64)]
                assert _conflicts(addrs, R32, 64) == 1
    for ks in range(8):
        for e in (0, 1):
            addrs = [(l & 15) * (ROWS * 2) + 8 * ((8 * ks + 2 * (l >> 4) + e) ^ gswz(l & 15)) for l in range(64)]
            assert _conflicts(addrs, R32, 64) == 1


def test_swizzle_is_a_bijection_per_row():
    for h in range(128):
        assert sorted(q ^ gswz(h) for q in range(64)) == list(range(64))


# ds_read_b128 is serviced in 4 lane groups of 16 that are not contiguous (MI355X_MICROARCH.md, LDS table)
G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[l + 32 for l in grp] for grp in G128]


def _conflicts16(addrs, groups):
    worst = 1
    for grp in groups:
        per_bank = {}
        for lane in grp:
            for d in range(addrs[lane] // 4, addrs[lane] // 4 + 4):
                per_bank.setdefault(d % 64, set()).add(d)
        worst = max(worst, max(len(v) for v in per_bank.values()))
    return worst


def test_w2_plane_reads_conflict_free():
    # W2 planes [16 classes][W2PP = 288 B]: lane (r = l & 15, g = l >> 4) reads class r, halves 32 kk + 8 g .. +7
    W2PP = 128 * 2 + 32
    for kk in range(4):
        addrs = [(l & 15) * W2PP + 2 * (32 * kk + 8 * (l >> 4)) for l in range(64)]
        assert _conflicts16(addrs, G128) == 1
    # (an unpadded 256-B pitch would be 8-way)
    assert _conflicts16([(l & 15) * 256 + 16 * (l >> 4) for l in range(64)], G128) == 8


# dl image [plane][row][16 classes] fp16: row R stored at physical row P(R) = R ^ (bit 3 of R) << 2, its four 8-byte
# class-group slots at s ^ ((P >> 2) & 3)
def dl_off(R, s):
    P = R ^ (((R >> 3) & 1) << 2)
    return P * 32 + 8 * (s ^ ((P >> 2) & 3))


def test_dl_image_writes_and_dw2_reads_conflict_free():
    # writes: lane (r, g) of row tile T stores classes 4g..4g+3 of row 16 T + r (ds_write_b64, 4 groups of 16)
    for T in range(16):
        addrs = [dl_off(16 * T + (l & 15), l >> 4) for l in range(64)]
        assert _conflicts(addrs, W16, 32) == 1
    # dW2 A operand: lane (r, g) supplies row 32 ks + 8 g + (r >> 2) (+ 4), slot r & 3 (ds_read_b64_tr_b16)
    for ks in range(8):
        for plus in (0, 4):
            addrs = [dl_off(32 * ks + 8 * (l >> 4) + ((l & 15) >> 2) + plus, l & 3) for l in range(64)]
            assert _conflicts(addrs, R32, 64) == 1


def test_dl_image_is_a_bijection():
    offs = sorted(dl_off(R, s) for R in range(256) for s in range(4))
    assert offs == list(range(0, 256 * 32, 8))


def test_h_image_write_addresses_as_base_xor():
    # head_block.h hid_base: hoff(0, h, qb | c) == hid_base(h, qb) ^ 8 c (qb with bits 1..3 clear, c = 8 i + 2 rq)
    for h in range(128):
        for wm in range(4):
            for h2 in range(2):
                qb = 16 * wm + h2
                base = h * (4 * ROWS) + 8 * (qb ^ gswz(h))
                for i in range(2):
                    for rq in range(4):
                        c = 8 * i + 2 * rq
                        assert hoff(0, h, qb | c) == base ^ (8 * c)
