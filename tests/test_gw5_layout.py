"""Host-side check of cim_bwd_gw5_kernel's operand layout (csrc/cimq_gw5.hip, planned by g5_plan in
csrc/cimq_host.h): a numpy walk of the same index arithmetic -- the (input block, output block) pair
blocks, the A-ready patch of ctx slices, the per-lane row offsets (aoff), the pixel-pair offsets (poff),
the K order (pixel pair x slots j = 0, 1, 2, pad) of v_mfma_f32_16x16x32_bf16, the tile of each 16-row
block and the grad_alpha ownership -- must give the reference's grad_w contraction and grad_alpha sums
(lsq.py:321-356: gw[f, o] = sum_j sum_m xhat_j[m, f] g[m, o] D_j[m, o]; ga[i, kj, o] = sum_m code g), here
with integer-valued g so the check is exact.  No GPU: this pins the index plan; the GPU tests pin the kernel."""
import numpy as np
import pytest


def pass_mask_j(j):
    return sum(1 << (3 * (k * 3 + j)) for k in range(3))


@pytest.mark.parametrize("C,O,H,S", [(16, 16, 32, 1), (32, 32, 16, 1), (64, 64, 8, 1), (16, 32, 32, 2), (32, 64, 16, 2)])
def test_gw5_plan_grad_w_and_alpha(C, O, H, S):
    rng = np.random.default_rng(C + O + H + S)
    W = H
    Ho = Wo = H // S
    P = Ho * Wo
    PI = min(P, 128)
    IPM, R = 128 // PI, PI // Wo
    RH = (R - 1) * S + 3
    WP, CH = W + 2, IPM * RH
    K = 9 * C
    T = -(-K // 128)
    B = IPM * max(1, P // 128) if P < 128 else 1  # one m-tile's images
    nmt_img = max(1, P // 128)
    # inputs: ctx slices xhat[b, c, h, w, j] (small ints), grad_out g[b, o, p] (integers), state words
    xh = rng.integers(-1, 2, (B, C, H, W, 3))
    g = rng.integers(-3, 4, (B, O, P)).astype(np.int64)
    st = rng.integers(0, 1 << 27, (T, B * P, O), dtype=np.int64)
    # reference over the m-tile's pixels (the first 128 of image 0, or all IPM images)
    pix = [(b, p) for b in range(B) for p in (range(P) if P <= 128 else range(128))]
    ref_gw = np.zeros((K, O), np.int64)
    ref_ga = np.zeros((T, 9, O), np.int64)
    xp = np.pad(xh, ((0, 0), (0, 0), (1, 1), (1, 1), (0, 0)))
    for b, p in pix:
        oh, ow = divmod(p, Wo)
        m = b * P + p
        for f in range(K):
            c, q = divmod(f, 9)
            kh, kw = divmod(q, 3)
            i = f // 128
            s = st[i, m]
            for j in range(3):
                D = np.array([bin(int(v) & pass_mask_j(j)).count("1") << j for v in s])
                ref_gw[f] += xp[b, c, oh * S + kh, ow * S + kw, j] * g[b, :, p] * D
        for i in range(T):
            s = st[i, m]
            for kj in range(9):
                f2 = (s >> (3 * kj + 1)) & 3
                code = np.where(f2 == 1, 1, np.where(f2 == 3, -1, 0))
                ref_ga[i, kj] += code * g[b, :, p]
    got_gw = np.zeros((K, O), np.int64)
    got_ga = np.zeros((T, 9, O), np.int64)
    for cb in range(C // 16):
        i_lo, i_hi = (144 * cb) // 128, (144 * cb + 143) // 128
        own = [q <= i_hi - i_lo and ((i_lo + q) * 128) // 144 == cb for q in range(2)]
        # the A-ready patch of the block's 16 channels: [c][slot][row][col][slot j]
        pat = np.zeros((16 * CH * WP, 4), np.int64)
        for c in range(16):
            for sl in range(IPM):
                for row in range(RH):
                    ih = row - 1  # the m-tile's first output row is 0
                    if 0 <= ih < H:
                        cr = c * CH + sl * RH + row
                        pat[cr * WP + 1:cr * WP + 1 + W, :3] = xh[sl, 16 * cb + c, ih, :, :]
        for ob in range(O // 16):
            acc = np.zeros((9, 16, 16), np.int64)  # [fb][f row][o col]
            ga = np.zeros((2, 9, 16), np.int64)
            for wave in range(8):
                for s in range(2):
                    A = np.zeros((9, 64, 8), np.int64)
                    Bm = np.zeros((2, 64, 8), np.int64)
                    for lane in range(64):
                        r16, g4 = lane & 15, lane >> 4
                        pw = 16 * wave + 4 * g4
                        sl, pin0 = pw // PI, pw % PI
                        pin = pin0 + 2 * s
                        poff = (sl * RH + (pin // Wo) * S) * WP + (pin % Wo) * S
                        o = ob * 16 + r16
                        for e, pp in enumerate((pin, pin + 1)):
                            m = sl * P + pp
                            for q in range(i_hi - i_lo + 1):
                                sw = int(st[i_lo + q, m, o])
                                gv = g[sl, o, pp]
                                for j in range(3):
                                    Bm[q, lane, 4 * e + j] = gv * (bin(sw & pass_mask_j(j)).count("1") << j)
                                if own[q] and lane < 64:
                                    for kj in range(9):
                                        f2 = (sw >> (3 * kj + 1)) & 3
                                        ga[q, kj, r16] += (1 if f2 == 1 else -1 if f2 == 3 else 0) * gv
                        for fb in range(9):
                            f = 16 * fb + r16
                            c, q9 = divmod(f, 9)
                            kh, kw = divmod(q9, 3)
                            aoff = (c * CH + kh) * WP + kw
                            A[fb, lane, 0:4] = pat[aoff + poff]
                            A[fb, lane, 4:8] = pat[aoff + poff + S]
                    for fb in range(9):
                        q = (144 * cb + 16 * fb) // 128 - i_lo
                        a = A[fb].reshape(4, 16, 8)  # [g4][row][k]
                        bb = Bm[q].reshape(4, 16, 8)  # [g4][col][k]
                        acc[fb] += np.einsum("grk,gck->rc", a, bb)
            for fb in range(9):
                got_gw[144 * cb + 16 * fb:144 * cb + 16 * fb + 16, ob * 16:ob * 16 + 16] = acc[fb]
            for q in range(2):
                if own[q]:
                    got_ga[i_lo + q, :, ob * 16:ob * 16 + 16] = ga[q]
    np.testing.assert_array_equal(got_gw, ref_gw)
    np.testing.assert_array_equal(got_ga, ref_ga)
