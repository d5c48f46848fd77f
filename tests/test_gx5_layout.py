"""Host-side check of cim_bwd_gx5_kernel's operand layout (csrc/cimq_gx5.hip, planned by x5_plan in
csrc/cimq_host.h): a numpy walk of the same index arithmetic -- the G patch of six output rows per
4-input-row m-tile ([row][col + 1][k*16 + o], zero padding columns), the wave / lane pixel mapping, the A
read at the (kh, kw)-shifted patch position with the padded second K-step, the weight operand wg5_item
([tile][half][position][K-step][channel block][lane]: channel 16 cb + (l & 15), kappa = 32 s + 8 (l >> 4) + e) and the lane order of
v_mfma_f32_16x16x32_bf16 -- must give the reference's folded grad_x contraction (lsq.py:336-386:
gx[c, ih, iw] = sum over (kh, kw) of gx_unf[(ih + 1 - kh, iw + 1 - kw), (c, kh, kw)], gx_unf[m, f] =
sum_{k,o} G_tile(f)[m, (k, o)] What_k[o, f]), exactly on integer inputs.  No GPU: this pins the index plan."""
import numpy as np
import pytest


@pytest.mark.parametrize("C,H", [(16, 32), (32, 16)])
def test_gx5_plan_folded_grad_x(C, H):
    rng = np.random.default_rng(5 + C)
    O, W = C, H
    K = 9 * C
    T = -(-K // 128)
    CBN, NPG = C // 16, W // 4
    G = rng.integers(-4, 5, (T, H, W, 3, O))  # G_i[out pixel, k, o] (integers: an exact check)
    Wt = rng.integers(-1, 2, (3, O, K))  # What_k[o, f]
    tile = np.arange(K) // 128
    # reference: unfolded product per tile of f, folded over (kh, kw)
    ref = np.zeros((C, H, W), np.int64)
    for f in range(K):
        c, p = divmod(f, 9)
        kh, kw = divmod(p, 3)
        unf = np.einsum("hwko,ko->hw", G[tile[f]], Wt[:, :, f])  # gx_unf[(oh, ow), f]
        for ih in range(H):
            oh = ih + 1 - kh
            if not 0 <= oh < H:
                continue
            for iw in range(W):
                ow = iw + 1 - kw
                if 0 <= ow < W:
                    ref[c, ih, iw] += unf[oh, ow]
    # wg5 fragments [i][h][p][s][cb][lane][8]
    wg5 = np.zeros((T, CBN, 9, 2, CBN, 64, 8), np.int64)
    for i in range(T):
        for h in range(CBN):
            for p in range(9):
                for s in range(2):
                    for cb in range(CBN):
                        for lane in range(64):
                            c = 16 * cb + (lane & 15)
                            f = 9 * c + p
                            if f // 128 != i:
                                continue
                            for e in range(8):
                                kap = 32 * s + 8 * (lane >> 4) + e
                                k, o = kap >> 4, 16 * h + (kap & 15)
                                if k < 3:
                                    wg5[i, h, p, s, cb, lane, e] = Wt[k, o, f]
    got = np.zeros_like(ref)
    WP = W + 2
    for r0 in range(0, H, 4):  # one m-tile per 4 input rows (one image)
        acc = np.zeros((8, 16, 16), np.int64)  # [wave][row = input pixel][col = channel]
        for i in range(T):
            for h in range(CBN):
                patch = np.zeros(6 * WP * 48 + 16, np.int64)  # one plane (hi / mid / lo alike)
                for row in range(6):
                    oh = r0 - 1 + row
                    if 0 <= oh < H:
                        for col in range(W):
                            patch[(row * WP + col + 1) * 48:(row * WP + col + 2) * 48] = \
                                G[i, oh, col, :, 16 * h:16 * h + 16].reshape(48)
                for wave in range(8):
                    cb, pg = divmod(wave, NPG)
                    rl, iw0 = divmod(pg, W // 16)
                    iw0 *= 16
                    c_lo, c_hi = 16 * cb, 16 * cb + 15
                    if 9 * c_hi + 8 < 128 * i or 9 * c_lo >= 128 * (i + 1):
                        continue
                    for p in range(9):
                        kh, kw = divmod(p, 3)
                        for s in range(2):
                            A = np.zeros((64, 8), np.int64)
                            for lane in range(64):
                                r16, g4 = lane & 15, lane >> 4
                                base = ((rl + 2 - kh) * WP + iw0 + r16 + 2 - kw) * 48 + 8 * g4 + 32 * s
                                A[lane] = patch[base:base + 8]
                            a = A.reshape(4, 16, 8)  # [g4][row][e]
                            b = wg5[i, h, p, s, cb].reshape(4, 16, 8)  # [g4][col][e]
                            acc[wave] += np.einsum("gre,gce->rc", a, b)
        for wave in range(8):
            cb, pg = divmod(wave, NPG)
            rl, iw0 = divmod(pg, W // 16)
            iw0 *= 16
            got[16 * cb:16 * cb + 16, r0 + rl, iw0:iw0 + 16] = acc[wave].T
    np.testing.assert_array_equal(got, ref)
