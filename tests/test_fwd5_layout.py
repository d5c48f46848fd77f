"""Host-side check of cim_fwd5_kernel's operand layout (csrc/cimq_fwd5.hip, planned by f5_plan in
csrc/cimq_host.h): a numpy walk of the same index arithmetic -- the (tile, channel-block) pairs and tile
groups, the weight fragments of wf5_item, the slice-planar channel-innermost patch, the per-lane patch
offsets of the three K-steps and the lane order of v_mfma_i32_16x16x64_i8 -- must give every crossbar
tile's partial sums of the reference's contraction (lsq.py:166-185: ps[b, i, k, j, p, o] = sum over the
tile's rows f of x_j[b, p, f] * w_k[f, o]).  No GPU: this pins the index plan; the GPU tests pin the
kernel (test_gpu_fullsize.py, test_gpu_bench_composition.py)."""
import numpy as np
import pytest


def f5_plan(C, H, W, stride, xbar=128, budget=80 * 1024, qp=7):
    """Mirror of f5_plan (cimq_host.h): pairs, groups and the LDS need."""
    K = 9 * C
    T = -(-K // xbar)
    Ho = (H + 2 - 3) // stride + 1
    P = Ho * Ho
    PI = min(P, 128)
    IPM, R = 128 // PI, PI // Ho
    RH, WP = (R - 1) * stride + 3, W + 2
    tc0, tcb = [], []
    for i in range(T):
        tc0.append(len(tcb))
        flo, fhi = i * xbar, min((i + 1) * xbar, K)
        tcb += list(range((flo // 9) // 16, ((fhi - 1) // 9) // 16 + 1))
    tc0.append(len(tcb))
    fixed = T * 9 * 16 * 20 + ((2 * (qp + 2) * 4 + 15) // 16) * 16 + 16

    def need(tcm, ncb):
        return fixed + tcm * 9 * 1024 + IPM * RH * ncb * WP * 48

    groups, tcmax, ncbp, i = [], 0, 0, 0
    while i < T:
        span = lambda a, b: tcb[tc0[b] - 1] - tcb[tc0[a]] + 1  # noqa: E731
        pairs = lambda a, b: tc0[b] - tc0[a]  # noqa: E731
        e = i + 1
        assert need(max(tcmax, pairs(i, e)), max(ncbp, span(i, e))) <= budget
        while e < T and need(max(tcmax, pairs(i, e + 1)), max(ncbp, span(i, e + 1))) <= budget:
            e += 1
        groups.append((i, e, tcb[tc0[i]], tcb[tc0[e] - 1]))
        tcmax, ncbp = max(tcmax, pairs(i, e)), max(ncbp, span(i, e))
        i = e
    return dict(K=K, T=T, Ho=Ho, P=P, IPM=IPM, R=R, RH=RH, WP=WP, tc0=tc0, tcb=tcb, groups=groups, NCBP=ncbp,
                lds=need(tcmax, ncbp))


def wf5(plan, ws, O):
    """wf5_item: [ob][pair][s][k][lane][16] int8 from the weight slices ws[k, f, o]."""
    K, tc0, tcb = plan["K"], plan["tc0"], plan["tcb"]
    ntc = len(tcb)
    out = np.zeros((O // 16, ntc, 3, 3, 64, 16), np.int64)
    for tc in range(ntc):
        i = max(t for t in range(plan["T"]) if tc0[t] <= tc)
        flo, fhi = i * 128, min((i + 1) * 128, K)
        for s in range(3):
            for lane in range(64):
                p = 4 * s + (lane >> 4)
                if p >= 9:
                    continue
                for e in range(16):
                    c = tcb[tc] * 16 + e
                    f = c * 9 + p
                    if c * 9 < K and flo <= f < fhi:
                        for ob in range(O // 16):
                            out[ob, tc, s, :, lane, e] = ws[:, f, ob * 16 + (lane & 15)]
    return out


@pytest.mark.parametrize("C,O,H,stride", [(16, 16, 32, 1), (16, 32, 32, 2), (32, 32, 16, 1), (64, 64, 8, 1)])
def test_fwd5_plan_partial_sums(C, O, H, stride):
    rng = np.random.default_rng(C + O + H + stride)
    plan = f5_plan(C, H, H, stride)
    assert plan["lds"] <= 80 * 1024
    if C == 64:
        assert len(plan["groups"]) > 1  # the weight side does not fit at once: staged per group
    B = plan["IPM"]  # one m-tile of 128 pixels
    K, T, Ho, P, RH, WP, NCBP = (plan[k] for k in ("K", "T", "Ho", "P", "RH", "WP", "NCBP"))
    W = H
    xs = rng.integers(0, 2, (3, B, C, H, H))  # activation slices (slice 0 up to 2 with the artifacts)
    xs[0] += rng.integers(0, 2, xs[0].shape) * (rng.random(xs[0].shape) < 0.05)
    ws = rng.integers(-1, 2, (3, K, O))  # weight slices
    # reference: unfold (c, kh, kw) order, per tile
    xp = np.pad(xs, ((0, 0), (0, 0), (0, 0), (1, 1), (1, 1)))
    unf = np.zeros((3, B, P, K), np.int64)
    for c in range(C):
        for kh in range(3):
            for kw in range(3):
                f = c * 9 + kh * 3 + kw
                unf[:, :, :, f] = xp[:, :, c, kh:kh + stride * Ho:stride, kw:kw + stride * Ho:stride].reshape(3, B, P)
    ref = np.zeros((T, 3, 3, B, P, O), np.int64)  # [i, k, j, b, p, o]
    for i in range(T):
        sl = slice(i * 128, min((i + 1) * 128, K))
        ref[i] = np.einsum("jbpf,kfo->kjbpo", unf[:, :, :, sl], ws[:, sl, :])
    frag = wf5(plan, ws, O)
    got = np.zeros_like(ref)
    PI = min(P, 128)
    for (t0, t1, cb0, cb1) in plan["groups"]:
        # the group's patch: [img][row][cb slot][col][slice][16 channels] (as bytes)
        patch = np.zeros((B, RH, NCBP, WP, 3, 16), np.int64)
        for sl in range(B):
            for row in range(RH):
                ih = row - 1  # one m-tile: its first output row is 0
                if not 0 <= ih < H:
                    continue
                for cb in range(cb0, cb1 + 1):
                    for e in range(16):
                        if cb * 16 + e < C:
                            patch[sl, row, cb - cb0, 1:W + 1, :, e] = xs[:, sl, cb * 16 + e, ih, :].T
        flat = patch.reshape(-1)  # byte offsets f5_off * 1 + 16 j + e, in 16-B units below
        IMGB = RH * NCBP * WP * 48
        for wave in range(8):
            pl = wave * 16 + np.arange(16)
            slot, pin = pl // PI, pl % PI
            pix = slot * IMGB + ((pin // Ho) * stride * NCBP * WP + (pin % Ho) * stride) * 48
            for i in range(t0, t1):
                ps = np.zeros((O // 16, 3, 3, 16, 16), np.int64)  # [ob, k, j, row, col]
                for tc in range(plan["tc0"][i], plan["tc0"][i + 1]):
                    cbo = (plan["tcb"][tc] - cb0) * WP * 48
                    for s in range(3):
                        A = np.zeros((3, 64, 16), np.int64)  # [j][lane][byte]
                        for lane in range(64):
                            p = min(4 * s + (lane >> 4), 8)
                            off = pix[lane & 15] + ((p // 3) * NCBP * WP + p % 3) * 48 + cbo
                            for j in range(3):
                                A[j, lane] = flat[off + 16 * j:off + 16 * j + 16]
                        # D[row, col] = sum over lane groups g4 and bytes e of A[row + 16 g4][e] B[col + 16 g4][e]
                        a = A.reshape(3, 4, 16, 16)  # [j][g4][row][e]
                        bb = frag[:, tc, s].reshape(O // 16, 3, 4, 16, 16)  # [ob][k][g4][col][e]
                        ps += np.einsum("jgrE,bkgcE->bkjrc", a, bb)
                got[i, :, :, slot, pin, :] = ps.transpose(3, 1, 2, 0, 4).reshape(16, 3, 3, O)
    m = slice(None) if P <= 128 else slice(0, 128)  # the m-tile's pixels
    np.testing.assert_array_equal(got[:, :, :, :, m], ref[:, :, :, :, m])
