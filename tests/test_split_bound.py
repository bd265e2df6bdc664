"""The split-bf16 ranking tile's error bound from its pieces' norms
(kge_rank_mfma.hip header, k_rank_window; round 6).

Each operand x is split as x = hi + lo + r with hi = bf16(x), lo = bf16(x - hi)
(round to nearest even) and r the exact remainder; the tile computes
Σ (q_hi e_hi + q_hi e_lo + q_lo e_hi).  Its distance from Σ q e is

    |Σ (q r_e + r_q e - r_q r_e + q_lo e_lo)|
        <= ‖q‖‖r_e‖ + ‖r_q‖‖e‖ + ‖r_q‖‖r_e‖ + ‖q_lo‖‖e_lo‖,

which the window evaluates with the table's maxima of ‖e‖, ‖r_e‖, ‖e_lo‖.
Checked here in float64 (products of fp32 values are exact there) on uniform,
sign-aligned and wide-range vectors, with the pieces computed exactly as the
kernels do (bf16_rne, bf16_split_scaled); and the bound's size on uniform rows
against the worst-case form of rounds 4-5 (770·u·‖q‖‖e‖).  Host arithmetic
only.
"""
import numpy as np

U = 2.0 ** -24


def bf16_rne(x):
    """kge_device.h bf16_rne, as the float value of the bf16 piece."""
    b = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) >> 16).astype(np.uint32) << np.uint32(16)
    return r.view(np.float32)


def split(x):
    x = np.asarray(x, np.float32)
    hi = bf16_rne(x)
    r1 = (x - hi).astype(np.float32)  # exact in fp32
    lo = bf16_rne(r1)
    r = (r1 - lo).astype(np.float32)  # exact in fp32
    assert np.array_equal(hi.astype(np.float64) + lo + r, x.astype(np.float64))
    return hi, lo, r


def bound_parts(q, e):
    qh, ql, rq = (p.astype(np.float64) for p in split(q))
    eh, el, re = (p.astype(np.float64) for p in split(e))
    q64, e64 = q.astype(np.float64), e.astype(np.float64)
    exact = (q64 * e64).sum(-1)
    tile = (qh * eh + qh * el + ql * eh).sum(-1)
    n = lambda v: np.sqrt((v * v).sum(-1))  # noqa: E731
    bound = n(q64) * n(re) + n(rq) * n(e64) + n(rq) * n(re) + n(ql) * n(el)
    return np.abs(exact - tile), bound, n(q64) * n(e64)


def test_bound_covers_uniform_aligned_and_wide_range():
    g = np.random.default_rng(3)
    for d in (16, 500, 1000):
        q = g.uniform(-1, 1, (400, d)).astype(np.float32)
        e = g.uniform(-1, 1, (400, d)).astype(np.float32)
        err, bound, _ = bound_parts(q, e)
        assert (err <= bound).all()
        # every error term of one sign: q along r_e, r_q along e (the Cauchy-Schwarz
        # equality direction), lo pieces of one sign
        _, _, re = split(e)
        qa = (np.abs(q) * np.where(re >= 0, 1, -1)).astype(np.float32)
        err, bound, _ = bound_parts(qa, e)
        assert (err <= bound).all() and (err > 0).any()
        # values over 30 orders of magnitude, exact zeros, equal vectors
        w = (g.uniform(-1, 1, (200, d)) * 10.0 ** g.uniform(-30, 3, (200, d))).astype(np.float32)
        w[g.random(w.shape) < 0.05] = 0
        err, bound, _ = bound_parts(w, w[::-1].copy())
        assert (err <= bound).all()
        err, bound, _ = bound_parts(w, w.copy())
        assert (err <= bound).all()


def test_bound_size_on_uniform_rows():
    """On uniform rows the pieces' norms give ≈126·u·‖q‖‖e‖ where the worst case
    gave 770·u·‖q‖‖e‖ — the window this narrows."""
    g = np.random.default_rng(4)
    q = g.uniform(-1, 1, (300, 500)).astype(np.float32)
    e = g.uniform(-1, 1, (300, 500)).astype(np.float32)
    _, bound, qe = bound_parts(q, e)
    ratio = bound / qe / U
    assert ratio.max() < 200 and ratio.min() > 60
