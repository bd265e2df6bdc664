// kge_rank_ref.h — reference-order scores for the ranking refinement.
//
// The fast ranking passes (MFMA tile, register tile, wave scan) sum a
// candidate's terms in their own order, so a candidate whose fp32 score lies
// within rounding distance of the true entity's can land on the other side of
// it than in the reference.  Those candidates (a per-query window δ_q, see
// k_rank_window) are re-scored here with the reference's own fp32 operation
// sequence, which this file restates:
//
//  * the per-element ops of model.py:166-249 as separate IEEE operations
//    (each ATen op rounds once; the build has -ffp-contract=off; RotatE's
//    stack(...).norm(dim=0) evaluates sqrt(fma(im, im, re*re)) — pinned on the
//    reference's output, tests/golden/make_golden.py `gen_rank_order`);
//  * ATen's CPU `sum(dim=2)` over the contiguous last dim (SumKernel's
//    vectorized_inner_sum / row_sum / multi_row_sum, 8-float vectors, 4
//    interleaved accumulators with the 4-level cascade) for DistMult, ComplEx,
//    RotatE and pRotatE;
//  * `torch.norm(p=1, dim=2)` as a sequential fp32 sum for TransE.
//
// Every fp32 operation matches the reference bit for bit.  The reference's
// vectorized CPU transcendentals cannot be reproduced on the device, so
// RotatE's cos / sin of the relation phases come from a table the caller
// evaluated with the reference's own ATen op (kge_model_desc.relation_trig);
// without one correctly rounded values are used (double evaluation rounded
// once), which differ from the reference's in the last bit on a few percent of
// arguments.  pRotatE's sin acts on per-candidate phase sums, so
// no table can carry it: the caller evaluates the sin of exactly the phase
// sums the refinement needs with the reference's own library call
// (kge_rank_sin_args → host → kge_rank_finish_sin), and the SIN form of
// ref_score_half sums those values; without them, correctly rounded sin.
#pragma once
#include "kge_device.h"

namespace kge {

// fp32 transcendentals from double: the double result (within an ulp of
// double) rounded to float — the correctly rounded float except when the
// exact value lies within that ulp of a float midpoint, so always within one
// float of it (abs_sin_bounds allows for that)
__device__ __forceinline__ float sin_rn(float x) { return (float)sin((double)x); }
// sin_rn and its possible alternative: the double sin y (within a few double
// ulps of sin x) rounds to r; when y lies within 2^-50·|y| of the midpoint
// between r and its neighbour on y's side, the correctly rounded float may be
// that neighbour — returned in *alt (else *alt = r).  The correctly rounded
// sin(x) is always r or *alt (sin_rn alone rounds twice).
__device__ __forceinline__ float sin_rn2(float x, float* alt) {
  const double y = sin((double)x);
  const float r = (float)y;
  const float nb = (y > (double)r) ? nextafterf(r, INFINITY) : nextafterf(r, -INFINITY);
  const double mid = 0.5 * ((double)r + (double)nb);
  *alt = (fabs(y - mid) <= ldexp(fabs(y), -50)) ? nb : r;
  return r;
}
__device__ __forceinline__ float cos_rn(float x) { return (float)cos((double)x); }
// correctly rounded sqrt, as ATen's: __builtin_sqrtf lowers to v_sqrt_f32 plus
// the fma residual correction (the build keeps HIP's default correctly rounded
// fp32 divide/sqrt).  NOT __fsqrt_rn: without OCML_BASIC_ROUNDED_OPERATIONS
// that is the native ~1-ulp v_sqrt_f32 — which made FB15k RotatE ranks tie
// (device) where the reference's differ by one ulp of the sum (2 / 256 queries).
__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_sqrtf(x); }

// reference q for one element (model.py association).  RotatE: the rotation
// (cos θ, sin θ) from the caller's table of the reference's own values when
// given (`trig` = this relation's [cos | sin] row, element k), else rounded
// once from double.
template <int M, int MODE>
__device__ __forceinline__ void ref_make_q(float xa, float xb, float ra, float rb, const Consts& c, float& qa,
                                           float& qb, const float* trig = nullptr, int k = 0, int K = 0) {
  if constexpr (M == ROTATE) {
    float cs, sn;
    if (trig) {
      cs = trig[k];
      sn = trig[K + k];
    } else {
      const float th = ra / c.kappa;  // model.py:209
      cs = cos_rn(th);
      sn = sin_rn(th);
    }
    Elem<M, MODE>::rotate(xa, xb, cs, sn, qa, qb);  // model.py:215-221
  } else {
    Elem<M, MODE>::make_q(xa, xb, ra, rb, c, qa, qb);  // exact already: no transcendentals
  }
}

// one element of the [B, E, K] tensor the reference reduces over dim 2
template <int M, int MODE>
__device__ __forceinline__ float ref_elem(float qa, float qb, float ea, float eb, const Consts& c) {
  constexpr bool HEAD = (MODE == HEAD_BATCH);
  if constexpr (M == TRANSE) {
    return fabsf(HEAD ? (ea + qa) : (qa - ea));
  } else if constexpr (M == DISTMULT) {
    return HEAD ? (ea * qa) : (qa * ea);
  } else if constexpr (M == COMPLEX) {
    return HEAD ? (ea * qa + eb * qb) : (qa * ea + qb * eb);
  } else if constexpr (M == ROTATE) {
    const float re = qa - ea, im = qb - eb;
    return sqrt_rn(__builtin_fmaf(im, im, re * re));
  } else {
    const float pe = ea / c.kappa_p;
    return fabsf(sin_rn(HEAD ? (pe + qa) : (qa - pe)));
  }
}

template <int M>
__device__ __forceinline__ float ref_finish(float total, const Consts& c) {
  if constexpr (M == TRANSE || M == ROTATE) return c.gamma - total;
  else if constexpr (M == PROTATE) return c.gamma - total * c.modulus;
  else return total;
}

__host__ __device__ inline int ceil_log2_i(int64_t x) {
  int r = 0;
  while (((int64_t)1 << r) < x) ++r;
  return r;
}

// Shuffle inside the caller's 32-lane half of the wave.
__device__ __forceinline__ float half_shfl(float v, int src_hl) {
  const int base = threadIdx.x & 32;
  return __int_as_float(__builtin_amdgcn_ds_bpermute((base + src_hl) << 2, __float_as_int(v)));
}

__device__ __forceinline__ tf2 half_shfl(tf2 v, int src_hl) { return tf2{half_shfl(v.x, src_hl), half_shfl(v.y, src_hl)}; }

// ATen's CPU sum(dim=2) over K elements, computed by one 32-lane half-wave
// (hl = lane within the half; every lane returns the total): 8-float
// vectors; vector v = 4·row + col over size_ilp = ⌊(K/8)/4⌋ rows
// (multi_row_sum, cascade levels of 2^lp rows), tail vectors into column 0,
// columns folded 0+1+2+3, then the scalar tail k ≥ 8·⌊K/8⌋ summed from 0 and
// the 8 vector lanes added in order.  Lane hl = 8·col + p owns elements
// 32·row + hl.  T = tf2 runs two sums through the same cascade side by side
// (the pRotatE screen's lower and upper bounds).
template <class T, class F>
__device__ T ref_cascade_half(F elem, int K, int hl) {
  const int nvec = K / 8;
  const int size = nvec / 4;
  const int lp0 = ceil_log2_i(size) / 4;
  const int lp = lp0 > 4 ? lp0 : 4;
  const int step = 1 << lp;
  const int64_t mask = step - 1;
  T acc[4] = {T{}, T{}, T{}, T{}};
  int i = 0;
  while (i + step <= size) {
    for (int j = 0; j < step; ++j, ++i) acc[0] += elem(32 * i + hl);
#pragma unroll
    for (int lv = 1; lv < 4; ++lv) {
      acc[lv] += acc[lv - 1];
      acc[lv - 1] = T{};
      if ((i & (mask << (lv * lp))) != 0) break;
    }
  }
  for (; i < size; ++i) acc[0] += elem(32 * i + hl);
  T col = acc[0];
#pragma unroll
  for (int lv = 1; lv < 4; ++lv) col += acc[lv];
  if (hl < 8)
    for (int v = 4 * size; v < nvec; ++v) col += elem(8 * v + hl);
  const T c1 = half_shfl(col, (hl + 8) & 31), c2 = half_shfl(col, (hl + 16) & 31), c3 = half_shfl(col, (hl + 24) & 31);
  const T vacc = ((col + c1) + c2) + c3;  // valid in lanes 0..7
  T fin = T{};
  for (int k = 8 * nvec; k < K; ++k) fin += elem(k);
#pragma unroll
  for (int p = 0; p < 8; ++p) fin += half_shfl(vacc, p);
  return fin;
}

// Reference-order score of the candidate row e against the query's reference
// q, computed by one 32-lane half-wave (hl = lane within the half); every
// lane of the half returns the score.  q / e: [K] real, or [re K | im K].
// SIN (pRotatE): e holds the K values sin(phase sum) as the caller's library
// evaluated them; the element is their abs (model.py:245-246), q is unused.
template <int M, int MODE, bool SIN = false>
__device__ float ref_score_half(const float* __restrict__ q, const float* __restrict__ e, int K, const Consts& c,
                                int hl) {
  constexpr bool CPLX = Traits<M>::cplx;
  auto elem = [&](int k) -> float {
    if constexpr (SIN) return fabsf(e[k]);
    const float qa = q[k], ea = e[k];
    const float qb = CPLX ? q[K + k] : 0.f, eb = CPLX ? e[K + k] : 0.f;
    return ref_elem<M, MODE>(qa, qb, ea, eb, c);
  };
  if constexpr (M == TRANSE) {
    // torch.norm(p=1): one fp32 accumulator, ascending k.  Lanes compute 32
    // elements at a time; lane 0 adds them in order.
    float acc = 0.f;
    for (int k0 = 0; k0 < K; k0 += 32) {
      const int k = k0 + hl;
      const float v = (k < K) ? elem(k) : 0.f;
      const int m = (K - k0 < 32) ? (K - k0) : 32;
      for (int j = 0; j < m; ++j) acc += half_shfl(v, j);
    }
    return ref_finish<M>(acc, c);
  } else {
    return ref_finish<M>(ref_cascade_half<float>(elem, K, hl), c);
  }
}

// pRotatE: the interval the reference's score must lie in when its sin is a
// library's whose result is within one ulp of the exact value — one of the
// two floats around sin(x), so within [prev(r), next(r)] of the correctly
// rounded r (x is the fp32 phase sum; sin(x) is never a float for x ≠ 0),
// bounded here around the device's sinf (see SIN_FAST_*).
// Every later operation is monotone in its operand — |·| on an interval that
// does not contain 0, each round-to-nearest add of the sum(dim=2) cascade,
// the product with the modulus, γ − ·  — so the reference's score lies in
// [γ − fl(S_hi·mod), γ − fl(S_lo·mod)] (mod ≥ 0; swapped otherwise), S_lo /
// S_hi the same cascade over the elements' lower / upper |sin| bounds.
// Returns (lo, hi); NaN in either when an argument is not finite.
// The device's own fp32 sinf, against the correctly rounded value, checked on
// every float of the range (kge_selftest_sin; tests/test_rank_parity_gpu.py
// runs it on each GPU box): at most SIN_FAST_D1 floats apart for |x| ≤
// SIN_FAST_R1 and SIN_FAST_D2 for |x| ≤ SIN_FAST_R2 (ROCm 7.2: 1 and 2) —
// measured against BOTH floats sin_rn2 cannot tell apart where the double sin
// lies next to a float midpoint, so against the correctly rounded r whichever
// it is (the double result rounded once more is not always r).  So
// r lies within that many floats of sinf(x), the library's value within one
// more, and the interval is taken around sinf(x) — no double-precision sin
// (the interval screen's cost) — except beyond SIN_FAST_R2, where it is taken
// around sin_rn2's one or two candidates, ±1 float.
constexpr float SIN_FAST_R1 = 16.f, SIN_FAST_R2 = 65536.f;
constexpr int SIN_FAST_D1 = 1, SIN_FAST_D2 = 2;
__device__ __forceinline__ int32_t float_ord(float f) {  // monotone in f (±0 → 0)
  const int32_t b = __float_as_int(f);
  return b >= 0 ? b : -(b & 0x7fffffff);
}
__device__ __forceinline__ float ord_float(int32_t o) { return __int_as_float(o >= 0 ? o : ((-o) | (int32_t)0x80000000)); }
__device__ __forceinline__ float sin_fast(float x) { return sinf(x); }
__device__ __forceinline__ tf2 abs_sin_bounds(float x) {
  float p, n;
  const float ax = fabsf(x);
  if (ax <= SIN_FAST_R2) {
    const float d = sin_fast(x);
    const int j = (ax <= SIN_FAST_R1 ? SIN_FAST_D1 : SIN_FAST_D2) + 1;
    const int32_t o = float_ord(d);
    p = ord_float(o - j);
    n = ord_float(o + j);
  } else {
    float alt;
    const float r = sin_rn2(x, &alt);
    if (r != r) return tf2{r, r};
    const int32_t o = float_ord(r), oa = float_ord(alt);
    p = ord_float((o < oa ? o : oa) - 1);
    n = ord_float((o > oa ? o : oa) + 1);
  }
  if (x != x) return tf2{x, x};
  if (p <= 0.f && n >= 0.f) return tf2{0.f, fmaxf(-p, n)};
  const float ap = fabsf(p), an = fabsf(n);
  return tf2{fminf(ap, an), fmaxf(ap, an)};
}
template <int MODE>
__device__ tf2 ref_score_half_prot_bounds(const float* __restrict__ q, const float* __restrict__ e, int K,
                                          const Consts& c, int hl) {
  auto elem = [&](int k) -> tf2 {
    const float pe = e[k] / c.kappa_p;  // model.py:236 / :238
    return abs_sin_bounds((MODE == HEAD_BATCH) ? (pe + q[k]) : (q[k] - pe));  // model.py:240-245
  };
  const tf2 S = ref_cascade_half<tf2>(elem, K, hl);
  const float a = S.x * c.modulus, b = S.y * c.modulus;
  if ((a != a) || (b != b)) return tf2{NAN, NAN};
  return tf2{c.gamma - fmaxf(a, b), c.gamma - fminf(a, b)};
}

}  // namespace kge
