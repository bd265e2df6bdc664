// kge_device.h — device-side model math for the MI355X KGE hot path.
//
// Row layout in HBM (the reference's nn.Parameter layout, model.py:42-57):
//   entity   [E, Le] fp32 row-major; complex models (ComplEx, RotatE) keep
//            re = [0, K), im = [K, 2K) with K = Le/2 (torch.chunk(., 2, dim=2),
//            model.py:185-187, 204-205).
//   relation [R, Lr] fp32; RotatE rows are K phases, ComplEx rows re/im halves,
//            TransE/DistMult/pRotatE rows are plain Le-vectors.
//
// A wave (64 lanes) owns a whole row.  The row is cut into SLOTS of VEC
// consecutive floats (VEC = 4 → one 16-byte load per slot and per half);
// lane l holds slots l, l+64, l+128, ... (NS slots per lane).  Complex models
// cut the K complex dims the same way and each slot carries the matching
// re/im float groups.  Every per-row sum is: lane-local over its slots in
// ascending order, then a 64-lane xor-butterfly — a fixed order, so a score is
// bit-identical wherever it is computed (training, forward, ranking).
//
// Every score plug-in of model.py:166-249 is written here in the factored form
//     score(i, j) = finish( Σ_k phi(q_i[k], e_j[k]) )
// with q_i a per-positive-row vector (the part of the triple the negatives
// share) and e_j the gathered candidate row:
//     tail-batch / single: q = f(h, r), e = t       (model.py:126-146, 83-102)
//     head-batch:          q = f(r, t), e = h       (model.py:104-124)
// The association of each reference expression is kept (e.g. TransE head-batch
// is h + (r - t), model.py:168), and the build uses -ffp-contract=off, so the
// per-element arithmetic rounds like the reference's elementwise ATen ops.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kge {

enum Model : int { TRANSE = 0, DISTMULT = 1, COMPLEX = 2, ROTATE = 3, PROTATE = 4 };
enum Mode : int { SINGLE = 0, HEAD_BATCH = 1, TAIL_BATCH = 2 };
// (ranking refinement launches only: both directions' queries in one grid)
constexpr int BOTH_DIRS = 3;

template <int M>
struct Traits {
  static constexpr bool cplx = (M == COMPLEX || M == ROTATE);
  // RotatE relation rows carry K phases (one float per complex dim).
  static constexpr bool rel_phase = (M == ROTATE);
};

struct Consts {
  float gamma;
  float kappa;    // embedding_range / pi     (model.py:209)
  float kappa_p;  // embedding_range / pi'    (model.py:236-238, pi typo)
  float modulus;  // pRotatE modulus value, read from the device parameter
};

// ---------------------------------------------------------------- loads
typedef float tf2 __attribute__((ext_vector_type(2)));  // a register pair (v_pk_*_f32 operand)
typedef float tf4 __attribute__((ext_vector_type(4)));

template <int VEC>
__device__ __forceinline__ void ldv(const float* __restrict__ p, float (&x)[VEC]) {
  if constexpr (VEC == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else {
#pragma unroll
    for (int k = 0; k < VEC; ++k) x[k] = p[k];
  }
}
template <int VEC>
__device__ __forceinline__ void stv(float* __restrict__ p, const float (&x)[VEC]) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  } else {
#pragma unroll
    for (int k = 0; k < VEC; ++k) p[k] = x[k];
  }
}
template <int VEC>
__device__ __forceinline__ void zv(float (&x)[VEC]) {
#pragma unroll
  for (int k = 0; k < VEC; ++k) x[k] = 0.f;
}

// A row as one lane holds it: NS slots, each VEC floats of the real part (a)
// and, for complex models, VEC floats of the imaginary part (b).
template <int NS, int VEC, bool CPLX>
struct Row {
  float a[NS][VEC];
  float b[CPLX ? NS : 1][VEC];
};

struct RowGeom {
  int S;     // slots per half-row (complex) or per row (real)
  int half;  // float offset of the imaginary half (complex), 0 otherwise
};

// Branch-free: every lane loads (a lane past the row end re-reads slot 0, a
// line the wave fetches anyway) and lanes past the end are zeroed by a select.
// Only slots s >= NS/2 can be partial (NS is the smallest power of two with
// 64*NS >= S), so the selects are confined to those.
template <int NS, int VEC, bool CPLX>
__device__ __forceinline__ void load_row(const float* __restrict__ base, RowGeom g, int lane,
                                         Row<NS, VEC, CPLX>& r) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int slot = lane + 64 * s;
    constexpr bool maybe_partial = true;
    const bool ok = (s < NS / 2) ? true : (slot < g.S);
    const int sl = ok ? slot : 0;
    ldv<VEC>(base + sl * VEC, r.a[s]);
    if constexpr (CPLX) ldv<VEC>(base + g.half + sl * VEC, r.b[s]);
    if (maybe_partial && s >= NS / 2) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        r.a[s][v] = ok ? r.a[s][v] : 0.f;
        if constexpr (CPLX) r.b[s][v] = ok ? r.b[s][v] : 0.f;
      }
    }
  }
}
template <int NS, int VEC, bool CPLX>
__device__ __forceinline__ void store_row(float* __restrict__ base, RowGeom g, int lane,
                                          const Row<NS, VEC, CPLX>& r) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int slot = lane + 64 * s;
    if (slot < g.S) {
      stv<VEC>(base + slot * VEC, r.a[s]);
      if constexpr (CPLX) stv<VEC>(base + g.half + slot * VEC, r.b[s]);
    }
  }
}
// RotatE relation rows: K phases, same slot cut as the complex half.
template <int NS, int VEC>
__device__ __forceinline__ void load_phase(const float* __restrict__ base, int S, int lane,
                                           float (&p)[NS][VEC]) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int slot = lane + 64 * s;
    if (slot < S) ldv<VEC>(base + slot * VEC, p[s]);
    else zv<VEC>(p[s]);
  }
}

template <int NS, int VEC, bool CPLX>
__device__ __forceinline__ void zero_row(Row<NS, VEC, CPLX>& r) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    zv<VEC>(r.a[s]);
    if constexpr (CPLX) zv<VEC>(r.b[s]);
  }
}

// Wave index inside the workgroup as a scalar: threadIdx.x >> 6 is
// wave-uniform, but only readfirstlane tells the compiler so — and with it
// every row id and row base address derived from it stays in SGPRs, so the
// row loads use the scalar-base + 32-bit-lane-offset form.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Buffer descriptors (wave-uniform base and size): lanes with nothing to do
// pass an out-of-range offset, so loads return 0 and stores are dropped by
// the hardware range check — no exec branches around memory operations,
// which keeps the vmcnt bookkeeping static across the software pipeline.
constexpr uint32_t BUF_OOB = 0x7FFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint64_t bytes) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)n, 0x00020000);
}
// (the b32 builtins move raw 32-bit words: reinterpret, never convert)
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ int32_t buf_ldi(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}

__device__ __forceinline__ void buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t off, float (&x)[4]) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  x[0] = __uint_as_float(v.x); x[1] = __uint_as_float(v.y); x[2] = __uint_as_float(v.z); x[3] = __uint_as_float(v.w);
}

// Σ subsampling_weight (model.py:285-286) by one 256-thread block in a fixed
// order (strided partial sums, then a tree in `red`); every caller gets the
// same bits.  Returns the sum in every thread.
__device__ __forceinline__ float block_weight_sum(const float* __restrict__ w, int64_t B, float* red) {
  float s = 0.f;
  for (int64_t k = threadIdx.x; k < B; k += 256) s += w[k];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float tot = red[0];
  __syncthreads();
  return tot;
}

// ------------------------------------------------------------ reductions
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float readlanef(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// Full-wave sum, identical bits in every lane, fixed order.  Four DPP steps
// (lane^1, lane^2, half-row mirror, row mirror) leave each 16-lane row holding
// its row sum in every lane — each step pairs the same two partial sums on
// both sides, so the bits agree — then the four row sums are combined as
// (r0 + r1) + (r2 + r3) from scalar reads.  No LDS traffic.  Must be called
// with all 64 lanes active.
__device__ __forceinline__ float wave_sum(float x) {
  x = x + dppf<0xB1>(x);   // quad_perm [1,0,3,2]
  x = x + dppf<0x4E>(x);   // quad_perm [2,3,0,1]
  x = x + dppf<0x141>(x);  // row_half_mirror
  x = x + dppf<0x140>(x);  // row_mirror
  return (readlanef(x, 0) + readlanef(x, 16)) + (readlanef(x, 32) + readlanef(x, 48));
}

// bf16 bits of x, round-to-nearest-even (NaN → quiet NaN): the split-bf16
// ranking tile's operand pieces (kge_rank_mfma.hip)
__device__ __forceinline__ uint32_t bf16_rne(float x) {
  const uint32_t b = __float_as_uint(x);
  if (x != x) return 0x7FC0u;
  return (b + 0x7FFFu + ((b >> 16) & 1u)) >> 16;
}
// x = hi + lo + r exactly, hi = bf16(x), lo = bf16(x − hi) (both differences
// are exact in fp32): the lo piece and the residual r, scaled by 2^8 and 2^16
// (exact) so their squares stay normal wherever x's do — the split tile's
// data-dependent error bound sums them (k_split_stats, k_rank_window)
__device__ __forceinline__ void bf16_split_scaled(float x, float& lo8, float& r16) {
  const float r1 = x - __uint_as_float(bf16_rne(x) << 16);
  const float lo = __uint_as_float(bf16_rne(r1) << 16);
  lo8 = lo * 256.f;
  r16 = (r1 - lo) * 65536.f;
}

// Hardware square root / reciprocal (v_sqrt_f32 / v_rcp_f32, ~1 ulp) for the
// per-element modulus of RotatE; the reference's scalar division (the phase,
// model.py:209) stays an IEEE division.
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }

// F.logsigmoid (ATen CPU: min(x,0) - log1p(exp(-|x|))) and sigmoid.
__device__ __forceinline__ float log_sigmoid(float x) {
  return fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

// torch.optim.Adam single-tensor update of one element (torch/optim/adam.py,
// non-capturable branch; run.py:266-269 builds it with the defaults):
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//   denom = v.sqrt() / bias_correction2_sqrt + eps; p.addcdiv_(m, denom, -step_size)
struct AdamT {
  float* p;
  float* m;
  float* v;
  float step_size, bc2s;
};
struct AdamK {
  float b1, b2, eps;
};
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamK& k, float step_size,
                                          float bc2s) {
  const float w = 1.f - k.b1;  // lerp weight < 0.5 → self + w * (end - self)
  m = m + w * (g - m);
  v = v * k.b2 + (1.f - k.b2) * (g * g);
  const float denom = sqrtf(v) / bc2s + k.eps;
  p = p + (-step_size) * (m / denom);
}

// ------------------------------------------------------------ model math
// q construction for the element (a, b) of one slot.
//   TAIL/SINGLE: inputs (x = head, r); HEAD: inputs (r, x = tail)
// For RotatE `ra` is the relation phase-angle element; `rb` is unused.
template <int M, int MODE>
struct Elem {
  static constexpr bool HEAD = (MODE == HEAD_BATCH);

  // RotatE's rotation of x by (cos θ, sin θ) — the complex product of
  // model.py:215-221, one IEEE op per ATen op.  Shared by the fast q and the
  // reference-order q, so given the same cos / sin both have the same bits.
  __device__ static __forceinline__ void rotate(float xa, float xb, float cs, float sn, float& qa, float& qb) {
    if constexpr (HEAD) {                 // model.py:215-216
      qa = cs * xa + sn * xb;
      qb = cs * xb - sn * xa;
    } else {                              // model.py:220-221
      qa = xa * cs - xb * sn;
      qb = xa * sn + xb * cs;
    }
  }

  __device__ static __forceinline__ void make_q(float xa, float xb, float ra, float rb, const Consts& c,
                                                float& qa, float& qb) {
    if constexpr (M == TRANSE) {
      if constexpr (HEAD) qa = ra - xa;   // (relation - tail), model.py:168
      else qa = xa + ra;                  // (head + relation), model.py:170
      qb = 0.f;
    } else if constexpr (M == DISTMULT) {
      qa = HEAD ? (ra * xa) : (xa * ra);  // model.py:177 / :179
      qb = 0.f;
    } else if constexpr (M == COMPLEX) {
      if constexpr (HEAD) {               // model.py:190-191
        qa = ra * xa + rb * xb;
        qb = ra * xb - rb * xa;
      } else {                            // model.py:194-195
        qa = xa * ra - xb * rb;
        qb = xa * rb + xb * ra;
      }
    } else if constexpr (M == ROTATE) {
      const float th = ra / c.kappa;      // true fp32 division, model.py:209
      float sn, cs;
      sincosf(th, &sn, &cs);              // model.py:211-212
      rotate(xa, xb, cs, sn, qa, qb);
    } else {                            // PROTATE, model.py:236-243
      const float pr = ra / c.kappa_p;
      const float px = xa / c.kappa_p;
      qa = HEAD ? (pr - px) : (px + pr);
      qb = 0.f;
    }
  }

  // per-element term of the reduction over dim 2
  __device__ static __forceinline__ float phi(float qa, float qb, float ea, float eb, const Consts& c) {
    if constexpr (M == TRANSE) {
      return fabsf(HEAD ? (ea + qa) : (qa - ea));           // torch.norm(p=1), model.py:172
    } else if constexpr (M == DISTMULT) {
      return HEAD ? (ea * qa) : (qa * ea);                  // model.py:181
    } else if constexpr (M == COMPLEX) {
      return HEAD ? (ea * qa + eb * qb) : (qa * ea + qb * eb);  // model.py:192,196
    } else if constexpr (M == ROTATE) {
      const float dr = qa - ea, di = qb - eb;               // model.py:217-223
      return fsqrt(dr * dr + di * di);                      // stack+norm(dim=0), model.py:225-226
    } else {
      const float pe = ea / c.kappa_p;
      const float x = HEAD ? (pe + qa) : (qa - pe);
      return fabsf(sinf(x));                                // model.py:245-246
    }
  }

  // score from the summed terms
  __device__ static __forceinline__ float finish(float total, const Consts& c) {
    if constexpr (M == TRANSE || M == ROTATE) return c.gamma - total;       // model.py:172,228
    else if constexpr (M == PROTATE) return c.gamma - total * c.modulus;    // model.py:248
    else return total;                                                       // model.py:181,198
  }

  // d score / d q and d score / d e for one element
  __device__ static __forceinline__ void grads(float qa, float qb, float ea, float eb, const Consts& c,
                                               float& gqa, float& gqb, float& gea, float& geb) {
    if constexpr (M == TRANSE) {
      const float v = HEAD ? (ea + qa) : (qa - ea);
      const float sg = sgnf(v);
      gqa = -sg;
      gea = HEAD ? -sg : sg;
      gqb = geb = 0.f;
    } else if constexpr (M == DISTMULT) {
      gqa = ea; gea = qa; gqb = geb = 0.f;
    } else if constexpr (M == COMPLEX) {
      gqa = ea; gqb = eb; gea = qa; geb = qb;
    } else if constexpr (M == ROTATE) {
      const float dr = qa - ea, di = qb - eb;
      const float s2 = dr * dr + di * di;
      const float inv = (s2 > 0.f) ? frsq(s2) : 0.f;  // 1/|.|; norm backward is masked at 0
      const float ur = dr * inv, ui = di * inv;
      gqa = -ur; gqb = -ui; gea = ur; geb = ui;
    } else {
      const float pe = ea / c.kappa_p;
      const float x = HEAD ? (pe + qa) : (qa - pe);
      float sn, cs;
      sincosf(x, &sn, &cs);
      const float dx = -c.modulus * sgnf(sn) * cs;
      gqa = dx;
      gea = (HEAD ? dx : -dx) / c.kappa_p;
      gqb = geb = 0.f;
    }
  }

  // phi for one element, and (ea, eb) overwritten in place with what the
  // q-gradient needs, so the training row pass evaluates each element once:
  //   d score / d q = dq_of(ea', eb')  (see dq_of)
  __device__ static __forceinline__ float phi_dir(float qa, float qb, float& ea, float& eb, const Consts& c) {
    if constexpr (M == TRANSE) {
      const float v = HEAD ? (ea + qa) : (qa - ea);
      ea = sgnf(v);
      return fabsf(v);
    } else if constexpr (M == DISTMULT) {
      return HEAD ? (ea * qa) : (qa * ea);
    } else if constexpr (M == COMPLEX) {
      return HEAD ? (ea * qa + eb * qb) : (qa * ea + qb * eb);
    } else if constexpr (M == ROTATE) {
      const float dr = qa - ea, di = qb - eb;
      const float rho = fsqrt(dr * dr + di * di);
      const float inv = (rho > 0.f) ? frcp(rho) : 0.f;
      ea = dr * inv;
      eb = di * inv;
      return rho;
    } else {
      const float pe = ea / c.kappa_p;
      const float x = HEAD ? (pe + qa) : (qa - pe);
      float sn, cs;
      sincosf(x, &sn, &cs);
      ea = sgnf(sn) * cs;
      return fabsf(sn);
    }
  }
  // d score / d q from phi_dir's transformed element, scaled by w
  __device__ static __forceinline__ void dq_of(float ga, float gb, float w, const Consts& c, float& oa, float& ob) {
    if constexpr (M == TRANSE || M == ROTATE) {
      oa = -w * ga;
      ob = -w * gb;
    } else if constexpr (M == PROTATE) {
      oa = -(w * c.modulus) * ga;
      ob = 0.f;
    } else {
      oa = w * ga;
      ob = w * gb;
    }
  }

  // d score / d modulus = -phi summed (pRotatE only); uses the raw total.

  // chain d q → d x (head for tail/single, tail for head-batch) and d r
  __device__ static __forceinline__ void chain(float xa, float xb, float ra, float rb, float dqa, float dqb,
                                               const Consts& c, float& dxa, float& dxb, float& dra,
                                               float& drb) {
    if constexpr (M == TRANSE) {
      dra = dqa;
      dxa = HEAD ? -dqa : dqa;
      dxb = drb = 0.f;
    } else if constexpr (M == DISTMULT) {
      // tail q = x*r ; head q = r*x
      dxa = dqa * ra;
      dra = dqa * xa;
      dxb = drb = 0.f;
    } else if constexpr (M == COMPLEX) {
      if constexpr (HEAD) {
        // qa = ra xa + rb xb ; qb = ra xb - rb xa   (x = tail)
        dxa = dqa * ra - dqb * rb;
        dxb = dqa * rb + dqb * ra;
        dra = dqa * xa + dqb * xb;
        drb = dqa * xb - dqb * xa;
      } else {
        // qa = xa ra - xb rb ; qb = xa rb + xb ra   (x = head)
        dxa = dqa * ra + dqb * rb;
        dxb = dqb * ra - dqa * rb;
        dra = dqa * xa + dqb * xb;
        drb = dqb * xa - dqa * xb;
      }
    } else if constexpr (M == ROTATE) {
      const float th = ra / c.kappa;
      float sn, cs;
      sincosf(th, &sn, &cs);
      float dth;
      if constexpr (HEAD) {
        // qa = cs xa + sn xb ; qb = cs xb - sn xa
        dxa = dqa * cs - dqb * sn;
        dxb = dqa * sn + dqb * cs;
        const float qa = cs * xa + sn * xb, qb = cs * xb - sn * xa;
        dth = dqa * qb - dqb * qa;
      } else {
        // qa = xa cs - xb sn ; qb = xa sn + xb cs
        dxa = dqa * cs + dqb * sn;
        dxb = dqb * cs - dqa * sn;
        const float qa = xa * cs - xb * sn, qb = xa * sn + xb * cs;
        dth = dqb * qa - dqa * qb;
      }
      dra = dth / c.kappa;
      drb = 0.f;
    } else {
      dra = dqa / c.kappa_p;
      dxa = HEAD ? -(dqa / c.kappa_p) : (dqa / c.kappa_p);
      dxb = drb = 0.f;
    }
  }
};

// Sum of phi over the lane's slots (fixed ascending order).
template <int M, int MODE, int NS, int VEC, bool CPLX>
__device__ __forceinline__ float lane_total(const Row<NS, VEC, CPLX>& q, const Row<NS, VEC, CPLX>& e,
                                            const Consts& c) {
  using EL = Elem<M, MODE>;
  float acc = 0.f;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      float t;
      if constexpr (CPLX) t = EL::phi(q.a[s][v], q.b[s][v], e.a[s][v], e.b[s][v], c);
      else t = EL::phi(q.a[s][v], 0.f, e.a[s][v], 0.f, c);
      acc += t;
    }
  }
  return acc;
}

// q for a row: x = head row (tail/single) or tail row (head-batch).
template <int M, int MODE, int NS, int VEC, bool CPLX>
__device__ __forceinline__ void build_q(const Row<NS, VEC, CPLX>& x, const Row<NS, VEC, CPLX>& r,
                                        const Consts& c, Row<NS, VEC, CPLX>& q) {
  using EL = Elem<M, MODE>;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      float qa, qb;
      if constexpr (CPLX) EL::make_q(x.a[s][v], x.b[s][v], r.a[s][v], r.b[s][v], c, qa, qb);
      else EL::make_q(x.a[s][v], 0.f, r.a[s][v], 0.f, c, qa, qb);
      q.a[s][v] = qa;
      if constexpr (CPLX) q.b[s][v] = qb;
    }
  }
}

// Load the relation row into a Row: RotatE phases go to `a` (b unused).
template <int M, int NS, int VEC, bool CPLX>
__device__ __forceinline__ void load_rel(const float* __restrict__ base, RowGeom eg, int lane,
                                         Row<NS, VEC, CPLX>& r) {
  if constexpr (Traits<M>::rel_phase) {
    load_phase<NS, VEC>(base, eg.S, lane, r.a);
#pragma unroll
    for (int s = 0; s < NS; ++s) zv<VEC>(r.b[s]);
  } else {
    load_row<NS, VEC, CPLX>(base, eg, lane, r);
  }
}
template <int M, int NS, int VEC, bool CPLX>
__device__ __forceinline__ void store_rel(float* __restrict__ base, RowGeom eg, int lane,
                                          const Row<NS, VEC, CPLX>& r) {
  if constexpr (Traits<M>::rel_phase) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int slot = lane + 64 * s;
      if (slot < eg.S) stv<VEC>(base + slot * VEC, r.a[s]);
    }
  } else {
    store_row<NS, VEC, CPLX>(base, eg, lane, r);
  }
}

}  // namespace kge
