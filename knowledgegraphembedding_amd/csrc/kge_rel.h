// kge_rel.h — the relation-row gradient pass and the loss finalisation as
// device functions, shared by k_rel_rows / k_finalize (kge_common.hip) and the
// trailing blocks of k_entity_sl.
#pragma once
#include "kge_internal.h"

namespace kge {

// -------------------------------------------------- relation gradient rows
// One wave per relation row: Σ of the rows' relation contributions in id
// order (+ 3λ r|r|), written densely; with a fused optimizer the Adam update
// of the row is applied while the gradient is in registers.  Lanes own float4
// chunks c = lane + 64u of the row (scalar tail when Lr % 4 != 0).
// P4: four occurrence rows in flight (the standalone k_rel_rows; the trailing
// blocks of k_entity_sl keep one, so the entity pass's register budget is
// not set by this path)
template <int U, bool P4 = false>
__device__ __forceinline__ void rel_row_chunks(const RelArgs& a, int64_t rr, int lane) {
  // the rows of this relation: its CSR bucket (ascending occurrence ids)
  const int32_t b0 = a.off[a.E + rr], b1 = a.off[a.E + rr + 1];
  const float* row = a.rel + rr * a.Lr;
  const bool v4 = (a.Lr % 4) == 0;
  const int nchunk = v4 ? a.Lr / 4 : a.Lr;  // float4 chunks, or single floats
  float part = 0.f;
  for (int c0 = 0; c0 < nchunk; c0 += 64 * U) {
    float acc[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[u][e] = 0.f;
    int32_t p = b0;
    if (P4 && v4) {
      // four occurrences' rows in flight per iteration (a relation can have
      // thousands of occurrences in a large global batch); the sums keep the
      // ascending occurrence order, so the bits are those of the plain loop
      for (; p + 4 <= b1; p += 4) {
        float4 x[4][U];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float4* src = reinterpret_cast<const float4*>(a.rel_contrib + (a.occ[p + t] - a.Bn - 2 * a.B) * a.Lr);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int c = c0 + u * 64 + lane;
            x[t][u] = (c < nchunk) ? src[c] : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u][0] += x[t][u].x; acc[u][1] += x[t][u].y; acc[u][2] += x[t][u].z; acc[u][3] += x[t][u].w;
          }
      }
    }
    // the occurrences in order (the rest of the bucket)
    for (; p < b1; ++p) {
      const int64_t i = a.occ[p] - a.Bn - 2 * a.B;
      const float* src = a.rel_contrib + i * a.Lr;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = c0 + u * 64 + lane;
        if (c < nchunk) {
          if (v4) {
            const float4 x = reinterpret_cast<const float4*>(src)[c];
            acc[u][0] += x.x; acc[u][1] += x.y; acc[u][2] += x.z; acc[u][3] += x.w;
          } else {
            acc[u][0] += src[c];
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * 64 + lane;
      if (c >= nchunk) continue;
      const int nel = v4 ? 4 : 1;
      const int k0 = v4 ? 4 * c : c;
      float x[4] = {0.f, 0.f, 0.f, 0.f};
      for (int e = 0; e < nel; ++e) x[e] = row[k0 + e];
      for (int e = 0; e < nel; ++e) {
        if (a.reg3 != 0.f) {
          acc[u][e] += a.reg3 * (x[e] * fabsf(x[e]));
          part += fabsf(x[e]) * x[e] * x[e];
        }
        if (a.write_grad) a.grad_rel[rr * a.Lr + k0 + e] = acc[u][e];
      }
      if (a.adam.p) {
        float* P = a.adam.p + rr * a.Lr + k0;
        float* Mm = a.adam.m + rr * a.Lr + k0;
        float* Vv = a.adam.v + rr * a.Lr + k0;
        for (int e = 0; e < nel; ++e) {
          float pv = x[e], mv = Mm[e], vv = Vv[e];
          adam_elem(pv, acc[u][e], mv, vv, a.adamk, a.adam.step_size, a.adam.bc2s);
          P[e] = pv; Mm[e] = mv; Vv[e] = vv;
        }
      }
    }
  }
  if (a.reg3 != 0.f) {
    part = wave_sum(part);
    if (lane == 0) a.reg_partial[rr] = part;
  }
}

// ------------------------------------------------------------ finalise
// Loss scalars (model.py:279-297) and d/dmodulus, one workgroup of NT threads.
// The sums are those of 1024 virtual threads v (rows v, v + 1024, ...) folded
// as a 1024-wide tree whatever NT is: the levels o >= NT in registers, the
// rest in LDS — so k_finalize (NT = 1024) and the entity launch's fused last
// block (NT = 256) produce identical bits.  red: [6][NT] floats of LDS.
template <int NT>
__device__ __forceinline__ void finalize_block(const FinArgs& a, float* red) {
  constexpr int V = 1024, K = V / NT;
  const int tid = threadIdx.x;
  float acc[6][K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float sw = 0.f, swp = 0.f, swn = 0.f, sp = 0.f, sn = 0.f, mg = 0.f;
    for (int64_t i = tid + k * NT; i < a.B; i += V) {
      const float* st = a.row_stats + i * 4;
      const float w = a.sub_w ? a.sub_w[i] : 1.f;
      sw += w;
      swp += w * st[0];
      swn += w * st[1];
      sp += st[0];
      sn += st[1];
      mg += st[2];
    }
    acc[0][k] = sw; acc[1][k] = swp; acc[2][k] = swn;
    acc[3][k] = sp; acc[4][k] = sn; acc[5][k] = mg;
  }
  auto tree = [&](float (&x)[K], float* r) -> float {
    // virtual v < o takes v + o: for o >= NT that is register k + o/NT
#pragma unroll
    for (int o = V / 2; o >= NT; o >>= 1)
#pragma unroll
      for (int k = 0; k < o / NT; ++k) x[k] += x[k + o / NT];
    r[tid] = x[0];
    __syncthreads();
    for (int o = NT / 2; o > 0; o >>= 1) {
      if (tid < o) r[tid] += r[tid + o];
      __syncthreads();
    }
    const float t = r[0];
    __syncthreads();
    return t;
  };
  float tot[6];
#pragma unroll
  for (int u = 0; u < 6; ++u) tot[u] = tree(acc[u], red + u * NT);
  float reg = 0.f;
  const int64_t na = a.reg_a1 - a.reg_a0, nreg = na + (a.reg_b1 - a.reg_b0);
  if (a.reg_partial && nreg > 0) {
    float s[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      s[k] = 0.f;
      for (int64_t v = tid + k * NT; v < nreg; v += V) s[k] += a.reg_partial[v < na ? a.reg_a0 + v : a.reg_b0 + (v - na)];
    }
    reg = a.regularization * tree(s, red);
  }
  if (tid == 0) {
    float pos_loss, neg_loss;
    if (a.uni_weight) {
      // - score.mean(): sum / batch  (model.py:282-283)
      pos_loss = -(tot[3] / a.uni_n);
      neg_loss = -(tot[4] / a.uni_n);
    } else {
      // - (w * score).sum() / w.sum()  (model.py:285-286)
      const float wsum = a.w_sum ? a.w_sum[0] : tot[0];
      pos_loss = -(tot[1] / wsum);
      neg_loss = -(tot[2] / wsum);
    }
    float loss = (pos_loss + neg_loss) / 2.f;
    loss = loss + reg;
    if (a.losses) {
      a.losses[0] = pos_loss;
      a.losses[1] = neg_loss;
      a.losses[2] = loss;
      a.losses[3] = reg;
      // the device error flag rides along, so the caller's one read-back of
      // the losses also tells it whether any index was out of range
      a.losses[4] = a.err ? (float)__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
    }
    if (a.grad_modulus) a.grad_modulus[0] = tot[5];
    if (a.adam.p) {  // pRotatE modulus, fused optimizer step
      float pv = a.adam.p[0], mv = a.adam.m[0], vv = a.adam.v[0];
      adam_elem(pv, tot[5], mv, vv, a.adamk, a.adam.step_size, a.adam.bc2s);
      a.adam.p[0] = pv; a.adam.m[0] = mv; a.adam.v[0] = vv;
    }
  }
}

}  // namespace kge
