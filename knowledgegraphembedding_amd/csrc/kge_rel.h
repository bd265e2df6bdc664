// kge_rel.h — the relation-row gradient pass as a device function, shared by
// k_rel_rows (kge_common.hip) and the trailing blocks of k_entity_sl.
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

}  // namespace kge
