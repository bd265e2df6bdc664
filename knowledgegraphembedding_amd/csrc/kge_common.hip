// kge_common.hip — model-independent kernels: occurrence CSR (deterministic
// counting sort), relation-gradient row sums, loss finalisation, Σw and Adam.
#include <rocprim/device/device_scan.hpp>

#include <cstdlib>

#include "kge_common.h"
#include "kge_rel.h"

namespace kge {

// -------------------------------------------------------------- CSR build
// Keys of one training/backward call, in id order:
//   [0, Bn)            negative occurrence (i, j): entity neg[i*ns + j]
//   [Bn, Bn+2B)        row slot s: entity pos[(s/2)*3 + (s&1 ? 2 : 0)]
//   [Bn+2B, Bn+3B)     relation of row i: bucket E + pos[i*3 + 1]
__global__ __launch_bounds__(256) void k_csr_hist(CsrArgs a) {
  const int64_t N = a.Bn + 3 * a.B;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < N; k += (int64_t)gridDim.x * 256) {
    int64_t key;
    if (k < a.Bn) {
      const int64_t i = k / a.n, j = k - i * a.n;
      key = a.neg[i * a.neg_stride + j];
      if (key < 0 || key >= a.E) key = -1;
    } else if (k < a.Bn + 2 * a.B) {
      const int64_t s = k - a.Bn;
      key = a.pos[(s >> 1) * 3 + ((s & 1) ? 2 : 0)];
      if (key < 0 || key >= a.E) key = -1;
    } else {
      const int64_t i = k - a.Bn - 2 * a.B;
      key = a.pos[i * 3 + 1];
      key = (key < 0 || key >= a.R) ? -1 : (a.E + key);
    }
    if (key < 0) {
      atomicOr(a.err, KGE_DEVERR_INDEX);
      a.keys[k] = -1;
      continue;
    }
    if (key < a.E && (key < a.e_lo || key >= a.e_hi)) {  // another owner's row: not bucketed here
      a.keys[k] = -1;
      continue;
    }
    a.keys[k] = (int32_t)key;
    atomicAdd(&a.cnt[key], 1);
  }
}

// Unordered fill: slot = off[key] + (--cnt[key]).
__global__ __launch_bounds__(256) void k_csr_fill(CsrArgs a) {
  const int64_t N = a.Bn + 3 * a.B;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < N; k += (int64_t)gridDim.x * 256) {
    const int32_t key = a.keys[k];
    if (key < 0) continue;
    const int32_t p = atomicSub(&a.cnt[key], 1) - 1;
    a.tmp[a.off[key] + p] = (int32_t)k;
  }
}

// Deterministic order: each id's final slot is its rank among the ids of its
// bucket (ids are unique), so buckets come out ascending whatever order the
// atomics filled them in.  One wave per bucket: the bucket's ids are read once,
// 64 at a time, and each lane counts the smaller ids by broadcasting the
// others' lane by lane (readlane) — ⌈m/64⌉²·64 register steps per bucket
// instead of m global reads per id, which matters once buckets hold
// hundreds of ids (the factor exchange's global batch).
__device__ __forceinline__ void csr_rank_bucket(const CsrArgs& a, int64_t b, int lane) {
  const int32_t b0 = a.off[b], b1 = a.off[b + 1];
  for (int32_t c0 = b0; c0 < b1; c0 += 64) {
    const bool mine = c0 + lane < b1;
    const int32_t v = mine ? a.tmp[c0 + lane] : 0x7fffffff;
    int32_t r = 0;
    for (int32_t d0 = b0; d0 < b1; d0 += 64) {
      const int32_t o = (d0 + lane < b1) ? a.tmp[d0 + lane] : 0x7fffffff;
      const int cnt = (b1 - d0 < 64) ? (b1 - d0) : 64;
      for (int l = 0; l < cnt; ++l) r += (__builtin_amdgcn_readlane(o, l) < v) ? 1 : 0;
    }
    if (mine) a.occ[b0 + r] = v;
  }
}
__global__ __launch_bounds__(256) void k_csr_rank_w(CsrArgs a, int64_t nb) {
  const int lane = threadIdx.x & 63;
  for (int64_t b = (int64_t)blockIdx.x * 4 + wave_id(); b < nb; b += (int64_t)gridDim.x * 4)
    csr_rank_bucket(a, b, lane);
}

__global__ __launch_bounds__(256) void k_rel_rows(RelArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t rr = (int64_t)blockIdx.x * 4 + wave_id();
  if (rr >= a.R) return;
  rel_row_chunks<4, true>(a, rr, lane);
}

// ------------------------------------------------------------ finalise
// Loss scalars (model.py:279-297) and d/dmodulus.  One workgroup, fixed
// reduction order (finalize_block, kge_rel.h).
__global__ __launch_bounds__(1024) void k_finalize(FinArgs a) {
  __shared__ float red[6 * 1024];
  finalize_block<1024>(a, red);
}

// Same fixed order as k_row's / k_build_q's in-kernel Σw (block_weight_sum,
// 256 threads), so a Σw computed here is bit-identical to the one a single
// process computes for the same weights (the data-parallel factor exchange).
__global__ __launch_bounds__(256) void k_weight_sum(const float* __restrict__ w, int64_t n, float* out) {
  __shared__ float red[256];
  const float tot = block_weight_sum(w, n, red);
  if (threadIdx.x == 0) out[0] = tot;
}

// ------------------------------------------------------------------ Adam
// Standalone dense Adam over one tensor (KGEAdam.step / kge_adam_step).
// NT: non-temporal (streaming) loads/stores — every byte is touched once.
// U: float4 groups per thread and iteration (loads of all U issued first).
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* base, int64_t i) {
  if constexpr (NT) {
    const tf4 v = __builtin_nontemporal_load(reinterpret_cast<const tf4*>(base) + i);
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return reinterpret_cast<const float4*>(base)[i];
  }
}
template <bool NT>
__device__ __forceinline__ void st4(float* base, int64_t i, const float4& x) {
  if constexpr (NT) __builtin_nontemporal_store(tf4{x.x, x.y, x.z, x.w}, reinterpret_cast<tf4*>(base) + i);
  else reinterpret_cast<float4*>(base)[i] = x;
}
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v, int64_t n, AdamK k,
                                              float step_size, float bc2s) {
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += stride * U) {
    float4 P[U], G[U], Mv[U], Vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n4) {
        P[u] = ld4<NT>(p, i); G[u] = ld4<NT>(g, i); Mv[u] = ld4<NT>(m, i); Vv[u] = ld4<NT>(v, i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n4) continue;
      adam_elem(P[u].x, G[u].x, Mv[u].x, Vv[u].x, k, step_size, bc2s);
      adam_elem(P[u].y, G[u].y, Mv[u].y, Vv[u].y, k, step_size, bc2s);
      adam_elem(P[u].z, G[u].z, Mv[u].z, Vv[u].z, k, step_size, bc2s);
      adam_elem(P[u].w, G[u].w, Mv[u].w, Vv[u].w, k, step_size, bc2s);
      st4<NT>(p, i, P[u]);
      st4<NT>(m, i, Mv[u]);
      st4<NT>(v, i, Vv[u]);
    }
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float P = p[i], Mv = m[i], Vv = v[i];
    adam_elem(P, g[i], Mv, Vv, k, step_size, bc2s);
    p[i] = P; m[i] = Mv; v[i] = Vv;
  }
}

// ------------------------------------------------------------ launchers
static inline unsigned grid_for(int64_t n, unsigned cap = 4096) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  return (unsigned)(g < cap ? g : cap);
}

// Bucket offsets: a device-wide exclusive scan of cnt[0..nb] (cnt[nb] = 0, so
// off[nb] = total) — rocPRIM's decoupled look-back scan, integer and exact;
// its scratch comes from the caller's workspace.
size_t csr_scan_temp_bytes(int64_t nb) {
  static thread_local int64_t last_nb = -1;  // the query is per size; remember the last one
  static thread_local size_t last_bytes = 0;
  if (nb == last_nb) return last_bytes;
  size_t bytes = 0;
  if (rocprim::exclusive_scan(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr, int32_t(0), (size_t)nb + 1,
                              rocprim::plus<int32_t>()) != hipSuccess)
    bytes = 0;
  last_nb = nb;
  last_bytes = bytes;
  return bytes;
}

int launch_csr(const CsrArgs& a, hipStream_t s) {
  const int64_t nb = a.E + a.R;
  const int64_t N = a.Bn + 3 * a.B;
  // (grids capped at 32 / 128 / 512 blocks, to leave k_row more CU slots,
  // measured 0.697 / 0.578 / 0.559-0.560 ms per step against 0.561: the CSR
  // has to finish inside k_row's window; profiles/r06/csr/bench_cap*.json)
  const unsigned gk = grid_for(N);
  const unsigned gb = (unsigned)((nb + 3) / 4);
  hipError_t e = hipMemsetAsync(a.cnt, 0, sizeof(int32_t) * (nb + 1), s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_csr_hist, dim3(gk), dim3(256), 0, s, a);
  // (one-workgroup scan measured instead: no gain at FB15k, 469.5-471.1 vs
  // 470.5-471.9 M triples/s, and 0.19 ms of join at YAGO3-10's 123 k buckets;
  // its launch, like rocPRIM's, shows ≈210 µs beside k_row: waiting for a
  // slot, not working; profiles/r06/csr/)
  size_t bytes = a.scan_tmp_bytes;
  e = rocprim::exclusive_scan(a.scan_tmp, bytes, a.cnt, a.off, int32_t(0), (size_t)nb + 1, rocprim::plus<int32_t>(), s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_csr_fill, dim3(gk), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_csr_rank_w, dim3(gb), dim3(256), 0, s, a, nb);
  return (int)hipGetLastError();
}

int launch_rel_rows(const RelArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_rel_rows, dim3((unsigned)((a.R + 3) / 4)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int launch_finalize(const FinArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, s, a);
  return (int)hipGetLastError();
}

int launch_weight_sum(const float* w, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_weight_sum, dim3(1), dim3(256), 0, s, w, n, out);
  return (int)hipGetLastError();
}

int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float b1, float b2, float eps,
                float step_size, float bc2s, hipStream_t s) {
  AdamK k;
  k.b1 = b1; k.b2 = b2; k.eps = eps;
  // non-temporal, two float4 groups per thread and iteration: 5.6 TB/s on the
  // FB15k table against 5.0-5.2 for plain float4 (profiles/r01/adam_rate_variants.jsonl)
  const dim3 grid(grid_for((n + 3) / 4, 8192));
  hipLaunchKernelGGL((k_adam<true, 2>), grid, dim3(256), 0, s, p, g, m, v, n, k, step_size, bc2s);
  return (int)hipGetLastError();
}

}  // namespace kge
