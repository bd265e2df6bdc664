// kge_rank_mfma.hip — filtered ranking for the bilinear models (DistMult,
// ComplEx) as an fp32 MFMA tile (model.py:346-418 with TestDataset's filter,
// dataloader.py:134-154).
//
// Both models score a candidate e as a dot product of the query vector q
// (DistMult: h∘r or r∘t; ComplEx: the rotated complex vector, [re | im]) with
// the candidate's stored row, so a block of queries against all entities is
// S = Q · Eᵀ.  v_mfma_f32_32x32x2_f32 computes exact fp32 as a k-ordered fma
// chain; the true entity's score comes from the SAME kernel in "gather" mode
// (B columns = the queries' true rows), so s_true and every candidate score
// are produced by identical instruction sequences and compare consistently.
//
// Tile: 128 queries × 128 candidates per workgroup (4 waves as 2×2, each
// 64×64 = 2×2 MFMA tiles), K staged through LDS 32 deep, rows kept row-major
// with each 8-k group permuted into MFMA consumption order, so one
// ds_read_b128 per operand feeds four k-steps; the next slab's global loads
// are issued into registers before the current slab's MFMAs, so their
// latency hides behind the matrix work.
// Candidates are the MFMA rows and queries the columns, so each lane owns two
// query columns: the epilogue tests its 32 candidates per query against s_true
// and a 2-word slice of the query's exclusion bitmap (filtered ids, the true
// id, ids past E) with plain per-lane integer counts, adds the two lane halves,
// and issues one LDS and then one global integer atomic per (block, query):
// exact and order-free.  Candidates within the query's near-tie window are not
// counted but listed (win_count) for the reference-order refinement
// (kge_rank_ref.h): the fma order here is not the reference's sum order.
#include "kge_common.h"

namespace kge {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 32;
// LDS slab: row-major [128 rows][LDK], each group of 8 k stored in MFMA
// consumption order [k0, k0+2, k0+4, k0+6 | k0+1, k0+3, k0+5, k0+7] so one
// ds_read_b128 gives a lane (row li, half kh) its operands for 4 k-steps.
constexpr int LDK = BK + 4;
constexpr int F4 = (BM * BK / 4) / 256;  // float4 per thread per operand per slab

struct MfmaArgs {
  const float* q;        // [nq, K]
  const float* ent;      // [E, K]
  int64_t nq, E;
  int K;
  const int64_t* true_id;  // [nq]
  float* s_true;           // [nq]  gather pass writes, scan pass reads
  const uint32_t* fbits;   // [nq, W] filtered-candidate bitmap (scan pass)
  int64_t W;
  int32_t* gt;             // [nq]
  RankWin win;
};

// One [128 rows × BK] slab of row-major [*, K] data: thread t holds float4
// f = t + 256u (row f / (BK/4), k = (f % (BK/4))·4 .. +3) in registers
// (fetch), then writes it transposed into LDS as [k][row] (put).
__device__ __forceinline__ void fetch(float4 (&r)[F4], const float* __restrict__ src, const int64_t* rows, int K,
                                      int k0, int t) {
#pragma unroll
  for (int u = 0; u < F4; ++u) {
    const int f = t + 256 * u;
    const int row = f / (BK / 4), kq = (f % (BK / 4)) * 4;
    const int64_t gr = rows[row];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gr >= 0) {
      const float* p = src + gr * (int64_t)K + k0 + kq;
      if (k0 + kq + 3 < K) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        if (k0 + kq + 0 < K) v.x = p[0];
        if (k0 + kq + 1 < K) v.y = p[1];
        if (k0 + kq + 2 < K) v.z = p[2];
      }
    }
    r[u] = v;
  }
}
__device__ __forceinline__ void put(float (*dst)[LDK], const float4 (&r)[F4], int t) {
#pragma unroll
  for (int u = 0; u < F4; ++u) {
    const int f = t + 256 * u;
    const int row = f / (BK / 4), kq = (f % (BK / 4)) * 4;
    // k = kq..kq+3 → positions (k & 1)·4 + ((k & 7) >> 1) inside the 8-group
    const int base = (kq & ~7) + ((kq & 4) ? 2 : 0);
    *reinterpret_cast<float2*>(&dst[row][base]) = make_float2(r[u].x, r[u].z);
    *reinterpret_cast<float2*>(&dst[row][base + 4]) = make_float2(r[u].y, r[u].w);
  }
}

template <bool GATHER>
__global__ __launch_bounds__(256, 3) void k_rank_mfma(MfmaArgs a) {
  __shared__ __attribute__((aligned(16))) float As[BM][LDK];
  __shared__ __attribute__((aligned(16))) float Bs[BN][LDK];
  __shared__ int64_t arow[128], brow[128];
  __shared__ float sts[128], sdl[128];
  __shared__ int32_t cgt[128];
  const int t = threadIdx.x, lane = t & 63, w = wave_id();
  const int wm = w >> 1, wn = w & 1;
  const int64_t q0 = (int64_t)blockIdx.y * BM;
  const int64_t e0 = (int64_t)blockIdx.x * BN;
  if (t < 128) {
    const int64_t q = q0 + t;
    arow[t] = (q < a.nq) ? q : -1;
    const int64_t tid_ = (q < a.nq) ? a.true_id[q] : -1;
    if (GATHER) {
      brow[t] = (tid_ >= 0 && tid_ < a.E) ? tid_ : -1;
    } else {
      const int64_t e = e0 + t;
      brow[t] = (e < a.E) ? e : -1;
      sts[t] = (q < a.nq) ? a.s_true[q] : 0.f;
      sdl[t] = (q < a.nq) ? a.win.delta[q] : 0.f;
    }
    cgt[t] = 0;
  }
  __syncthreads();

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int kh = lane >> 5, li = lane & 31;
  float4 ra[F4], rb[F4];
  fetch(ra, a.q, arow, a.K, 0, t);
  fetch(rb, a.ent, brow, a.K, 0, t);
  for (int k0 = 0; k0 < a.K; k0 += BK) {
    put(As, ra, t);
    put(Bs, rb, t);
    __syncthreads();
    if (k0 + BK < a.K) {  // next slab's global loads in flight behind the MFMAs
      fetch(ra, a.q, arow, a.K, k0 + BK, t);
      fetch(rb, a.ent, brow, a.K, k0 + BK, t);
    }
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      // k order: step 4g + u takes k = k0 + 8g + 2u (lanes 0-31) and + 1
      // (lanes 32-63) — ascending k across the loop, the same in both passes.
      // Candidates are the MFMA rows (A), queries the columns (B): a lane's
      // accumulator column is one query, so the epilogue counts per lane.
      float4 e4[2], q4[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) e4[i] = *reinterpret_cast<const float4*>(&Bs[wm * 64 + i * 32 + li][g * 8 + kh * 4]);
#pragma unroll
      for (int j = 0; j < 2; ++j) q4[j] = *reinterpret_cast<const float4*>(&As[wn * 64 + j * 32 + li][g * 8 + kh * 4]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float ef[2] = {u == 0 ? e4[0].x : u == 1 ? e4[0].y : u == 2 ? e4[0].z : e4[0].w,
                             u == 0 ? e4[1].x : u == 1 ? e4[1].y : u == 2 ? e4[1].z : e4[1].w};
        const float qf[2] = {u == 0 ? q4[0].x : u == 1 ? q4[0].y : u == 2 ? q4[0].z : q4[0].w,
                             u == 0 ? q4[1].x : u == 1 ? q4[1].y : u == 2 ? q4[1].z : q4[1].w};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ef[i], qf[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // C/D layout: col (query) = lane & 31, row (candidate) = (reg & 3) + 8·(reg >> 2) + 4·(lane >> 5)
  if (GATHER) {
    // diagonal: candidate row m == query column n; for column li that is
    // register r = 4·(li >> 3) + (li & 3) of the lane half kh = (li >> 2) & 1
    if (wm != wn || kh != ((li >> 2) & 1)) return;
    const int rd = 4 * (li >> 3) + (li & 3);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = wn * 64 + i * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r == rd && arow[n] >= 0) a.s_true[q0 + n] = acc[i][i][r];
    }
    return;
  }
  const int64_t wbase = e0 >> 5;  // the tile's 128 candidates = bitmap words wbase .. wbase+3
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 64 + j * 32 + li;
    const int64_t q = arow[n];
    const float st = sts[n], dlt = sdl[n];
    // excluded candidates of this query among rows wm·64 .. +63: filtered ids
    // and the true id (bitmap), and ids past E
    uint32_t ex[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t widx = wbase + wm * 2 + i;
      const int64_t cbase = e0 + wm * 64 + i * 32;
      uint32_t word = (q >= 0 && widx < a.W) ? a.fbits[q * a.W + widx] : ~0u;
      const int64_t valid = a.E - cbase;
      if (valid < 32) word |= (valid <= 0) ? ~0u : (~0u << valid);
      ex[i] = word;
    }
    int g = 0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mloc = (r & 3) + 8 * (r >> 2) + 4 * kh;
        const bool ok = ((ex[i] >> mloc) & 1u) == 0u;
        const float sc = acc[i][j][r];
        const float diff = sc - st;
        g += (ok && diff > dlt) ? 1 : 0;
        if (ok && !(diff > dlt) && diff >= -dlt) {  // near tie: listed, not counted
          const int idx = atomicAdd(&a.win.ucnt[q], 1);
          if (idx < a.win.cap) a.win.ulist[q * (int64_t)a.win.cap + idx] = (int32_t)(e0 + wm * 64 + i * 32 + mloc);
        }
      }
    // lanes l and l + 32 hold the two row halves of the same query column
    g += __shfl_xor(g, 32);
    if (kh == 0 && q >= 0 && g) atomicAdd(&cgt[n], g);
  }
  __syncthreads();
  if (t < 128 && arow[t] >= 0 && cgt[t]) atomicAdd(&a.gt[q0 + t], cgt[t]);
}

// filtered-candidate bitmap from the CSR (one thread per filtered id)
__global__ __launch_bounds__(256) void k_filter_bits(const int64_t* __restrict__ off, const int64_t* __restrict__ ids,
                                                     const int64_t* __restrict__ true_id, int64_t nq, int64_t E,
                                                     int64_t W, uint32_t* __restrict__ bits, int32_t* err) {
  const int64_t q = blockIdx.y;
  if (q >= nq) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the true entity is never counted against itself
    const int64_t t = true_id[q];
    if (t >= 0 && t < E) atomicOr(&bits[q * W + (t >> 5)], 1u << (t & 31));
  }
  const int64_t b = off[q], e_ = off[q + 1];
  for (int64_t p = b + (int64_t)blockIdx.x * 256 + threadIdx.x; p < e_; p += (int64_t)gridDim.x * 256) {
    const int64_t e = ids[p];
    if (e < 0 || e >= E) {
      atomicOr(err, KGE_DEVERR_INDEX);
      continue;
    }
    atomicOr(&bits[q * W + (e >> 5)], 1u << (e & 31));
  }
}

// rank = 1 + #{strictly greater} (counted beyond the window + refined inside
// it), or the exact rescan's count for an overflowed window
__global__ __launch_bounds__(256) void k_rank_emit(EmitArgs a) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= a.nq) return;
  const bool ok = a.true_id[q] >= 0;
  const bool ovf = a.ucnt[q] > a.cap;
  a.ranks[q] = ok ? 1 + (int64_t)(ovf ? a.gtx[q] : a.gt[q]) : 0;
  if (a.ties) a.ties[q] = ok ? (ovf ? a.eqx[q] : a.eq[q]) : 0;
  if (a.listed) a.listed[q] = ok ? a.ucnt[q] : 0;
}

}  // namespace

int launch_filter_bits(const int64_t* filt_off, const int64_t* filt_ids, const int64_t* true_id, int64_t nq,
                       int64_t E, uint32_t* bits, int32_t* err, hipStream_t s) {
  const int64_t W = (E + 31) / 32;
  hipError_t he = hipMemsetAsync(bits, 0, (size_t)nq * W * 4, s);
  if (he != hipSuccess) return (int)he;
  if (nq > 65535) return -1;
  hipLaunchKernelGGL(k_filter_bits, dim3(4, (unsigned)nq), dim3(256), 0, s, filt_off, filt_ids, true_id, nq, E, W,
                     bits, err);
  return (int)hipGetLastError();
}

int launch_rank_emit(const EmitArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_rank_emit, dim3((unsigned)((a.nq + 255) / 256)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// q and true ids come from k_rank_prep.  gather = 1: s_true (the queries'
// true rows as the candidate block, diagonal kept); 0: the counting pass
// against all E candidates, with the window from k_rank_window.
int launch_rank_mfma(int gather, const float* q, const float* ent, int64_t nq, int64_t E, int K,
                     const int64_t* true_id, float* s_true, const uint32_t* bits, int32_t* gt, const RankWin& win,
                     hipStream_t s) {
  MfmaArgs a;
  a.q = q; a.ent = ent; a.nq = nq; a.E = E; a.K = K; a.true_id = true_id; a.s_true = s_true;
  a.fbits = bits; a.W = (E + 31) / 32; a.gt = gt; a.win = win;
  const unsigned gy = (unsigned)((nq + BM - 1) / BM);
  // 3 waves/SIMD (158 VGPRs, no spills); 4 fits only with 13 spilled VGPRs
  // and measured 12 % slower
  if (gather) {
    hipLaunchKernelGGL((k_rank_mfma<true>), dim3(1, gy), dim3(256), 0, s, a);
  } else {
    const dim3 gs((unsigned)((E + BN - 1) / BN), gy);
    hipLaunchKernelGGL((k_rank_mfma<false>), gs, dim3(256), 0, s, a);
  }
  return (int)hipGetLastError();
}

// Entity-table statistics for the ranking windows: stats[0] = max row L2
// norm, stats[1] = max |x| (non-negative floats order like their bit
// patterns, so an integer atomicMax is exact).  One wave per row, rows
// strided over a bounded grid; the block's four waves combine in LDS and the
// block issues one atomic per statistic (an atomic per row on the same two
// words serialised: 0.93 ms for wn18rr's 40,943 rows).
__global__ __launch_bounds__(256) void k_table_stats(const float* __restrict__ ent, int64_t E, int Le,
                                                     float* stats) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, w = wave_id();
  float bn = 0.f, bm = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * 4 + w; e < E; e += (int64_t)gridDim.x * 4) {
    const float* row = ent + e * Le;
    float s2 = 0.f, mx = 0.f;
    if ((Le & 3) == 0 && (((uintptr_t)ent) & 15) == 0) {  // float4 rows
      for (int k = lane; k < Le / 4; k += 64) {
        const float4 v = reinterpret_cast<const float4*>(row)[k];
        s2 += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    } else {
      for (int k = lane; k < Le; k += 64) {
        const float v = row[k];
        s2 += v * v;
        mx = fmaxf(mx, fabsf(v));
      }
    }
    s2 = wave_sum(s2);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    bn = fmaxf(bn, sqrtf(s2) * 1.0001f);
    bm = fmaxf(bm, mx);
  }
  if (lane == 0) { red[0][w] = bn; red[1][w] = bm; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float n = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    const float m = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
    atomicMax(reinterpret_cast<unsigned int*>(&stats[0]), __float_as_uint(n));
    atomicMax(reinterpret_cast<unsigned int*>(&stats[1]), __float_as_uint(m));
  }
}

int launch_table_stats(const float* ent, int64_t E, int Le, float* stats, hipStream_t s) {
  hipError_t e = hipMemsetAsync(stats, 0, 2 * sizeof(float), s);
  if (e != hipSuccess) return (int)e;
  const int64_t blocks = (E + 3) / 4;  // one row per wave: every row in flight at once
  hipLaunchKernelGGL(k_table_stats, dim3((unsigned)(blocks < 65535 ? blocks : 65535)), dim3(256), 0, s, ent, E, Le,
                     stats);
  return (int)hipGetLastError();
}

}  // namespace kge
