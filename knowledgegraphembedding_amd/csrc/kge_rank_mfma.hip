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
// 64×64 = 2×2 MFMA tiles), K staged through LDS 16 deep by LDS-DMA into two
// alternating buffers (details at k_rank_mfma).
// Candidates are the MFMA rows and queries the columns, so each lane owns two
// query columns: the epilogue tests its 32 candidates per query against s_true
// and a 2-word slice of the query's exclusion bitmap (filtered ids, the true
// id, ids past E) with plain per-lane integer counts, adds the two lane halves,
// and issues one LDS and then one global integer atomic per (block, query):
// exact and order-free.  Candidates within the query's near-tie window are not
// counted but listed (win_count) for the reference-order refinement
// (kge_rank_ref.h): the fma order here is not the reference's sum order.
#include <algorithm>
#include <cstdlib>

#include "kge_common.h"
#include "kge_rank_ref.h"

namespace kge {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128;

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

// The tile's K slabs go global → LDS by LDS-DMA
// (buffer_load_dwordx4 … lds: no staging VGPRs, no LDS write pass), 16 deep
// and double-buffered, so each slab costs one barrier and its loads run behind
// the previous slab's MFMAs; 36 KB of LDS and ≤ 128 VGPRs give 4 workgroups
// per CU.  The DMA image is lane-linear (16 rows × 64 B per wave-instruction),
// so the k order inside an MFMA step is chosen to read contiguous 16-B chunks:
// step u of 8-group g pairs k = 8g + u (lanes 0-31) with k = 8g + 4 + u
// (lanes 32-63), and each row's four 16-B chunks are XOR-swizzled by
// (row >> 2) & 3 on the SOURCE address, which makes every ds_read_b128 of the
// operand fragments conflict-free.  Rows past nq / E and k ≥ K read as zero
// (buffer range check), so edge tiles need no selects.  Same epilogue as v1;
// the fast score's fma order differs from v1 (the near-tie window bounds any
// order, and the gather pass runs the same kernel).  An earlier version
// staged 32-deep slabs through registers with two barriers per slab (158
// VGPRs, 3 workgroups per CU): 68 % MFMA-busy against 79 % here.
constexpr int BK2 = 16;
constexpr int STAGE2 = 2 * 128 * BK2;  // floats per stage: A [128][16] then B [128][16]
constexpr uint32_t OOB2 = 0x7FFFFFF0u;

template <bool GATHER>
__global__ __launch_bounds__(256, 4) void k_rank_mfma(MfmaArgs a) {
  // one LDS array (a second __shared__ object can cost a vmcnt(0) per k-step):
  // [2 stages][A | B] slabs, then arow/brow (int64), sts, sdl, cgt
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE2 + 128 * 2 + 128 * 2 + 128 * 3];
  int64_t* arow = reinterpret_cast<int64_t*>(smem + 2 * STAGE2);
  int64_t* brow = arow + 128;
  float* sts = reinterpret_cast<float*>(brow + 128);
  float* sdl = sts + 128;
  int32_t* cgt = reinterpret_cast<int32_t*>(sdl + 128);
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

  const auto rq = buf_rsrc(a.q, (uint64_t)a.nq * a.K * 4u);
  const auto re = buf_rsrc(a.ent, (uint64_t)a.E * a.K * 4u);
  // this lane's DMA pieces: wave-instruction t2 ∈ {2w, 2w+1} of each operand
  // covers rows 16·t2 .. +15, lane l → row 16·t2 + l/4, LDS chunk p = l & 3,
  // source chunk p ^ ((row >> 2) & 3)
  int64_t growA[2], growB[2];
  int cpos[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 16 * (2 * w + h) + (lane >> 2);
    growA[h] = arow[row];
    growB[h] = brow[row];
    cpos[h] = (lane & 3) ^ ((row >> 2) & 3);
  }
  auto issue = [&](int k0, int stage) {
    float* base = smem + stage * STAGE2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kk = k0 + 4 * cpos[h];
      const bool kin = kk < a.K;
      const uint32_t oa = (kin && growA[h] >= 0) ? (uint32_t)((growA[h] * a.K + kk) * 4) : OOB2;
      const uint32_t ob = (kin && growB[h] >= 0) ? (uint32_t)((growB[h] * a.K + kk) * 4) : OOB2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (__attribute__((address_space(3))) void*)(base + (2 * w + h) * 256),
                                               16, oa, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          re, (__attribute__((address_space(3))) void*)(base + 128 * BK2 + (2 * w + h) * 256), 16, ob, 0, 0, 0);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int kh = lane >> 5, li = lane & 31;
  const int nslab = (a.K + BK2 - 1) / BK2;
  // a wave whose 64 queries (or 64 candidates) all lie past nq (E) still
  // loads its share of every slab, but issues no MFMA: its SIMD's matrix core
  // goes to the co-resident workgroups (wn = 1 of the last query row of
  // blocks for wn18rr's 3134 queries: 2 % of the launch)
  const bool live = q0 + wn * 64 < a.nq && (GATHER || e0 + wm * 64 < a.E);
  // the epilogue's exclusion-bitmap words, loaded now so their latency hides
  // behind the K loop (loaded at the end they cost two memory round trips
  // per block: with the split tile 19 % of the launch)
  uint32_t exw[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t q = q0 + wn * 64 + j * 32 + (lane & 31);
      const int64_t widx = (e0 >> 5) + wm * 2 + i;
      const int64_t cbase = e0 + wm * 64 + i * 32;
      uint32_t word = (!GATHER && q < a.nq && widx < a.W) ? a.fbits[q * a.W + widx] : ~0u;
      const int64_t valid = a.E - cbase;
      if (valid < 32) word |= (valid <= 0) ? ~0u : (~0u << valid);
      exw[j][i] = word;
    }
  issue(0, 0);
  for (int s = 0; s < nslab; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of slab s has landed
    __syncthreads();                                   // ... every wave's; slab s-1's reads are done
    if (s + 1 < nslab) issue((s + 1) * BK2, (s + 1) & 1);
    if (!live) continue;
    const float* As = smem + (s & 1) * STAGE2;
    const float* Bs = As + 128 * BK2;
    const int kv = a.K - s * BK2;  // k past the reduction length read as 0: skip whole 8-k groups of them
#pragma unroll
    for (int g = 0; g < BK2 / 8; ++g) {
      if (g > 0 && 8 * g >= kv) break;
      float4 e4[2], q4[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 32 + li;
        e4[i] = *reinterpret_cast<const float4*>(Bs + row * BK2 + 4 * ((2 * g + kh) ^ ((row >> 2) & 3)));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wn * 64 + j * 32 + li;
        q4[j] = *reinterpret_cast<const float4*>(As + row * BK2 + 4 * ((2 * g + kh) ^ ((row >> 2) & 3)));
      }
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
  }

  // C/D layout: col (query) = lane & 31, row (candidate) = (reg & 3) + 8·(reg >> 2) + 4·(lane >> 5)
  if (GATHER) {
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
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 64 + j * 32 + li;
    const int64_t q = arow[n];
    const float st = sts[n], dlt = sdl[n];
    const uint32_t ex[2] = {exw[j][0], exw[j][1]};
    // branch-free count; the rare near-ties collect in a bit mask and are
    // listed in one loop afterwards (a branch per candidate cost more than
    // the count itself)
    // an excluded candidate's score becomes −∞ first: then "counted" is
    // d > δ and "near" is |d| ≤ δ (−δ ≤ d ≤ δ; false for −∞ and NaN), the
    // same sets as ok ∧ d > δ and ok ∧ ¬(d > δ) ∧ d ≥ −δ with fewer live
    // compare masks
    int g = 0;
    uint32_t near = 0;  // bit 16·i + r
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mloc = (r & 3) + 8 * (r >> 2) + 4 * kh;
        const float sc = ((ex[i] >> mloc) & 1u) ? -__builtin_inff() : acc[i][j][r];
        const float diff = sc - st;
        g += (diff > dlt) ? 1 : 0;
        near |= (__builtin_fabsf(diff) <= dlt) ? (1u << (16 * i + r)) : 0u;
      }
    if (__builtin_amdgcn_ballot_w64(near != 0u)) {
      while (near) {
        const int b = __builtin_ctz(near);
        near &= near - 1u;
        const int i = b >> 4, r = b & 15;
        const int mloc = (r & 3) + 8 * (r >> 2) + 4 * kh;
        const int idx = atomicAdd(&a.win.ucnt[q], 1);
        if (idx < a.win.cap) a.win.ulist[q * (int64_t)a.win.cap + idx] = (int32_t)(e0 + wm * 64 + i * 32 + mloc);
      }
    }
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

// The same bitmap from the whole filter index (KGE_RANK_FILTER_TABLE): one
// wave per query looks its key's range up in the dense start table and sets
// the bits of that range's ids (and the true id's)
__global__ __launch_bounds__(256) void k_filter_bits_tab(const int64_t* __restrict__ queries, int head,
                                                         const int64_t* __restrict__ tab,
                                                         const int64_t* __restrict__ vals,
                                                         const int64_t* __restrict__ true_id, int64_t nq, int64_t E,
                                                         int64_t R, int64_t W, uint32_t* __restrict__ bits,
                                                         int32_t* err) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= nq) return;
  const int64_t t = true_id[q];
  if (lane == 0 && t >= 0 && t < E) atomicOr(&bits[q * W + (t >> 5)], 1u << (t & 31));
  const int64_t h = queries[q * 3], r = queries[q * 3 + 1], tl = queries[q * 3 + 2];
  if (h < 0 || h >= E || tl < 0 || tl >= E || r < 0 || r >= R) return;  // (k_rank_prep flags bad ids)
  const int64_t key = head ? r * E + tl : h * R + r;
  const int64_t b = tab[key], e_ = tab[key + 1];
  for (int64_t p = b + lane; p < e_; p += 64) {
    const int64_t e = vals[p];
    if (e < 0 || e >= E) {
      atomicOr(err, KGE_DEVERR_INDEX);
      continue;
    }
    atomicOr(&bits[q * W + (e >> 5)], 1u << (e & 31));
  }
}

// Both bitmaps in one pass per query, built in LDS: one 256-thread block per
// query zeroes its W-word row in LDS, sets the true id's and the filtered
// ids' bits there (LDS atomics), and writes the whole row out with coalesced
// stores — no separate memset of the [nq, W] bitmap and no global atomics.
// `tab` non-null: the filter index's dense key → start table (k_filter_bits_tab's
// lookup, `head` picks the key); else per-query lists off / ids.  A grid of
// 2·nq blocks ranks both directions: blocks nq.. are tail-batch's, with the
// tail table / lists (tab1 / off1, ids1), the same queries and the second half
// of true_id and bits.
__global__ __launch_bounds__(256) void k_filter_bits_lds(const int64_t* __restrict__ queries, int head,
                                                         const int64_t* __restrict__ tab,
                                                         const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ ids,
                                                         const int64_t* __restrict__ true_id, int64_t nq, int64_t E,
                                                         int64_t R, int W, uint32_t* __restrict__ bits,
                                                         int32_t* err, const int64_t* __restrict__ tab1,
                                                         const int64_t* __restrict__ off1,
                                                         const int64_t* __restrict__ ids1) {
  extern __shared__ uint32_t fb_row[];
  const int64_t q = blockIdx.x;  // (index into true_id and bits)
  const bool d1 = q >= nq;
  const int64_t ql = d1 ? q - nq : q;  // (index into queries and the lists)
  if (d1) {
    tab = tab1;
    off = off1;
    ids = ids1;
    head = 0;
  }
  const int tid = threadIdx.x;
  for (int k = tid; k < W; k += 256) fb_row[k] = 0u;
  __syncthreads();
  const int64_t t = true_id[q];
  if (tid == 0 && t >= 0 && t < E) atomicOr(&fb_row[t >> 5], 1u << (t & 31));
  int64_t b = 0, e_ = 0;
  if (tab) {
    const int64_t h = queries[ql * 3], r = queries[ql * 3 + 1], tl = queries[ql * 3 + 2];
    if (h >= 0 && h < E && tl >= 0 && tl < E && r >= 0 && r < R) {  // (k_rank_prep flags bad ids)
      const int64_t key = head ? r * E + tl : h * R + r;
      b = tab[key];
      e_ = tab[key + 1];
    }
  } else {
    b = off[ql];
    e_ = off[ql + 1];
  }
  for (int64_t p = b + tid; p < e_; p += 256) {
    const int64_t e = ids[p];
    if (e < 0 || e >= E) {
      atomicOr(err, KGE_DEVERR_INDEX);
      continue;
    }
    atomicOr(&fb_row[e >> 5], 1u << (e & 31));
  }
  __syncthreads();
  uint32_t* dst = bits + q * (int64_t)W;
  for (int k = tid; k < W; k += 256) dst[k] = fb_row[k];
}

// rows up to this many words go through k_filter_bits_lds (E ≤ 393,216)
constexpr int FB_LDS_WORDS = 12288;

// rank = 1 + #{strictly greater} (counted beyond the window + refined inside
// it), or the exact rescan's count for an overflowed window
__global__ __launch_bounds__(256) void k_rank_emit(EmitArgs a) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (a.ltag && q == 0) {  // (pRotatE list stage) what the later stages must match
    a.ltag[0] = a.ltag_v[0];
    a.ltag[1] = a.ltag_v[1];
    a.ltag[2] = a.ltag_v[2];
  }
  if (q >= a.nq) return;
  const bool ok = a.true_id[q] >= 0;
  const bool ovf = a.ucnt[q] > a.cap;
  if (a.ranks) a.ranks[q] = ok ? 1 + (int64_t)(ovf ? a.gtx[q] : a.gt[q]) : 0;  // null: lists only
  if (a.ties) a.ties[q] = ok ? (ovf ? a.eqx[q] : a.eq[q]) : 0;
  if (a.listed) a.listed[q] = ok ? a.ucnt[q] : 0;
}


// --------------------------------------------------------------------------
// Split-bf16 MFMA tile (path "mfma", the default for DistMult / ComplEx).
//
// fp32 MFMA runs at 1/16 of the bf16 rate on gfx950 (v_mfma_f32_32x32x2_f32:
// 64 cycles per 4096 flop; v_mfma_f32_32x32x16_bf16: 32 cycles per 32768).
// The fast pass only has to place each candidate on the right side of s_true
// up to the near-tie window — the window's candidates are re-scored in the
// reference's fp32 order anyway — so it may compute in any precision whose
// error it bounds.  Each operand x is split as x = x_hi + x_lo + r with
// x_hi = bf16(x), x_lo = bf16(x − x_hi), both round-to-nearest-even with 8
// significant bits: |x − x_hi| ≤ 2^-8 |x|, |x_lo| ≤ 2^-8 (1 + 2^-8) |x|,
// |r| ≤ 2^-16 |x|.  Per 16-k slab one MFMA chain computes e_hi·q_hi from a
// zero accumulator, then adds e_hi·q_lo and e_lo·q_hi (bf16 × bf16 products
// are exact in fp32); the chain's result joins an fp32 running sum (one
// rounding per slab); e_lo·q_lo is never computed.  Error per score against
// the exact Σ e_k q_k, u = 2^-24, P = Σ|q_k||e_k| ≤ ‖q‖‖e‖:
//   the split itself         Σ|q||r_e| + Σ|r_q||e| + Σ|r_q||r_e| + Σ|q_lo||e_lo|
//                            ≤ ‖q‖‖r_e‖ + ‖r_q‖‖e‖ + ‖r_q‖‖r_e‖ + ‖q_lo‖‖e_lo‖, from the
//                            pieces' actual norms (round 6; k_split_stats / k_table_stats
//                            keep the table's maxima, k_rank_window computes q's) — the
//                            worst case 2·2^-16·P + 2^-16 (1 + 2^-8)^2·P = 770·u·P of
//                            rounds 4-5 is ≈ 126·u·P on uniform tables
//   the final add            1.2·u·P
//   the three chained MFMAs  ≤ 32·u each on partial sums ≤ (1 + 2^-8)^2 (1 + 2^-7)·P_slab
//                            (2u per internal add, any order)      →  97.6·u·P
//   the running sum          1.02·nslab·u·P
// → fast_u = (98.8 + 1.02·nslab)·u·P plus the split term (kge_capi.hip rank_impl,
// RefArgs.fast_u; the window k_rank_window sizes from both), against the fp32 tile's K·u.
//
// Operands are split once per call into a tile-linear layout
// [row block of 128][16-k slab][hi | lo][128 rows][16 k] bf16 (k_split_bf16),
// so each slab of a 128-row block is 8 KB contiguous: four 1 KB LDS-DMA
// instructions per piece.  Row r's k-half h sits at r·32 + (h ^ r₃)·16 bytes
// (r₃ = bit 3 of r): gfx950 serves a ds_read_b128 in lane groups
// {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, … whose rows, unswizzled, put
// two lanes on every bank quad of a group they use (2-way conflicts, half
// the banks idle: SQ_LDS_BANK_CONFLICT ≈ the LDS-active cycles); with the
// swap each group's 16 lanes cover all 64 banks.  Rows past nq / E and k ≥ K are
// zeros in the split buffers.
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int XS_BK = 16;                   // k per slab = one 32x32x16 MFMA step
constexpr int XS_PIECE = 128 * XS_BK;       // bf16 per (row block, slab, hi|lo) = 4 KB
constexpr uint32_t XS_OOB = 0x7FFFFFF0u;

// dst[(rb·nslab + s)·2 + piece][rr][kk] for rows < rows, k < K (zeros elsewhere).
// A wave takes 8 rows × 64 k: lane (r8, g8) = (lane >> 3, lane & 7) converts
// the 8 floats k = 64·chunk + 8·g8 … of row 8·group + r8, so each row is read
// as 256 contiguous bytes and, per slab, the 8 rows' hi (lo) pieces are
// written as 256 contiguous bytes.
__global__ __launch_bounds__(256) void k_split_bf16(const float* __restrict__ src, int64_t rows, int K, int nslab,
                                                    int64_t nrb, uint16_t* __restrict__ dst, const int64_t* skip) {
  if (skip && *skip) return;  // the workspace already holds this table's split (k_rank_tag)
  const int64_t wg = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int nc = (nslab * XS_BK + 63) / 64;  // 64-k chunks per row
  const int64_t rg = wg / nc;
  if (rg >= nrb * 16) return;
  const int kg = (int)(wg % nc) * 8 + (lane & 7);  // 8-k group
  if (kg >= nslab * 2) return;
  const int64_t row = rg * 8 + (lane >> 3);
  const int k0 = kg * 8;
  float x[8];
  const float* p = src + row * K + k0;
  if (row < rows && k0 + 8 <= K && ((K & 3) == 0) && ((((uintptr_t)src) & 15) == 0)) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (row < rows && k0 + j < K) ? p[j] : 0.f;
  }
  uint32_t hi[8], lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = bf16_rne(x[j]);
    lo[j] = bf16_rne(x[j] - __uint_as_float(hi[j] << 16));  // exact difference
  }
  const uint4 vh = {hi[0] | (hi[1] << 16), hi[2] | (hi[3] << 16), hi[4] | (hi[5] << 16), hi[6] | (hi[7] << 16)};
  const uint4 vl = {lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16), lo[4] | (lo[5] << 16), lo[6] | (lo[7] << 16)};
  const int64_t rb = row >> 7;
  uint16_t* o = dst + ((rb * nslab + (kg >> 1)) * 2) * XS_PIECE + (row & 127) * XS_BK +
                ((kg & 1) ^ (int)((row >> 3) & 1)) * 8;
  *reinterpret_cast<uint4*>(o) = vh;
  *reinterpret_cast<uint4*>(o + XS_PIECE) = vl;
}

// The entity table's split and its statistics (k_table_stats' four maxima,
// TS_NSTAT) in one read of the table: a wave takes 8 whole rows (lane
// (r8, g8) converts floats 64·c + 8·g8 … of row r8 for every 64-k chunk c, the
// same per-slab stores as k_split_bf16), its 8 lanes per row reduce the row's
// sums, and each block writes its partial maxima to stats[4 + 4·block] for
// k_stats_reduce.  Row groups are strided
// over ≤ TS_BLOCKS blocks.  (The separate statistics pass re-read the 84 MB
// wn18rr table: 19 µs of a 1.07 ms DistMult evaluation.)
// one row's contribution to the TS_NSTAT maxima from its Σx², max |x| and
// the Σ of its scaled split pieces (bf16_split_scaled: lo·2^8, r·2^16); each
// norm × mg = 1.0001 + Le·3.1e-8 for its fp32 sum of ≤ Le terms in any order
// (√ of a γ_Le-relative sum: ≤ γ_Le / 2 + u)
__device__ __forceinline__ void table_stats_row(float (&bs)[TS_NSTAT], float s2, float mx, float sl, float sr,
                                                float mg) {
  bs[0] = fmaxf(bs[0], sqrtf(s2) * mg);
  bs[1] = fmaxf(bs[1], mx);
  bs[2] = fmaxf(bs[2], sqrtf(sr) * mg * 0x1p-16f);
  bs[3] = fmaxf(bs[3], sqrtf(sl) * mg * 0x1p-8f);
}

__global__ __launch_bounds__(256) void k_split_stats(const float* __restrict__ src, int64_t rows, int K, int nslab,
                                                     int64_t nrb, uint16_t* __restrict__ dst, float* stats,
                                                     const int64_t* skip_stats, const int64_t* skip_split) {
  const bool do_stats = !(skip_stats && *skip_stats), do_split = !(skip_split && *skip_split);
  if (!do_stats && !do_split) return;  // the workspace holds both for this table (k_rank_tag)
  __shared__ float red[TS_NSTAT][4];
  const int lane = threadIdx.x & 63, w = wave_id();
  const int r8 = lane >> 3, g8 = lane & 7;
  const int nc = (nslab * XS_BK + 63) / 64;  // 64-k chunks per row
  const bool vec = ((K & 3) == 0) && ((((uintptr_t)src) & 15) == 0);
  float bs[TS_NSTAT] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t rg = (int64_t)blockIdx.x * 4 + w; rg < nrb * 16; rg += (int64_t)gridDim.x * 4) {
    const int64_t row = rg * 8 + r8;
    const int64_t rb = row >> 7;
    float s2 = 0.f, mx = 0.f, sr = 0.f, sl = 0.f;
    for (int c = 0; c < nc; ++c) {
      const int kg = c * 8 + g8;  // 8-k group
      if (kg >= nslab * 2) break;
      const int k0 = kg * 8;
      float x[8];
      const float* p = src + row * K + k0;
      if (row < rows && k0 + 8 <= K && vec) {
        const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = (row < rows && k0 + j < K) ? p[j] : 0.f;
      }
      uint32_t hi[8], lo[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s2 += x[j] * x[j];
        mx = fmaxf(mx, fabsf(x[j]));
        hi[j] = bf16_rne(x[j]);
        lo[j] = bf16_rne(x[j] - __uint_as_float(hi[j] << 16));  // exact difference
        float l8, r16;
        bf16_split_scaled(x[j], l8, r16);
        sl += l8 * l8;
        sr += r16 * r16;
      }
      if (do_split) {
        const uint4 vh = {hi[0] | (hi[1] << 16), hi[2] | (hi[3] << 16), hi[4] | (hi[5] << 16), hi[6] | (hi[7] << 16)};
        const uint4 vl = {lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16), lo[4] | (lo[5] << 16), lo[6] | (lo[7] << 16)};
        uint16_t* o = dst + ((rb * nslab + (kg >> 1)) * 2) * XS_PIECE + (row & 127) * XS_BK +
                      ((kg & 1) ^ (int)((row >> 3) & 1)) * 8;
        *reinterpret_cast<uint4*>(o) = vh;
        *reinterpret_cast<uint4*>(o + XS_PIECE) = vl;
      }
    }
    // the row's 8 lanes: the sums (any order: the norms' 1.0001 covers γ_K) and max |x|
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      s2 += __shfl_xor(s2, o);
      sl += __shfl_xor(sl, o);
      sr += __shfl_xor(sr, o);
      mx = fmaxf(mx, __shfl_xor(mx, o));
    }
    table_stats_row(bs, s2, mx, sl, sr, 1.0001f + (float)K * 3.1e-8f);
  }
  if (!do_stats) return;
#pragma unroll
  for (int o = 8; o < 64; o <<= 1)
#pragma unroll
    for (int i = 0; i < TS_NSTAT; ++i) bs[i] = fmaxf(bs[i], __shfl_xor(bs[i], o));
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < TS_NSTAT; ++i) red[i][w] = bs[i];
  __syncthreads();
  if (threadIdx.x < TS_NSTAT) {
    const int i = threadIdx.x;
    stats[TS_NSTAT + TS_NSTAT * blockIdx.x + i] = fmaxf(fmaxf(red[i][0], red[i][1]), fmaxf(red[i][2], red[i][3]));
  }
}

struct XArgs {
  const uint16_t* qs;  // split q
  const uint16_t* es;  // split entity table
  uint32_t qs_bytes, es_bytes;
  int64_t nq, E;
  int nslab;
  int gx, gy, group;   // counting pass: candidate / query tiles, candidate tiles per L2 group (xcd_tile)
  const int64_t* true_id;
  float* s_true;
  const uint32_t* fbits;
  int64_t W;
  int32_t* gt;
  RankWin win;
};

// Counting pass tile order.  Workgroups are dealt to the 8 XCDs round-robin
// (b mod 8), each XCD with its own 4 MB L2.  XCD k takes the candidate tiles
// x ≡ k (mod 8) in groups of `group` tiles (≤ 2 MB of split rows) and runs
// every query tile against one group before the next: a candidate tile is
// fetched into that L2 once per group instead of once per query tile (the
// plain grid re-read the whole 84 MB split table from MALL for each of
// wn18rr's 25 query tiles: 2.2 GB per launch, 43 % MFMA-busy).  The order is
// a speed property only.  Returns false for the grid's idle tail blocks.
__device__ __forceinline__ bool xcd_tile(const XArgs& a, int& x, int& y) {
  const int b = blockIdx.x, k = b & 7, i = b >> 3;  // (1-D grid)
  const int nxk = (a.gx - k + 7) >> 3;  // candidate tiles of XCD k
  if (i >= nxk * a.gy) return false;
  const int per = a.group * a.gy;
  const int g = i / per, rem = i - g * per;
  const int gsz = min(a.group, nxk - g * a.group);
  x = (g * a.group + rem % gsz) * 8 + k;
  y = rem / gsz;
  return true;
}

// The counting tile: 256 threads as 2 × 2 waves over 128 candidates × 128
// queries, 64 × 64 per wave (2 × 2 blocks of 32 × 32), a 3-stage LDS ring
// (two slabs in flight), three workgroups per CU (≈170 VGPRs).  Per 16-k slab
// and 32 × 32 block, hi·hi starts a fresh MFMA chain (zero accumulator) and
// the hi·lo and lo·hi products chain onto it; the chain's result is added to
// the fp32 running sum one slab later (so no add waits on its MFMA).  The lo·lo
// product is not computed: its |e_lo q_lo| ≤ 2^-16 |e||q| joins the window's
// bound (launch_rank_mfma_x's caller, fast_u).  Measured and rejected, the
// numbers in DESIGN §5 and profiles/r04/rank/: a separate correction
// accumulator, a 4-stage ring at two workgroups per CU, 64 × 32 per wave, a
// 256-candidate 8-wave tile with 4-6 ring stages, a persistent ring, keeping
// the lo·lo product, and (round 5) the same tile on v_mfma_f32_16x16x32_bf16
// (each MFMA over a 32-k slab pair, 4 × 4 blocks of 16 × 16 per wave, 199
// VGPRs, two workgroups per CU: DistMult 399-404 against 374-375 µs, ComplEx
// 705-714 against 711-712, profiles/r05/rank/ab_tile_16x16x32_rejected.txt),
// and (round 6) two slabs per ring stage in a 2-stage ring — half the
// barriers and DMA waits, two workgroups per CU in the same 64 KB: 875 against
// 773 µs per two-direction DistMult launch — and a 2-stage one-slab ring (one
// slab in flight, 37 KB, four workgroups per CU): 798 against 767 µs
// (profiles/r06/rank_tile/).
// s_waitcnt vmcnt(n) for the DMA counts of the ring (n = younger slabs × CPW)
__device__ __forceinline__ void wait_vmcnt_dma(int n) {
  switch (n) {
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

struct XTile {
  static constexpr int TQ = 2;                   // 32-query column tiles per wave
  static constexpr int BQ = 64 * TQ;             // queries per workgroup
  static constexpr int BNX = 128;                // candidates per workgroup
  static constexpr int NST = 3;                  // LDS ring stages (NST − 1 slabs in flight)
  // bf16 per ring stage: E hi | lo (4 KB each), then Q hi | lo (2·TQ KB each)
  static constexpr int STAGE = (8 + 4 * TQ) * 512;
  static constexpr int CPW = (8 + 4 * TQ) / 4;   // 1 KB DMA chunks per wave per slab
};

template <bool GATHER>
__global__ __launch_bounds__(256, 3) void k_rank_mfma_x(XArgs a) {
  using X = XTile;
  constexpr int TQ = X::TQ, NST = X::NST;
  // one LDS array: [NST stages][E_hi | E_lo | Q_hi | Q_lo] then arow/brow, sts, sdl, cgt
  __shared__ __attribute__((aligned(16))) uint16_t smem[NST * X::STAGE + 128 * 4 * 2 + 128 * 2 * 2 + 128 * 2 * 3];
  int64_t* arow = reinterpret_cast<int64_t*>(smem + NST * X::STAGE);
  int64_t* brow = arow + 128;
  float* sts = reinterpret_cast<float*>(brow + 128);
  float* sdl = sts + 128;
  int32_t* cgt = reinterpret_cast<int32_t*>(sdl + 128);
  const int t = threadIdx.x, lane = t & 63, w = wave_id();
  const int wm = w >> 1, wn = w & 1;
  int tx = 0, ty = (int)blockIdx.y;
  if (!GATHER && !xcd_tile(a, tx, ty)) return;  // (block-uniform)
  const int64_t q0 = (int64_t)ty * X::BQ;
  const int64_t e0 = (int64_t)tx * X::BNX;
  if (t < 128) {
    const int64_t q = q0 + t;
    const bool in = t < X::BQ && q < a.nq;
    arow[t] = in ? q : -1;
    const int64_t tid_ = in ? a.true_id[q] : -1;
    if (GATHER) {
      brow[t] = (tid_ >= 0 && tid_ < a.E) ? tid_ : -1;  // candidate row t = query t's true entity
    } else {
      sts[t] = in ? a.s_true[q] : 0.f;
      sdl[t] = in ? a.win.delta[q] : 0.f;
    }
    cgt[t] = 0;
  }
  __syncthreads();

  const auto rq = buf_rsrc(a.qs, a.qs_bytes);
  const auto re = buf_rsrc(a.es, a.es_bytes);
  const int nslab = a.nslab;
  // 1 KB chunk c of a stage (LDS bytes c·1024 …): c < 8 candidate pieces (hi
  // 0-3, lo 4-7; 32 rows each), then the query pieces (hi, lo: 2·TQ chunks
  // each).  Wave w moves chunks CPW·w … CPW·w + CPW − 1.
  int64_t grow[X::CPW];  // GATHER: this lane's source row of each candidate chunk
#pragma unroll
  for (int k = 0; k < X::CPW; ++k) {
    const int c = X::CPW * w + k;
    grow[k] = (GATHER && c < 8) ? brow[(c & 3) * 32 + (lane >> 1)] : 0;
  }
  const int64_t qrb = (int64_t)ty * X::BQ / 128;           // the queries' 128-row block in the split layout
  const uint32_t qsub = (uint32_t)((ty * X::BQ) & 127) * 32;  // … and their byte offset inside it
  // each chunk's source offset at slab 0, computed once: a slab adds its hi +
  // lo pieces (8 KB) in both split layouts, so the loop only adds sl · 8 KB
  // (GATHER: XS_OOB stays out of range for absent rows)
  constexpr uint32_t SLAB_BYTES = 2u * (2u * XS_PIECE);
  uint32_t off0[X::CPW];
#pragma unroll
  for (int k = 0; k < X::CPW; ++k) {
    const int c = X::CPW * w + k;
    if (c < 8) {
      const int piece = (c >> 2) & 1, sub = c & 3;
      if (GATHER) {
        const int64_t r = grow[k];
        // LDS row (lane >> 1) of the chunk, half (lane & 1) holds k-half
        // (lane & 1) ^ (bit 3 of that row); the source keeps its own swap
        const int src_half = (lane & 1) ^ ((lane >> 4) & 1) ^ (int)((r >> 3) & 1);
        off0[k] = (r >= 0) ? (uint32_t)(((r >> 7) * nslab * 2 + piece) * (2 * XS_PIECE) + (r & 127) * 32 +
                                        src_half * 16)
                           : XS_OOB;
      } else {
        off0[k] = (uint32_t)((((int64_t)tx * nslab * 2 + piece) * (2 * XS_PIECE) + sub * 1024 + lane * 16));
      }
    } else {
      const int cc = c - 8, piece = cc / (2 * TQ), sub = cc % (2 * TQ);
      off0[k] = (uint32_t)((qrb * nslab * 2 + piece) * (2 * XS_PIECE) + qsub + sub * 1024 + lane * 16);
    }
  }
  auto issue = [&](int sl, int st) {
    uint16_t* base = smem + st * X::STAGE;
#pragma unroll
    for (int k = 0; k < X::CPW; ++k) {
      const int c = X::CPW * w + k;
      const uint32_t off = (GATHER && off0[k] == XS_OOB) ? XS_OOB : off0[k] + (uint32_t)sl * SLAB_BYTES;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(c < 8 ? re : rq,
                                               (__attribute__((address_space(3))) void*)(base + c * 512), 16, off, 0,
                                               0, 0);
    }
  };
  // DMAs issued after slab sl's, when sl is waited for: those of the next
  // min(NST − 2, nslab − 1 − sl) slabs, CPW instructions each (vmcnt counts in order)
  static_assert(X::CPW == 4 && NST == 3, "vmcnt immediates of wait_vmcnt_dma");
  auto wait_slab = [&](int sl) {
    const int left = nslab - 1 - sl;
    const int after = left < NST - 2 ? left : NST - 2;
    wait_vmcnt_dma(after * X::CPW);
  };

  f32x16 run[2][TQ], mprev[2][TQ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TQ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) run[i][j][r] = mprev[i][j][r] = 0.f;
  const f32x16 zero = {};

  const int kh = lane >> 5, li = lane & 31;
  const int khs = kh ^ ((li >> 3) & 1);  // the k-half's slot in the swapped row (every fragment row ≡ li mod 32)
  const int wq0 = wn * 32 * TQ;  // this wave's first query column in the workgroup
  const bool live = q0 + wq0 < a.nq && (GATHER || e0 + wm * 64 < a.E);
  // the epilogue's exclusion-bitmap words, loaded now so their latency hides
  // behind the K loop
  uint32_t exw[TQ][2];
#pragma unroll
  for (int j = 0; j < TQ; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t q = q0 + wq0 + j * 32 + li;
      const int64_t widx = (e0 >> 5) + wm * 2 + i;
      const int64_t cbase = e0 + wm * 64 + i * 32;
      uint32_t word = (!GATHER && q < a.nq && widx < a.W) ? a.fbits[q * a.W + widx] : ~0u;
      const int64_t valid = a.E - cbase;
      if (valid < 32) word |= (valid <= 0) ? ~0u : (~0u << valid);
      exw[j][i] = word;
    }
#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nslab) issue(p, p);
  for (int sl = 0; sl < nslab; ++sl) {
    wait_slab(sl);                 // this wave's DMA of slab sl has landed
    __builtin_amdgcn_s_barrier();  // ... every wave's; slab sl-1's reads are done (no fence: the
                                   // vmcnt above covers the DMA, __syncthreads' would be vmcnt(0))
    if (sl + NST - 1 < nslab) issue(sl + NST - 1, (sl + NST - 1) % NST);
    if (!live) continue;
    const uint16_t* Es = smem + (sl % NST) * X::STAGE;
    const uint16_t* Qh = Es + 2 * XS_PIECE;
    const uint16_t* Ql = Qh + TQ * 1024;
    bf16x8 eh[2], el[2], qh[TQ], ql[TQ];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wm * 64 + i * 32 + li;
      eh[i] = *reinterpret_cast<const bf16x8*>(Es + row * XS_BK + khs * 8);
      el[i] = *reinterpret_cast<const bf16x8*>(Es + XS_PIECE + row * XS_BK + khs * 8);
    }
#pragma unroll
    for (int j = 0; j < TQ; ++j) {
      const int row = wq0 + j * 32 + li;
      qh[j] = *reinterpret_cast<const bf16x8*>(Qh + row * XS_BK + khs * 8);
      ql[j] = *reinterpret_cast<const bf16x8*>(Ql + row * XS_BK + khs * 8);
    }
    // the running sum takes the PREVIOUS slab's chain (long done: an add
    // right behind the MFMA it reads stalls the wave ~40 cycles), then this
    // slab's hi·hi, hi·lo and lo·hi MFMAs chain from zero
    // the MFMA block at raised wave priority: with three waves per SIMD on one
    // matrix core, a wave that reached its MFMAs issues them ahead of the
    // others' fragment reads and DMA issue (DistMult 385 -> 378-387 us, ComplEx
    // 735 -> 716-717 us, alternated; the reads / DMA raised instead: 383 / 727-732,
    // profiles/r05/rank/ab_setprio.txt)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TQ; ++j) {
        run[i][j] += mprev[i][j];  // (v_pk_add_f32 pairs)
        mprev[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(eh[i], qh[j], zero, 0, 0, 0);
        mprev[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(eh[i], ql[j], mprev[i][j], 0, 0, 0);
        mprev[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(el[i], qh[j], mprev[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  }
  f32x16 acc[2][TQ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TQ; ++j) acc[i][j] = run[i][j] + mprev[i][j];

  // C/D layout as the fp32 tile: col (query) = lane & 31, row (candidate) = (reg & 3) + 8·(reg >> 2) + 4·(lane >> 5)
  if (GATHER) {
    // query n's true row is candidate row n: wave wm = n / 64, tile i = (n % 64) / 32, row li
    if (kh != ((li >> 2) & 1)) return;
    const int rd = 4 * (li >> 3) + (li & 3);
#pragma unroll
    for (int j = 0; j < TQ; ++j) {
      const int n = wq0 + j * 32 + li;
      if ((n >> 6) != wm) continue;
      const int i = (n & 63) >> 5;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r == rd && arow[n] >= 0) a.s_true[q0 + n] = (i == 0) ? acc[0][j][r] : acc[1][j][r];
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TQ; ++j) {
    const int n = wq0 + j * 32 + li;
    const int64_t q = arow[n];
    const float st = sts[n], dlt = sdl[n];
    const uint32_t ex[2] = {exw[j][0], exw[j][1]};
    // branch-free count; the rare near-ties collect in a bit mask and are
    // listed in one loop afterwards (a branch per candidate cost more than
    // the count itself).  An excluded candidate's score becomes −∞ first:
    // then "counted" is d > δ and "near" is |d| ≤ δ (−δ ≤ d ≤ δ; false for −∞
    // and NaN), the same sets as ok ∧ d > δ and ok ∧ ¬(d > δ) ∧ d ≥ −δ with
    // fewer live compare masks
    int g = 0;
    uint32_t near = 0;  // bit 16·i + r
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mloc = (r & 3) + 8 * (r >> 2) + 4 * kh;
        const float sc = ((ex[i] >> mloc) & 1u) ? -__builtin_inff() : acc[i][j][r];
        const float diff = sc - st;
        g += (diff > dlt) ? 1 : 0;
        near |= (__builtin_fabsf(diff) <= dlt) ? (1u << (16 * i + r)) : 0u;
      }
    if (__builtin_amdgcn_ballot_w64(near != 0u)) {
      while (near) {
        const int b = __builtin_ctz(near);
        near &= near - 1u;
        const int i = b >> 4, r = b & 15;
        const int mloc = (r & 3) + 8 * (r >> 2) + 4 * kh;
        const int idx = atomicAdd(&a.win.ucnt[q], 1);
        if (idx < a.win.cap) a.win.ulist[q * (int64_t)a.win.cap + idx] = (int32_t)(e0 + wm * 64 + i * 32 + mloc);
      }
    }
    g += __shfl_xor(g, 32);
    if (kh == 0 && q >= 0 && g) atomicAdd(&cgt[n], g);
  }
  __syncthreads();
  if (t < X::BQ && arow[t] >= 0 && cgt[t]) atomicAdd(&a.gt[q0 + t], cgt[t]);
}

}  // namespace

int launch_filter_bits(const int64_t* filt_off, const int64_t* filt_ids, const int64_t* true_id, int64_t nq,
                       int64_t E, uint32_t* bits, int32_t* err, hipStream_t s) {
  const int64_t W = (E + 31) / 32;
  if (nq > 65535) return -1;
  if (W <= FB_LDS_WORDS) {
    hipLaunchKernelGGL(k_filter_bits_lds, dim3((unsigned)nq), dim3(256), (size_t)W * 4, s, nullptr, 0, nullptr,
                       filt_off, filt_ids, true_id, nq, E, (int64_t)0, (int)W, bits, err, nullptr, nullptr, nullptr);
    return (int)hipGetLastError();
  }
  hipError_t he = hipMemsetAsync(bits, 0, (size_t)nq * W * 4, s);
  if (he != hipSuccess) return (int)he;
  hipLaunchKernelGGL(k_filter_bits, dim3(4, (unsigned)nq), dim3(256), 0, s, filt_off, filt_ids, true_id, nq, E, W,
                     bits, err);
  return (int)hipGetLastError();
}

int launch_filter_bits_tab(const int64_t* queries, int head, const int64_t* tab, const int64_t* vals,
                           const int64_t* true_id, int64_t nq, int64_t E, int64_t R, uint32_t* bits, int32_t* err,
                           hipStream_t s) {
  const int64_t W = (E + 31) / 32;
  if (W <= FB_LDS_WORDS && nq <= 0x7fffffff) {
    hipLaunchKernelGGL(k_filter_bits_lds, dim3((unsigned)nq), dim3(256), (size_t)W * 4, s, queries, head, tab,
                       nullptr, vals, true_id, nq, E, R, (int)W, bits, err, nullptr, nullptr, nullptr);
    return (int)hipGetLastError();
  }
  hipError_t he = hipMemsetAsync(bits, 0, (size_t)nq * W * 4, s);
  if (he != hipSuccess) return (int)he;
  hipLaunchKernelGGL(k_filter_bits_tab, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, s, queries, head, tab, vals,
                     true_id, nq, E, R, W, bits, err);
  return (int)hipGetLastError();
}

int launch_filter_bits_both(const int64_t* queries, int tab, const int64_t* off_h, const int64_t* ids_h,
                            const int64_t* off_t, const int64_t* ids_t, const int64_t* true_id, int64_t nq,
                            int64_t E, int64_t R, uint32_t* bits, int32_t* err, hipStream_t s) {
  const int64_t W = (E + 31) / 32;
  if (W > FB_LDS_WORDS || 2 * nq > 0x7fffffff) return -1;  // (the caller runs a launch per direction)
  if (tab)
    hipLaunchKernelGGL(k_filter_bits_lds, dim3((unsigned)(2 * nq)), dim3(256), (size_t)W * 4, s, queries, 1, off_h,
                       nullptr, ids_h, true_id, nq, E, R, (int)W, bits, err, off_t, nullptr, ids_t);
  else
    hipLaunchKernelGGL(k_filter_bits_lds, dim3((unsigned)(2 * nq)), dim3(256), (size_t)W * 4, s, queries, 0,
                       nullptr, off_h, ids_h, true_id, nq, E, R, (int)W, bits, err, nullptr, off_t, ids_t);
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
  // k_rank_mfma is __launch_bounds__(256, 4): ≤ 128 VGPRs (96 used) and 36 KB
  // of LDS, 4 workgroups = 4 waves per SIMD (the LDS-DMA double buffer holds no
  // staging registers); buffer offsets are 32-bit: both operands below 4 GB
  if ((uint64_t)E * K * 4 >= 0xFFFFFF00ull || (uint64_t)nq * K * 4 >= 0xFFFFFF00ull) return -1;
  if (gather) {
    hipLaunchKernelGGL((k_rank_mfma<true>), dim3(1, gy), dim3(256), 0, s, a);
  } else {
    const dim3 gs((unsigned)((E + BN - 1) / BN), gy);
    hipLaunchKernelGGL((k_rank_mfma<false>), gs, dim3(256), 0, s, a);
  }
  return (int)hipGetLastError();
}

// split-bf16 tile: buffer sizes and launchers (path "mfma")
int64_t xsplit_nslab(int K) { return (K + XS_BK - 1) / XS_BK; }
int64_t xsplit_elems(int64_t rows, int K) { return ((rows + 127) / 128) * 128 * xsplit_nslab(K) * XS_BK * 2; }

int launch_split_bf16(const float* src, int64_t rows, int K, uint16_t* dst, hipStream_t s, const int64_t* skip) {
  const int64_t nrb = (rows + 127) / 128, nslab = xsplit_nslab(K);
  const int64_t waves = nrb * 16 * ((nslab * XS_BK + 63) / 64);  // 8 rows × 64 k each
  hipLaunchKernelGGL(k_split_bf16, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, src, rows, K, (int)nslab,
                     nrb, dst, skip);
  return (int)hipGetLastError();
}

// pRotatE's phase table for the register tile (k_rank_tile<PROTATE>): per
// element the (cos, sin) pair of the candidate phase x / kappa (entity rows,
// ent = 1; the true division the tile used to evaluate per block,
// model.py:245-246) or the (sin, cos) pair of the query's phase sum x (q rows,
// ent = 0), as [row][K][2] floats.  sincosf here is the same library call the
// tile's staging made, so the tile's products — and ranks — are unchanged; the
// tile no longer evaluates 8 sincos per thread and slab for every (query tile,
// candidate tile) pair (wn18rr: 640 times per element).  One thread per 4
// elements; K % 4 == 0 (the tile's own condition).
__global__ __launch_bounds__(256) void k_prot_phase(const float* __restrict__ src, int64_t rows, int K, float kappa,
                                                    int ent, float* __restrict__ dst, const int64_t* skip) {
  if (skip && *skip) return;  // the workspace already holds this table's phases (k_rank_tag)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t kq = K / 4;
  if (i >= rows * kq) return;
  const int64_t row = i / kq;
  const int k = (int)(i - row * kq) * 4;
  const float4 x = *reinterpret_cast<const float4*>(src + row * K + k);
  const float v[4] = {x.x, x.y, x.z, x.w};
  float o[8];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    float sv, cv;
    sincosf(ent ? v[u] / kappa : v[u], &sv, &cv);
    o[2 * u] = ent ? cv : sv;
    o[2 * u + 1] = ent ? sv : cv;
  }
  float4* d = reinterpret_cast<float4*>(dst + (row * K + k) * 2);
  d[0] = make_float4(o[0], o[1], o[2], o[3]);
  d[1] = make_float4(o[4], o[5], o[6], o[7]);
}

int launch_prot_phase(const float* src, int64_t rows, int K, float kappa, int ent, float* dst, hipStream_t s,
                      const int64_t* skip) {
  if (K % 4 != 0 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return -1;
  const int64_t n = rows * (K / 4);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_prot_phase, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, rows, K, kappa, ent, dst,
                     skip);
  return (int)hipGetLastError();
}

// kge_selftest_sin: the largest distance, in floats, between the device sinf
// and the correctly rounded sin over every float x with |x| ≤ range — against
// both of sin_rn2's candidates where it cannot tell which one that is
__global__ __launch_bounds__(256) void k_selftest_sin(uint32_t lim, int32_t* maxd) {
  const uint64_t n = (uint64_t)lim * 2;
  int32_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint32_t bits = (uint32_t)(i >> 1) | ((i & 1) ? 0x80000000u : 0u);
    const float x = __int_as_float((int32_t)bits);
    float alt;
    const float r = sin_rn2(x, &alt);
    const int32_t f = float_ord(sin_fast(x));
    const int32_t d = f - float_ord(r), da = f - float_ord(alt);
    m = max(m, max(d < 0 ? -d : d, da < 0 ? -da : da));
  }
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0 && m > 0) atomicMax(maxd, m);
}

int launch_selftest_sin(float range, int32_t* maxd, hipStream_t s) {
  if (!(range >= 0.f) || range > 3.0e38f) return -1;
  const uint32_t lim = (uint32_t)__builtin_bit_cast(int32_t, range) + 1u;  // bit patterns of [0, range]
  hipLaunchKernelGGL(k_selftest_sin, dim3(8192), dim3(256), 0, s, lim, maxd);
  return (int)hipGetLastError();
}

int launch_rank_mfma_x(int gather, const uint16_t* qs, const uint16_t* es, int64_t nq, int64_t E, int K,
                       const int64_t* true_id, float* s_true, const uint32_t* bits, int32_t* gt, const RankWin& win,
                       hipStream_t s) {
  XArgs a;
  a.qs = qs; a.es = es; a.nq = nq; a.E = E; a.nslab = (int)xsplit_nslab(K);
  const uint64_t qb = (uint64_t)xsplit_elems(nq, K) * 2u, eb = (uint64_t)xsplit_elems(E, K) * 2u;
  if (qb >= XS_OOB || eb >= XS_OOB) return -1;  // 32-bit buffer offsets, XS_OOB reads zeros
  a.qs_bytes = (uint32_t)qb; a.es_bytes = (uint32_t)eb;
  a.true_id = true_id; a.s_true = s_true; a.fbits = bits; a.W = (E + 31) / 32; a.gt = gt; a.win = win;
  const unsigned gy = (unsigned)((nq + XTile::BQ - 1) / XTile::BQ);
  a.gx = (int)((E + XTile::BNX - 1) / XTile::BNX);
  a.gy = (int)gy;
  // candidate tiles per L2 group: ≤ 2 MB of split rows (half an XCD's L2)
  const int64_t tile_bytes = (int64_t)XTile::BNX * a.nslab * XS_BK * 4;
  a.group = (int)std::max<int64_t>(1, (2 << 20) / tile_bytes);
  if (gather) {
    hipLaunchKernelGGL((k_rank_mfma_x<true>), dim3(1, gy), dim3(256), 0, s, a);
    return (int)hipGetLastError();
  }
  const int64_t per_xcd = (int64_t)((a.gx + 7) / 8) * a.gy;  // XCD 0 has the most candidate tiles
  hipLaunchKernelGGL((k_rank_mfma_x<false>), dim3((unsigned)(8 * per_xcd)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// Entity-table statistics for the ranking windows (TS_NSTAT maxima over the
// rows): stats[0] = max row L2 norm ‖e‖, stats[1] = max |x|, stats[2] = max
// ‖r_e‖ and stats[3] = max ‖lo_e‖ of the rows' bf16 splits (e = hi + lo + r;
// the split tile's error bound, k_rank_window).  Each wave takes TS_ROWS rows at a time with their
// loads interleaved (TS_ROWS float4s in flight per lane; one row per wave at a
// time left the pass latency-bound: 0.24 ms for wn18rr's 40,943 × 500 table,
// r02), rows strided over a bounded grid; each block writes its partial
// maxima to stats[4 + 4·block] and one small block reduces them (the
// per-block atomics on the same two words serialised at ≈11 ns each: 23 µs of
// the 35 µs pass; per row, 0.93 ms).  stats needs TS_NSTAT·(1 + TS_BLOCKS) floats.
constexpr int TS_ROWS = 4;
__global__ __launch_bounds__(256) void k_table_stats(const float* __restrict__ ent, int64_t E, int Le,
                                                     float* stats, const int64_t* skip) {
  if (skip && *skip) return;  // still valid in the workspace (k_rank_tag)
  __shared__ float red[TS_NSTAT][4];
  const int lane = threadIdx.x & 63, w = wave_id();
  const bool vec4 = (Le & 3) == 0 && (((uintptr_t)ent) & 15) == 0;
  const int nk = vec4 ? Le / 4 : Le;
  float bs[TS_NSTAT] = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)gridDim.x * 4 * TS_ROWS;
  for (int64_t e0 = ((int64_t)blockIdx.x * 4 + w) * TS_ROWS; e0 < E; e0 += stride) {
    float s2[TS_ROWS], mx[TS_ROWS], sl[TS_ROWS], sr[TS_ROWS];
#pragma unroll
    for (int r = 0; r < TS_ROWS; ++r) s2[r] = mx[r] = sl[r] = sr[r] = 0.f;
    auto acc = [&](int r, float v) {
      float l8, r16;
      bf16_split_scaled(v, l8, r16);
      s2[r] += v * v;
      sl[r] += l8 * l8;
      sr[r] += r16 * r16;
      mx[r] = fmaxf(mx[r], fabsf(v));
    };
    for (int k = lane; k < nk; k += 64) {
#pragma unroll
      for (int r = 0; r < TS_ROWS; ++r) {
        if (e0 + r >= E) continue;
        const float* row = ent + (e0 + r) * Le;
        if (vec4) {
          const float4 v = reinterpret_cast<const float4*>(row)[k];
          acc(r, v.x); acc(r, v.y); acc(r, v.z); acc(r, v.w);
        } else {
          acc(r, row[k]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < TS_ROWS; ++r) {
      float m = mx[r];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      table_stats_row(bs, wave_sum(s2[r]), m, wave_sum(sl[r]), wave_sum(sr[r]), 1.0001f + (float)Le * 3.1e-8f);
    }
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < TS_NSTAT; ++i) red[i][w] = bs[i];
  __syncthreads();
  if (threadIdx.x < TS_NSTAT) {
    const int i = threadIdx.x;
    stats[TS_NSTAT + TS_NSTAT * blockIdx.x + i] = fmaxf(fmaxf(red[i][0], red[i][1]), fmaxf(red[i][2], red[i][3]));
  }
}

__global__ __launch_bounds__(256) void k_stats_reduce(float* stats, int nblocks, const int64_t* skip) {
  if (skip && *skip) return;
  __shared__ float red[TS_NSTAT][4];
  const int lane = threadIdx.x & 63, w = wave_id();
  float v[TS_NSTAT] = {0.f, 0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < nblocks; b += 256)
#pragma unroll
    for (int i = 0; i < TS_NSTAT; ++i) v[i] = fmaxf(v[i], stats[TS_NSTAT + TS_NSTAT * b + i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < TS_NSTAT; ++i) v[i] = fmaxf(v[i], __shfl_xor(v[i], o));
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < TS_NSTAT; ++i) red[i][w] = v[i];
  __syncthreads();
  if (threadIdx.x < TS_NSTAT) {
    const int i = threadIdx.x;
    stats[i] = fmaxf(fmaxf(red[i][0], red[i][1]), fmaxf(red[i][2], red[i][3]));
  }
}

int launch_split_stats(const float* ent, int64_t E, int K, uint16_t* dst, float* stats, hipStream_t s,
                       const int64_t* skip_stats, const int64_t* skip_split) {
  const int64_t nrb = (E + 127) / 128, nslab = xsplit_nslab(K);
  const int64_t want = (nrb * 16 + 3) / 4;  // a wave per 8-row group
  const int blocks = (int)(want < TS_BLOCKS ? (want > 0 ? want : 1) : TS_BLOCKS);
  hipLaunchKernelGGL(k_split_stats, dim3((unsigned)blocks), dim3(256), 0, s, ent, E, K, (int)nslab, nrb, dst, stats,
                     skip_stats, skip_split);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(256), 0, s, stats, blocks, skip_stats);
  return (int)hipGetLastError();
}

int launch_table_stats(const float* ent, int64_t E, int Le, float* stats, hipStream_t s, const int64_t* skip) {
  const int64_t want = (E + 4 * TS_ROWS - 1) / (4 * TS_ROWS);
  const int blocks = (int)(want < TS_BLOCKS ? (want > 0 ? want : 1) : TS_BLOCKS);
  hipLaunchKernelGGL(k_table_stats, dim3((unsigned)blocks), dim3(256), 0, s, ent, E, Le, stats, skip);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(256), 0, s, stats, blocks, skip);
  return (int)hipGetLastError();
}

// The ranking workspace's table tag (KGE_RANK_REUSE_TABLE): tag = [entity
// pointer, nentity, entity_dim, statistics valid, derived-table valid, skip
// statistics, skip derived table, derived-table kind], [8..10] pRotatE's list
// tag, [11] the derived table's parameter.  The derived table is the split-bf16
// operands (kind 1) or pRotatE's phase table (kind 2, parameter = the phase
// divisor's bits).  With reuse requested, the statistics / derived table a
// previous call left are reused only if that call ranked the same table
// pointer and shape and actually wrote them, of the same kind and parameter
// (a scan-path call writes none; a DistMult call after a RotatE one finds no
// statistics; a pRotatE call after a DistMult one on the same tensor finds a
// split, not phases); the tag then describes what this call leaves behind.
// One thread, stream-ordered before the kernels that read the skip words.
__global__ void k_rank_tag(int64_t* tag, const float* ent, int64_t E, int Le, int reuse, int need_stats,
                           int split_kind, int64_t split_param) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool match = reuse && tag[0] == (int64_t)(uintptr_t)ent && tag[1] == E && tag[2] == Le;
  const int64_t sv = match ? tag[3] : 0;
  const int64_t xv = (match && tag[7] == split_kind && tag[11] == split_param) ? tag[4] : 0;
  tag[5] = (need_stats && sv) ? 1 : 0;
  tag[6] = (split_kind && xv) ? 1 : 0;
  tag[0] = (int64_t)(uintptr_t)ent;
  tag[1] = E;
  tag[2] = Le;
  tag[3] = need_stats ? 1 : sv;
  if (split_kind) {
    tag[4] = 1;
    tag[7] = split_kind;
    tag[11] = split_param;
  } else if (!match) {
    tag[4] = 0;
  }
  tag[8] = tag[9] = tag[10] = 0;  // any ranking call voids pRotatE's list tag (its list stage rewrites it)
}

int launch_rank_tag(int64_t* tag, const float* ent, int64_t E, int Le, int reuse, int need_stats, int split_kind,
                    int64_t split_param, hipStream_t s) {
  hipLaunchKernelGGL(k_rank_tag, dim3(1), dim3(64), 0, s, tag, ent, E, Le, reuse, need_stats, split_kind,
                     split_param);
  return (int)hipGetLastError();
}

}  // namespace kge
