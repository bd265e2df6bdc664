// kge_internal.h — argument blocks shared by the host dispatcher and the kernels.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "../../include/kge_hip.h"
#include "kge_device.h"

namespace kge {

enum RowOp : int { ROW_TRAIN = 0, ROW_GIVEN = 1 };

// Query shipping (kge_ship_step): this rank holds only the entity rows
// [own_lo, own_hi) of the table; the row kernels see the GLOBAL batch and
// the shipped q vectors, and touch only owned rows (the table pointer is the
// shard's base minus own_lo rows, so rows keep their global ids).
struct ShipArgs {
  int64_t own_lo, own_hi;
  int world, me;
  const float* q_in;      // [B, Le] q of every row (summed over the shards)
  const float* qp_in;     // [B, Le] head-batch: the positive's tail-form q (h∘r)
  float* qp_out;          // k_ship_q, head-batch
  float* part_out;        // [B, 4] this shard's (max T·s, Z, NL, MG) per row
  const float* parts_in;  // [world, B, 4] every shard's
  float* s_out;           // [B, n] raw scores of the owned negatives
  float* pq;              // [B, Le] head-batch: dL/d(h∘r) of the positive
  float* pstats;          // [B, 4] positive statistics (owner of t; zero elsewhere)
};

struct ScoreArgs {
  const float* ent;
  const float* rel;
  const float* modulus;
  const int64_t* pos;
  const int64_t* neg;
  int64_t neg_stride;  // neg index of (i, j) = neg[i * neg_stride + j]
  int64_t B, n, E, R;
  int Le, Lr;
  RowGeom eg;
  Consts c;
  int64_t jpw;  // candidates per wave work-unit
  float* out;
  int32_t* err;
};

struct RowArgs {
  const float* ent;
  const float* rel;
  const float* modulus;
  const int64_t* pos;
  const int64_t* neg;
  int64_t neg_stride;
  int64_t B, n, E, R;
  int Le, Lr;
  RowGeom eg;
  Consts c;
  int op;           // RowOp
  int adversarial;  // args.negative_adversarial_sampling
  float adv_T;      // args.adversarial_temperature
  int uni_weight;   // args.uni_weight
  float uni_inv;    // 1 / global batch (uni_weight)
  const float* sub_w;
  const float* w_sum;
  float* wsum_out;    // non-null: k_build_q's block 0 writes Σ sub_w here (= w_sum)
  const float* g_in;  // ROW_GIVEN: dL/dscore [B, n]
  float* g_out;       // ROW_TRAIN: dL/ds_ij [B, n]
  float* q_out;       // [B, Le]
  float* dq_out;      // [B, Le]  dL/dq of the negatives (k_row → k_row_epi)
  float* ent_contrib; // [2B, Le]  slot 0 = head row, slot 1 = tail row
  float* rel_contrib; // [B, Lr]
  float* row_stats;   // [B, 4]  logσ(s_pos), neg term, d/dmodulus, s_pos
  int n_lds;          // floats reserved for raw scores in LDS (TRAIN: n)
  int fuse_epi;       // 1: k_row runs the epilogue in its tail, no k_row_epi launch
  int32_t* err;
  void (*timer_mid)(hipStream_t);  // stage-timer hook between the row-pass launches (or null)
  ShipArgs sh;        // query shipping stages only
  float* q_sl;        // non-null (VEC = 4): q also slice-major for k_entity_sl, [slice][row][re 64 | im 64 slots]
  int q_sl_w;         //   slots per slice
};

// k_row's LDS merge buffer: [2][Le] floats, and at least the 256 floats the
// fused Σw reduction (block_weight_sum) uses as its tree
__host__ __device__ inline int vb_floats(int Le) { return 2 * Le > 256 ? 2 * Le : 256; }

// Rows wider than the register-tiled kernels hold (kge_wide.inc, check_model's
// ns = 0): the entity pass cuts each row into WIDE_PARTS column parts (its
// reg_partial slots per entity), and k_row_w keeps one float per negative in LDS
constexpr int WIDE_PARTS = 8;
inline size_t wide_row_lds(int64_t n) { return sizeof(float) * (size_t)(n > 0 ? n : 1); }

struct RelArgs {
  const float* rel;
  int64_t R, E, B, Bn;
  int Lr;
  const int32_t* off;
  const int32_t* occ;
  const float* rel_contrib;  // [B, Lr]
  float reg3;
  float* reg_partial;        // [R]
  float* grad_rel;
  int write_grad;            // store grad_rel (always, unless the optimizer is fused and asks not to)
  AdamT adam;                // fused optimizer step (adam.p == null: none)
  AdamK adamk;
};

// Loss finalisation (k_finalize, or the entity launch's last block: EntArgs.fin)
struct FinArgs {
  const float* row_stats;    // [B, 4]
  const float* sub_w;        // nullable
  const float* w_sum;        // nullable → Σ of sub_w
  int64_t B;
  int uni_weight;
  float uni_n;               // global batch size (uni_weight means)
  const float* reg_partial;  // or null; summed over [reg_a0, reg_a1) then [reg_b0, reg_b1)
  int64_t reg_a0, reg_a1, reg_b0, reg_b1;  // (entity parts, relation rows; a sub-range for an owner's step)
  float regularization;
  float* losses;             // [4]
  float* grad_modulus;       // nullable
  const int32_t* err;        // device error flag, copied to losses[4]
  AdamT adam;                // fused optimizer step of the pRotatE modulus (adam.p == null: none)
  AdamK adamk;
};

struct EntArgs {
  const float* ent;
  const float* modulus;
  int64_t E;
  int64_t e_begin, e_end;  // entity rows this launch covers (a chunk of [0, E))
  int Le;
  RowGeom eg;
  Consts c;
  const int32_t* off;   // CSR offsets (entity buckets first)
  const int32_t* occ;   // occurrence ids, ascending inside each bucket
  int64_t Bn;           // ids < Bn: negative (i, j) = (id / n, id % n)
  int64_t n;
  const float* g;       // [B, n]
  const float* q;       // [B, Le]
  const float* ent_contrib;  // ids >= Bn index [2B, Le]
  float reg3;           // 3 * regularization (0 = off)
  float* reg_partial;   // [E] Σ|x|^3 per row (when reg3 != 0)
  float* grad_ent;
  int write_grad;       // store grad_ent (unless the fused optimizer asks not to)
  int64_t B;            // batch rows (the q buffer's height)
  int nsl;              // > 0: column-sliced pass k_entity_sl with nsl slices of slice_w slots (VEC = 4)
  int slice_w;
  int align_sl;         // k_entity_sl: line-aligned 64-slot slices per row (entity_slice_align)
  const float* q_sl;    // k_entity_sl<.., QSL>: q slice-major (written by k_row; even slices only) or null
  AdamT adam;           // fused optimizer step (adam.p == null: none)
  AdamK adamk;
  RelArgs rel;          // rel_blocks > 0: trailing blocks of k_entity_sl run the relation pass
  int64_t rel_blocks;
  FinArgs fin;          // fin_fused: the launch's last block runs the loss finalisation
  int fin_fused;        // (only when nothing it reads is written by this launch)
};

// k_entity_sl's leading blocks: the fused finalisation and the relation rows,
// rounded up to a multiple of 8 (the XCD count) when there are any
__host__ __device__ inline unsigned ent_lead_blocks(const EntArgs& a) {
  const unsigned l = (unsigned)a.rel_blocks + (a.fin_fused ? 1u : 0u);
  return (l + 7u) & ~7u;
}

// Near-tie window of the fast ranking passes (all three): a candidate whose
// fast fp32 score lies within delta[q] of the query's fast true score is not
// counted but listed for the reference-order refinement (kge_rank_ref.h).
// a diagnostic switch read per launch: true when the variable is set to "0"
inline bool env_flag_off(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '0' && e[1] == 0;
}

struct RankWin {
  const float* delta;  // [nq]
  int32_t* ucnt;       // [nq]  listed candidates (may exceed cap: overflow)
  int32_t* ulist;      // [nq, cap]
  int cap;
};

__device__ __forceinline__ void win_count(const RankWin& w, int64_t q, int64_t e, float s, float st, float dlt,
                                          int& g) {
  const float diff = s - st;
  if (diff > dlt) {
    ++g;
  } else if (diff >= -dlt) {
    const int idx = atomicAdd(&w.ucnt[q], 1);
    if (idx < w.cap) w.ulist[q * (int64_t)w.cap + idx] = (int32_t)e;
  }
}

struct RankArgs {
  const float* ent;
  const float* rel;
  const float* modulus;
  const int64_t* queries;
  int64_t nq, E, R;
  int Le, Lr;
  RowGeom eg;
  Consts c;
  const int64_t* filt_off;
  const int64_t* filt_ids;
  int64_t cpw;          // candidates per wave work-unit
  float* q;             // [nq, Le]
  float* s_true;        // [nq]
  int64_t* true_id;     // [nq]
  int32_t* gt;          // [nq]
  const uint32_t* fbits;  // [nq, W] excluded candidates (filtered ids + the true id)
  int64_t W;
  RankWin win;
  int32_t* err;
  int prep_only;        // launch k_rank_prep only (the MFMA / tile paths count on their own)
  int zero_counts;      // k_rank_prep zeroes gt and the five counters after it (eq, gtx, eqx, ucnt, done)
  int both_dirs;        // (prep_only) both directions in one launch: queries [nq, 3] shared, per-query
                        // arrays of 2·nq (head-batch's first); not for wide rows
  int64_t cstride;      // distance between those counter arrays (the workspace's query count: nq, or 2·nq
                        // when both directions share one workspace and gt points into it)
  const float* trig;    // RotatE: [R, 2, Lr] reference cos | sin of the phases, or null
};

// Reference-order refinement (k_rank_window / k_rank_refine / k_rank_exact).
struct RefArgs {
  const float* ent;
  const float* rel;
  const float* modulus;
  const int64_t* queries;
  int64_t nq, E, R;
  int Le, Lr, K;           // K = reduction length (complex: Le / 2)
  Consts c;
  const float* q;          // [nq, Le] fast-path q (k_rank_prep)
  float* qref;             // [nq, Le] reference-order q
  const int64_t* true_id;  // [nq]
  const float* s_true;     // [nq] fast-path true score
  float* sref_true;        // [nq] reference-order true score
  float* s_true_w;         // [nq] k_rank_true_ref writes s_true here (the split-bf16 path's true score)
  int true_exact;          // s_true is the reference-order score (k_rank_true_ref): δ covers the candidate only
  float* delta;            // [nq] window
  const float* stats;      // [2] max row L2 norm, max |x| of the entity table
  int exact_fast;          // the fast pass is already in reference order (TransE on the register tile)
  const int32_t* ucnt;
  const int32_t* ulist;
  int cap;
  const uint32_t* fbits;
  int64_t W;
  int32_t* gt;             // += refined strictly-greater
  int32_t* eq;             // += refined ties
  int32_t* gtx;            // overflowed queries: exact counts over every candidate
  int32_t* eqx;
  int32_t* err;
  const float* trig;       // RotatE: [R, 2, Lr] reference cos | sin of the phases, or null
  float fast_u;            // > 0: the fast pass's error bound in u·‖q‖·max‖e‖ (split-bf16 tile)
  int ref_slots;           // k_rank_refine: half-waves with an LDS row slot (set by its launcher)
  int ref_global;          // k_rank_refine: q and rows read from global memory (rows too wide for LDS)
  // pRotatE with the caller's sin (kge_rank_sin_args / kge_rank_finish_sin):
  // query q's items [item_off[q], item_off[q+1]) — item 0 the true entity, then
  // the listed candidates (or, for an overflowed window, entity ids 0..E-1) —
  // each K phase sums (args) or their sin as the caller's library evaluates it
  const int64_t* item_off; // [nq + 1] or null
  const float* sins;       // [item_off[nq], K] or null (refine / exact read it)
  float* args;             // [item_off[nq], K] (k_rank_sin_args writes it)
  int lib_sin;             // window: the reference sin is a library's (≤ 1 ulp), not correctly rounded
  int screen;              // k_rank_refine (pRotatE list stage): each listed candidate's score interval
                           // under any library sin within 1 ulp (ref_score_half_prot_bounds); those
                           // whose interval clears the true one's are decided on the device, only the
                           // others stay in the list for the library sin
  int decide;              // (screen) 0: decide nothing, keep every listed candidate (diagnostic)
  int32_t* ucnt_w;         // (screen) the list, rewritten in place
  int32_t* ulist_w;
  float* sref_hi;          // [nq] (screen) the true score interval's upper end (sref_true: its lower)
  int32_t* done;           // [nq] finish stage: the query's items were delivered (a second delivery is an error)
  const int64_t* ltag;     // sin_args / finish: the list tag the list stage wrote, expected = ltag_v
  int64_t ltag_v[3];
};

// Register-tiled filtered ranking (kge_kernels.inc, k_rank_tile): 64 queries ×
// 64 candidates per workgroup, the dim-2 reduction done as one sequential sum
// per (query, candidate) pair.  The gather pass (B columns = the queries' true
// rows) writes s_true with the same instruction sequence the scan pass uses.
struct TileArgs {
  const float* q;          // [nq, Le]  from k_rank_prep ([re | im] for complex rows)
  const float* ent;        // [E, Le]
  const float* modulus;    // pRotatE
  int64_t nq, E;
  int Le, K;               // K = reduction length (complex: Le / 2)
  Consts c;
  const int64_t* true_id;  // [nq]
  float* s_true;           // [nq]  gather pass writes, scan pass reads
  const uint32_t* fbits;   // [nq, W] filtered-candidate bitmap
  int64_t W;
  int32_t* gt;             // [nq]
  RankWin win;
  const float* qph;        // pRotatE: [nq, K, 2] (sin, cos) of q's phase sums (launch_prot_phase)
  const float* eph;        // pRotatE: [E, K, 2] (cos, sin) of the candidate phases
};

struct ModelOps {
  int (*score)(int mode, int vec, int ns, const ScoreArgs&, int64_t units, hipStream_t);
  int (*row)(int mode, int vec, int ns, int stage, const RowArgs&, size_t lds, hipStream_t);
  int (*entity)(int mode, int vec, int ns, const EntArgs&, hipStream_t);
  int (*rank)(int mode, int vec, int ns, const RankArgs&, hipStream_t);
  int (*rank_tile)(int mode, int gather, const TileArgs&, hipStream_t);
  // stage 0: window (δ, reference q); 1: refine the listed candidates; 2: exact rescan of overflowed queries;
  // 3: pRotatE phase sums of every item (k_rank_sin_args)
  int (*rank_ref)(int mode, int stage, const RefArgs&, hipStream_t);
};

ModelOps model_ops_transe();
ModelOps model_ops_distmult();
ModelOps model_ops_complex();
ModelOps model_ops_rotate();
ModelOps model_ops_protate();

}  // namespace kge
