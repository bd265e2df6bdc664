// kge_internal.h — argument blocks shared by the host dispatcher and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "../../include/kge_hip.h"
#include "kge_device.h"

namespace kge {

enum RowOp : int { ROW_TRAIN = 0, ROW_GIVEN = 1 };

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
};

// k_row's LDS merge buffer: [2][Le] floats, and at least the 256 floats the
// fused Σw reduction (block_weight_sum) uses as its tree
__host__ __device__ inline int vb_floats(int Le) { return 2 * Le > 256 ? 2 * Le : 256; }

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
  AdamT adam;           // fused optimizer step (adam.p == null: none)
  AdamK adamk;
  RelArgs rel;          // rel_blocks > 0: trailing blocks of k_entity_sl run the relation pass
  int64_t rel_blocks;
};

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
  int32_t* eq;          // [nq]
  int64_t* ranks;
  int32_t* ties;
  int32_t* err;
  int prep_only;        // launch k_rank_prep only (the MFMA path counts on its own)
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
  int32_t* eq;             // [nq]
};

struct ModelOps {
  int (*score)(int mode, int vec, int ns, const ScoreArgs&, int64_t units, hipStream_t);
  int (*row)(int mode, int vec, int ns, int stage, const RowArgs&, size_t lds, hipStream_t);
  int (*entity)(int mode, int vec, int ns, const EntArgs&, hipStream_t);
  int (*rank)(int mode, int vec, int ns, const RankArgs&, hipStream_t);
  int (*rank_tile)(int mode, int gather, const TileArgs&, hipStream_t);
};

ModelOps model_ops_transe();
ModelOps model_ops_distmult();
ModelOps model_ops_complex();
ModelOps model_ops_rotate();
ModelOps model_ops_protate();

}  // namespace kge
