/*
 * kge_hip.h — C-ABI of the MI355X (gfx950) knowledge-graph-embedding hot path.
 *
 * Drop-in boundary for the scoring / self-adversarial-loss / filtered-ranking
 * path of kahrabian/KnowledgeGraphEmbedding.  The reference has no FFI: its
 * boundary is the Python methods of `KGEModel` (codes/model.py).  Each entry
 * point below names the reference interface it replaces (file:line); the
 * Python host mirror in knowledgegraphembedding_amd/ binds these through
 * ctypes (see INTEGRATION.md for the binding a reference maintainer would add).
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (hipMalloc / torch CUDA tensors),
 *     row-major and contiguous.  Embeddings are fp32, indices int64 — the
 *     reference's own dtypes (model.py:45,52; dataloader.py:63-65).
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *     Nothing here allocates, frees or synchronises: every call is
 *     graph-capturable.  Scratch comes from a caller-owned workspace whose
 *     size the matching *_workspace_bytes() query returns.
 *   - Return value: 0 on success, a KGE_ERR_* code for argument errors
 *     (checked on the host before anything is launched), or a hipError_t
 *     (offset by KGE_ERR_HIP_BASE) if a launch fails.
 *   - Index range errors (reference: index_select raises, model.py:86-146)
 *     cannot be checked on the host without a sync; kernels clamp nothing,
 *     skip the offending row, and set *err_flag (a device int32) to
 *     KGE_DEVERR_INDEX.  The host mirror reads the flag at its next sync
 *     point and raises IndexError.
 */
#ifndef KGE_HIP_H
#define KGE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Model ids: model.py:151-157 (the model_func plug-in registry). */
enum kge_model_id {
    KGE_TRANSE = 0,   /* model.py:166-173 */
    KGE_DISTMULT = 1, /* model.py:175-182 */
    KGE_COMPLEX = 2,  /* model.py:184-199 */
    KGE_ROTATE = 3,   /* model.py:201-229 */
    KGE_PROTATE = 4   /* model.py:231-249 */
};

/* Modes: model.py:83 'single', :104 'head-batch', :126 'tail-batch'. */
enum kge_mode_id { KGE_SINGLE = 0, KGE_HEAD_BATCH = 1, KGE_TAIL_BATCH = 2 };

enum kge_status {
    KGE_OK = 0,
    KGE_ERR_MODEL = 1,      /* ValueError('model %s not supported'), model.py:64,162 */
    KGE_ERR_MODE = 2,       /* ValueError('mode %s not supported'), model.py:149 */
    KGE_ERR_SHAPE = 3,      /* entity/relation dims inconsistent with the model (model.py:66-70) */
    KGE_ERR_ARG = 4,        /* null pointer / negative size */
    KGE_ERR_WORKSPACE = 5,  /* workspace smaller than *_workspace_bytes() */
    KGE_ERR_DIM = 6,        /* a size outside a kernel's range (negatives per row, queries per call, LDS) */
    KGE_ERR_ABI = 7,        /* kge_model_desc.struct_size != sizeof(kge_model_desc) of this library */
    KGE_ERR_HIP_BASE = 1000 /* + hipError_t */
};

/* Device-side error bits written to *err_flag. */
#define KGE_DEVERR_INDEX 1
#define KGE_DEVERR_SAMPLER 2 /* a row's true list left no room within max_draws draws */
#define KGE_DEVERR_ARG 4     /* kge_rank_sin_args / finish_sin: item_off or the list stage does not match */

/*
 * The parameters of one KGEModel (model.py:22-70).
 *   phase_divisor   = float(embedding_range.item() / 3.14159265358979323846)  model.py:202,209
 *   phase_divisor_p = float(embedding_range.item() / 3.14159262358979323846)  model.py:232,236-238
 *                     (the reference's pi typo is part of the contract)
 *   modulus         = device pointer to the pRotatE [1,1] modulus (model.py:59-60), else NULL
 *   relation_trig   = RotatE only, nullable: device [nrelation, 2, relation_dim] fp32 table of
 *                     (cos θ | sin θ) of every relation phase θ = relation / phase_divisor, as
 *                     the caller's reference evaluates them (model.py:209-212: the reference's
 *                     ATen CPU cos / sin).  The filtered ranking (kge_rank_filtered*) then builds
 *                     its queries' rotation from these values, so its ranks are the reference's
 *                     bit for bit; NULL = correctly rounded cos / sin on the device.  Training
 *                     and kge_score do not read it (scores are held to 1e-4, not to bits).
 *                     "The reference" is its CPU run: with --cuda its test_step evaluates
 *                     cos / sin and sum(dim=2) with ATen's GPU kernels, whose bits are not
 *                     reproduced here (parity against that configuration is unpinned).
 */
typedef struct kge_model_desc {
    int32_t model;
    int32_t entity_dim;   /* floats per entity row   (model.py:42) */
    int32_t relation_dim; /* floats per relation row (model.py:43) */
    int32_t struct_size;  /* = sizeof(kge_model_desc) as the caller compiled it (else KGE_ERR_ABI) */
    int64_t nentity;
    int64_t nrelation;
    float gamma;          /* model.py:32-35 */
    float phase_divisor;
    float phase_divisor_p;
    float reserved_f;
    const float *entity_embedding;   /* [nentity, entity_dim] */
    const float *relation_embedding; /* [nrelation, relation_dim] */
    const float *modulus;            /* [1] or NULL */
    const float *relation_trig;      /* RotatE [nrelation, 2, relation_dim] or NULL (ranking only) */
} kge_model_desc;

/* Library identity: "knowledgegraphembedding_amd <KGE_ABI_VERSION> gfx950".  The
 * version changes with every change of a struct, a signature or a call
 * protocol in this header (0.3: pRotatE's three-call item counts; 0.4:
 * kge_rank_filtered_both, the ranking timer counting directions; 0.5: the
 * one-step-ahead training CSR entry point of an earlier 0.4 build removed);
 * loaders refuse a library whose version differs from the header they bind. */
#define KGE_ABI_VERSION "0.5"
const char *kge_version(void);
const char *kge_status_string(int status);

/*
 * Scores of a batch — replaces KGEModel.forward(sample, mode) (model.py:72-164)
 * together with the score plug-ins (model.py:166-249).
 *   mode == KGE_SINGLE:      pos[batch,3] triples, neg ignored, nneg must be 1 → out[batch,1]
 *   mode == KGE_HEAD_BATCH:  sample = (tail_part=pos[batch,3], head_part=neg[batch,nneg])
 *   mode == KGE_TAIL_BATCH:  sample = (head_part=pos[batch,3], tail_part=neg[batch,nneg])
 *   out: [batch, nneg] fp32.
 */
int kge_score(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
              int64_t batch, int64_t nneg, float *out, int32_t *err_flag, void *stream);

/*
 * Gradient of sum(grad_scores * score) w.r.t. the tables — replaces the autograd
 * of KGEModel.forward (IndexSelectBackward = dense zero-fill + index_add_, then
 * the plug-in's elementwise backward).
 *   grad_entity [nentity, entity_dim], grad_relation [nrelation, relation_dim] are
 *   OVERWRITTEN densely (rows no sample touches become 0); grad_modulus [1] is
 *   overwritten when non-NULL (pRotatE).
 */
size_t kge_backward_workspace_bytes(const kge_model_desc *m, int32_t mode, int64_t batch, int64_t nneg);
int kge_score_backward(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                       int64_t batch, int64_t nneg, const float *grad_scores, float *grad_entity,
                       float *grad_relation, float *grad_modulus, void *workspace, size_t workspace_bytes,
                       int32_t *err_flag, void *stream);

/*
 * Fused negative scoring + self-adversarial logsigmoid loss + backward —
 * replaces KGEModel.train_step (model.py:252-301) from the forward calls up to
 * and including loss.backward(); the optimizer step stays separate (kge_adam_step).
 *   mode:            KGE_HEAD_BATCH or KGE_TAIL_BATCH (dataloader.py:171-177 alternates them)
 *   pos [batch,3], neg [batch,nneg], subsampling_weight [batch]
 *   weight_sum:      device scalar Σw over the GLOBAL batch (data-parallel ranks all-reduce it);
 *                    NULL = computed from subsampling_weight of this call.
 *   uni_weight:      args.uni_weight (model.py:281-286)
 *   uni_batch:       the global batch size used for the uni_weight means (0 = batch)
 *   adversarial:     args.negative_adversarial_sampling; temperature = args.adversarial_temperature
 *   regularization:  args.regularization (model.py:290-296); 0 disables
 *   losses_out [5]:  {positive_sample_loss, negative_sample_loss, loss, regularization,
 *                     error flag} (device fp32; the reference's log dict, model.py:305-310,
 *                    plus a copy of *err_flag so one read-back serves both)
 *   grad_* overwritten densely, as in kge_score_backward.
 */
size_t kge_train_workspace_bytes(const kge_model_desc *m, int64_t batch, int64_t nneg);
int kge_train_step_grads(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                         int64_t batch, int64_t nneg, const float *subsampling_weight,
                         const float *weight_sum, int32_t uni_weight, int64_t uni_batch,
                         int32_t adversarial, float adversarial_temperature, float regularization,
                         float *grad_entity, float *grad_relation, float *grad_modulus,
                         float *losses_out, void *workspace, size_t workspace_bytes,
                         int32_t *err_flag, void *stream);

/* Phases of kge_train_step_grads, for callers that overlap the entity-gradient
 * reduction with the entity pass (data parallel, distributed.py): ROWS runs
 * the q build, the fused scoring/loss row pass, the epilogue, the occurrence
 * CSR and the relation pass; ENTITY runs the entity-major pass over rows
 * [entity_begin, entity_end) only (call it once per chunk, in any order, until
 * every row is covered); FINALIZE joins the relation pass and writes the
 * losses (and the pRotatE modulus gradient).  Same stream, same workspace,
 * same arguments in every phase; ALL = one kge_train_step_grads call. */
#define KGE_PHASE_ROWS 1
#define KGE_PHASE_ENTITY 2
#define KGE_PHASE_FINALIZE 4
#define KGE_PHASE_ALL 7
int kge_train_step_grads_phased(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                                int64_t batch, int64_t nneg, const float *subsampling_weight,
                                const float *weight_sum, int32_t uni_weight, int64_t uni_batch,
                                int32_t adversarial, float adversarial_temperature, float regularization,
                                float *grad_entity, float *grad_relation, float *grad_modulus, float *losses_out,
                                void *workspace, size_t workspace_bytes, int32_t *err_flag, void *stream,
                                int32_t phases, int64_t entity_begin, int64_t entity_end);

/*
 * kge_train_step_grads + the optimizer step, fused — replaces model.py:268-303
 * (forward, loss, loss.backward() AND optimizer.step()) for a torch.optim.Adam
 * optimizer (run.py:266-269).  The dense Adam update of every entity /
 * relation row (zero-gradient rows included, as torch's dense Adam does) is
 * applied in the gradient passes while each gradient row is in registers, so
 * gradients are never re-read from HBM.  The parameter pointers must be the
 * model's own tables (m->entity_embedding etc.; they are updated in place).
 * Per-tensor step_size = lr / (1 - beta1^t) and bias_correction2_sqrt =
 * sqrt(1 - beta2^t), computed in double by the caller (torch's formula).
 * write_grad != 0 also stores the dense gradients into grad_* (as
 * loss.backward() leaves them in .grad); 0 skips those writes.
 */
typedef struct kge_adam_tensor {
    float *param;
    float *exp_avg;
    float *exp_avg_sq;
    float step_size;
    float bias_correction2_sqrt;
} kge_adam_tensor;

typedef struct kge_adam_desc {
    kge_adam_tensor entity;
    kge_adam_tensor relation;
    kge_adam_tensor modulus; /* pRotatE only (param NULL otherwise) */
    float beta1, beta2, eps;
    int32_t write_grad;
} kge_adam_desc;

int kge_train_step(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                   int64_t batch, int64_t nneg, const float *subsampling_weight, const float *weight_sum,
                   int32_t uni_weight, int64_t uni_batch, int32_t adversarial, float adversarial_temperature,
                   float regularization, const kge_adam_desc *adam, float *grad_entity, float *grad_relation,
                   float *grad_modulus, float *losses_out, void *workspace, size_t workspace_bytes,
                   int32_t *err_flag, void *stream);

/*
 * Data-parallel FACTOR EXCHANGE (distributed.py, exchange "factors"): instead
 * of all-reducing the dense [E, entity_dim] gradient, the ranks all-gather the
 * row pass's per-row factors — dL/ds [B, nneg], dL/dq [B, entity_dim] and the
 * row statistics [B, 4] — and every rank runs the rest of the step for the
 * GLOBAL batch itself.  On point-to-point xGMI with few ranks this moves
 * ~9 MB per rank instead of ~2·(N-1)/N · 120 MB (RotatE FB15k).
 *
 * kge_train_rows_slice: the negative-row pass (q build + k_row, no epilogue)
 * for `nrows` rows; pos/neg/subsampling_weight point at the slice's own rows,
 * weight_sum at the GLOBAL Σw (kge_weight_sum over all weights: the same
 * fixed order as a single process's in-kernel sum), uni_batch = global batch.
 * Writes g_out [nrows, nneg], dq_out [nrows, entity_dim] and columns 1-2 of
 * stats_out [nrows, 4] (pass the slice's place in the gathered buffers).
 * Workspace: kge_train_workspace_bytes(m, nrows, nneg).
 *
 * kge_train_step_from_rows: the rest of a kge_train_step (adam != NULL) or
 * kge_train_step_grads (adam == NULL) for the global batch from the gathered
 * buffers: q rebuilt, positive scores and chain rule, occurrence CSR, entity-
 * major and relation passes, losses.  Bit-identical to the single-process call
 * on the whole batch.  Workspace: kge_train_workspace_bytes(m, batch, nneg).
 */
int kge_train_rows_slice(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                         int64_t nrows, int64_t nneg, const float *subsampling_weight, const float *weight_sum,
                         int32_t uni_weight, int64_t uni_batch, int32_t adversarial, float adversarial_temperature,
                         float *g_out, float *dq_out, float *stats_out, void *workspace, size_t workspace_bytes,
                         int32_t *err_flag, void *stream);
int kge_train_step_from_rows(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                             int64_t batch, int64_t nneg, const float *subsampling_weight, const float *weight_sum,
                             int32_t uni_weight, int64_t uni_batch, float regularization, const float *g_in,
                             const float *dq_in, float *stats_inout, const kge_adam_desc *adam,
                             float *grad_entity, float *grad_relation, float *grad_modulus, float *losses_out,
                             void *workspace, size_t workspace_bytes, int32_t *err_flag, void *stream);

/*
 * The same split with the occurrence CSR built ahead: kge_train_csr builds
 * the CSR of the (gathered) batch into the workspace on `stream` — it needs
 * only the ids, so a rank runs it while the factors are still on the wire —
 * and kge_train_step_from_rows_csr is kge_train_step_from_rows reading that
 * CSR instead of building it (same workspace, same batch).  Bit-identical.
 */
int kge_train_csr(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg, int64_t batch,
                  int64_t nneg, void *workspace, size_t workspace_bytes, int32_t *err_flag, void *stream);

/*
 * kge_train_csr for an owner of the entity rows [entity_begin, entity_end):
 * only those entities' buckets are filled (the others stay empty; the
 * relation buckets are all built) — what kge_train_step_from_rows_phased /
 * _range with csr_ready read for that range, at 1/N of the fill and ordering
 * work of the whole batch's CSR.
 */
int kge_train_csr_range(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                        int64_t batch, int64_t nneg, int64_t entity_begin, int64_t entity_end, void *workspace,
                        size_t workspace_bytes, int32_t *err_flag, void *stream);
int kge_train_step_from_rows_csr(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                                 int64_t batch, int64_t nneg, const float *subsampling_weight,
                                 const float *weight_sum, int32_t uni_weight, int64_t uni_batch,
                                 float regularization, const float *g_in, const float *dq_in, float *stats_inout,
                                 const kge_adam_desc *adam, float *grad_entity, float *grad_relation,
                                 float *grad_modulus, float *losses_out, void *workspace, size_t workspace_bytes,
                                 int32_t *err_flag, void *stream);

/*
 * OWNER-COMPUTES step (partition.py, exchange "factors"): the rest of the step
 * from the gathered factors, with the entity-major pass — gradient, fused Adam
 * and regulariser — restricted to the caller's own rows [entity_begin,
 * entity_end) of the global batch's occurrences; the relation pass, the
 * positive epilogue and the losses cover the whole batch (identical on every
 * rank).  adam->entity.exp_avg / exp_avg_sq may point `entity_begin` rows
 * before the caller's shard-sized moment buffers (only owned rows are
 * touched).  reg_relations = 0 leaves the relation rows out of the
 * regularisation loss (another rank counts them); losses_out[3] then holds
 * this rank's part.  csr_ready: the CSR was built by kge_train_csr.
 */
int kge_train_step_from_rows_range(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                                   int64_t batch, int64_t nneg, const float *subsampling_weight,
                                   const float *weight_sum, int32_t uni_weight, int64_t uni_batch,
                                   float regularization, const float *g_in, const float *dq_in, float *stats_inout,
                                   const kge_adam_desc *adam, float *grad_entity, float *grad_relation,
                                   float *grad_modulus, float *losses_out, void *workspace, size_t workspace_bytes,
                                   int32_t *err_flag, void *stream, int64_t entity_begin, int64_t entity_end,
                                   int32_t csr_ready, int32_t reg_relations);

/*
 * kge_train_step_from_rows_range in phases (KGE_PHASE_ROWS: q rebuilt, the
 * positive epilogue, the relation pass; KGE_PHASE_ENTITY: the entity-major
 * pass + fused Adam of the rows [entity_begin, entity_end); KGE_PHASE_FINALIZE:
 * the losses, with the regulariser over [entity_begin, entity_end)), the same
 * arguments in every call.  An owner runs ROWS once, ENTITY once per chunk of
 * its rows — the all-gather of each finished chunk overlapping the next
 * chunk's pass — and FINALIZE over its whole range: bit-identical to one
 * kge_train_step_from_rows_range call.
 */
int kge_train_step_from_rows_phased(const kge_model_desc *m, int32_t mode, const int64_t *pos, const int64_t *neg,
                                    int64_t batch, int64_t nneg, const float *subsampling_weight,
                                    const float *weight_sum, int32_t uni_weight, int64_t uni_batch,
                                    float regularization, const float *g_in, const float *dq_in, float *stats_inout,
                                    const kge_adam_desc *adam, float *grad_entity, float *grad_relation,
                                    float *grad_modulus, float *losses_out, void *workspace, size_t workspace_bytes,
                                    int32_t *err_flag, void *stream, int32_t phases, int64_t entity_begin,
                                    int64_t entity_end, int32_t csr_ready, int32_t reg_relations);

/*
 * Query shipping: the training step of model.py:252-312 with the entity table
 * split into row shards, one per rank (no rank holds another's rows — the
 * reference's single table, model.py:45-53, never exists as a whole).  The
 * ranks exchange the global batch's ids and q vectors, not rows; every row-
 * side term is computed by the owner of the row.  The model descriptor's
 * entity_embedding points own_begin rows before this rank's shard and its
 * nentity is the GLOBAL entity count; the Adam entity pointers (and
 * grad_entity) are offset the same way.  Stages, each a call with the same
 * arguments, with the host's collectives between them:
 *   KGE_SHIP_Q      q_i (and head-batch the positive's h∘r) from the owner
 *                   of its row, zero elsewhere         → all-reduce(SUM) q[, qp]
 *   KGE_SHIP_ROWS   the owned negatives of every row: partial softmax state,
 *                   V relative to this shard's max (and the occurrence CSR,
 *                   on a side stream)                  → all-gather part → parts
 *   KGE_SHIP_MERGE  the rows' softmax over the shards (shard order), this
 *                   shard's dL/dq share and dL/ds; the positive triple on the
 *                   owner of t                         → all-reduce(SUM) dq | pstats [| pq]
 *   KGE_SHIP_CHAIN  chain rule on the owners of h / t; this shard's part of the
 *                   relation gradient (regulariser on rank 0) into
 *                   grad_relation                      → all-reduce(SUM) grad_relation,
 *                   relation Adam by the caller
 *   KGE_SHIP_ENTITY entity-major pass + fused Adam over [own_begin, own_end),
 *                   losses (regulariser partial of the owned rows; of the
 *                   relations on rank 0 only), pRotatE modulus grad + Adam
 * Same maths as one process on the global batch; the cross-shard sums run in
 * another order, so results agree to fp32 rounding, not bit for bit.
 */
#define KGE_SHIP_Q 1
#define KGE_SHIP_ROWS 2
#define KGE_SHIP_MERGE 3
#define KGE_SHIP_CHAIN 4
#define KGE_SHIP_ENTITY 5
typedef struct kge_ship_desc {
  int32_t world, rank;
  int64_t own_begin, own_end;       /* entity rows this rank owns (global ids) */
  const int64_t *pos, *neg;         /* [B,3], [B,n] the global batch (all ranks' rows, rank order) */
  int64_t batch, nneg;              /* B (global), n */
  const float *subsampling_weight;  /* [B] */
  const float *weight_sum;          /* global Σw (device scalar; unused with uni_weight) */
  int32_t uni_weight, adversarial;
  int64_t uni_batch;
  float adversarial_temperature, regularization;
  float *q, *qp;                    /* [B, Le] each; qp: head-batch only */
  float *part;                      /* [B, 4] */
  const float *parts;               /* [world, B, 4] */
  float *scores, *g;                /* [B, n] each */
  float *dq, *pq, *pstats;          /* [B, Le], [B, Le] (head-batch), [B, 4] */
  float *ent_contrib, *rel_contrib; /* [2B, Le], [B, Lr] */
  float *row_stats;                 /* [B, 4] */
} kge_ship_desc;
int kge_ship_step(const kge_model_desc *m, int32_t mode, const kge_ship_desc *ship, int32_t stage,
                  const kge_adam_desc *adam, float *grad_entity, float *grad_relation, float *grad_modulus,
                  float *losses_out, void *workspace, size_t workspace_bytes, int32_t *err_flag, void *stream);


/*
 * Σ subsampling_weight into *out (device scalar) — the denominator of
 * model.py:285-286; exposed so data-parallel ranks can all-reduce it.
 */
int kge_weight_sum(const float *w, int64_t n, float *out, void *stream);

/*
 * One dense Adam update — replaces torch.optim.Adam.step() as the reference
 * uses it (run.py:266-269, model.py:303; betas/eps defaults, no weight decay,
 * no amsgrad).  step_size = lr / (1 - beta1^t) and bias_correction2_sqrt =
 * sqrt(1 - beta2^t) are computed by the caller in double, as torch does.
 */
int kge_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t numel,
                  float beta1, float beta2, float eps, float step_size, float bias_correction2_sqrt,
                  void *stream);

/*
 * Filtered link-prediction ranks — replaces the per-batch body of
 * KGEModel.test_step (model.py:383-418) with TestDataset's filter semantics
 * (dataloader.py:134-154).
 *   queries [nq,3] (h,r,t); mode KGE_HEAD_BATCH ranks the head, KGE_TAIL_BATCH the tail.
 *   filter CSR: for query q the ids filt_ids[filt_off[q] .. filt_off[q+1]) are the
 *   candidates (other than the true one) that form a true triple in
 *   all_true_triples; the reference gives them bias -1 and the true id
 *   (dataloader.py:138-144), so they never outrank the positive.
 *   ranks_out [nq] int64: 1 + #{unfiltered e != true : score_e > score_true}.
 *   ties_out  [nq] int32 (nullable): #{unfiltered e != true : score_e == score_true}
 *   (the reference's argsort is not stable; a tie may land either side).
 * "score" is the reference's own fp32 score: a fast fp32 pass counts every
 * candidate whose score clears the true one's by more than a rounding bound
 * and lists the rest, which are re-scored in the reference's operation order
 * (the ATen elementwise ops and its sum(dim=2) / norm(p=1) reduction order) —
 * bit-exact to the reference for TransE, DistMult and ComplEx, and for RotatE
 * when m->relation_trig holds the reference's cos / sin of the relation phases
 * (without it: correctly rounded values, which differ from the reference's
 * CPU vector library in the last bit on a few percent of arguments).
 * pRotatE's sin acts on per-candidate phase sums, so it cannot be tabulated:
 * correctly rounded in this one-call form (ranks equal the reference's up to
 * that last bit); bit-exact with the three-call form below
 * (KGE_RANK_STAGE_LIST, kge_rank_sin_args, kge_rank_finish_sin).
 */
size_t kge_rank_workspace_bytes(const kge_model_desc *m, int64_t nq);
int kge_rank_filtered(const kge_model_desc *m, int32_t mode, const int64_t *queries, int64_t nq,
                      const int64_t *filt_off, const int64_t *filt_ids, int64_t *ranks_out,
                      int32_t *ties_out, void *workspace, size_t workspace_bytes, int32_t *err_flag,
                      void *stream);
/*
 * The same with the fast pass chosen (path: 0 auto, 1 split-bf16 MFMA tile —
 * DistMult / ComplEx, 4 fp32 MFMA tile — DistMult / ComplEx with float4-aligned
 * rows, 2 register tile — reduction length % 4 == 0, 3 wave scan; KGE_ERR_ARG
 * if the rows do not suit the requested path) and
 * listed_out [nq] int32 (nullable): near-ties re-scored per query (above the
 * 1024-per-query list capacity the query is rescanned exactly).  Every path
 * returns the same ranks and ties.  path | KGE_RANK_REUSE_TABLE: the caller
 * asserts that the entity table's CONTENTS are unchanged since the last
 * ranking call on this workspace (the other direction or another query block
 * of one evaluation, any nq).  The table statistics and split operands that
 * call left at the start of the workspace are reused only where a tag written
 * beside them (on the device, stream-ordered) shows they were written for the
 * same table pointer and shape — a call on another table, or one whose path
 * wrote no split operands, makes this call recompute them.
 */
#define KGE_RANK_REUSE_TABLE 0x100
/* path | KGE_RANK_STAGE_LIST (pRotatE only, listed_out required, ranks_out
 * unused): stop after the fast pass — listed_out holds each query's near-tie
 * count and the lists stay in the workspace for kge_rank_sin_args /
 * kge_rank_finish_sin below. */
#define KGE_RANK_STAGE_LIST 0x200
/* path | KGE_RANK_FILTER_TABLE: filt_off / filt_ids are the whole filter
 * index instead of per-query lists: filt_off [E·R + 1] int64 start offsets,
 * by key h·R + r (tail-batch) or r·E + t (head-batch), into filt_ids — every
 * true triple's tail (tail-batch) or head (head-batch), sorted by key.  The
 * device looks each query's list up itself (no per-query CSR on the host);
 * the same ranks and ties. */
#define KGE_RANK_FILTER_TABLE 0x400
#define KGE_RANK_LIST_CAP 1024 /* listed near-ties per query; above it the query is rescanned in full */
int kge_rank_filtered_ex(const kge_model_desc *m, int32_t mode, const int64_t *queries, int64_t nq,
                         const int64_t *filt_off, const int64_t *filt_ids, int64_t *ranks_out,
                         int32_t *ties_out, int32_t *listed_out, int32_t path, void *workspace,
                         size_t workspace_bytes, int32_t *err_flag, void *stream);
/*
 * Both directions of one evaluation in one pass (model.py:349-418 ranks every
 * test triple as a head-batch query, then as a tail-batch query): the same
 * ranks and ties as kge_rank_filtered_ex(KGE_HEAD_BATCH, ...) followed by
 * kge_rank_filtered_ex(KGE_TAIL_BATCH, ...) on the same queries, written to
 *   ranks_out / ties_out / listed_out [2·nq]: the head-batch direction's nq,
 *   then the tail-batch direction's;
 * filt_off_head / filt_ids_head and filt_off_tail / filt_ids_tail: each
 * direction's filter (per-query lists, or with KGE_RANK_FILTER_TABLE each
 * direction's whole filter index).  The workspace holds 2·nq queries
 * (kge_rank_workspace_bytes(m, 2·nq)).  The mode-independent stages — the
 * table's statistics and split operands, the split of every q, the MFMA
 * counting tile and the emission — run once over all 2·nq queries; the
 * mode-dependent ones (q, filter bitmap, windows, refinement) once per
 * direction.  Not with KGE_RANK_STAGE_LIST (pRotatE's three-call form is per
 * direction): KGE_ERR_ARG.
 */
int kge_rank_filtered_both(const kge_model_desc *m, const int64_t *queries, int64_t nq,
                           const int64_t *filt_off_head, const int64_t *filt_ids_head,
                           const int64_t *filt_off_tail, const int64_t *filt_ids_tail, int64_t *ranks_out,
                           int32_t *ties_out, int32_t *listed_out, int32_t path, void *workspace,
                           size_t workspace_bytes, int32_t *err_flag, void *stream);

/*
 * pRotatE ranks bit-exact to the reference — whose sin (model.py:245) is its
 * CPU vector library's (ATen → MKL VML here), which no device instruction
 * sequence reproduces — in three calls on one stream and workspace:
 *   1. kge_rank_filtered_ex(..., path | KGE_RANK_STAGE_LIST, listed_out): fast
 *      pass, windows widened by the library's ≤ 1 ulp, near-tie lists; then
 *      every listed candidate's score as an interval under ANY sin within one
 *      ulp of the exact value, in the reference's operation order (each later
 *      operation is monotone), and the candidates whose interval clears the
 *      true score's are decided on the device.  listed_out[q] = the candidates
 *      left for the library sin (0: the query is fully ranked; > KGE_RANK_LIST_CAP:
 *      a degenerate window with more undecided candidates than a list, ranked on
 *      the device with correctly rounded sin instead).
 *   2. the caller sets item_off [nq + 1] (device int64, exclusive scan) to
 *      n_items(q) = 1 + listed_out[q] for 1 ≤ listed_out[q] ≤ KGE_RANK_LIST_CAP,
 *      else 0; kge_rank_sin_args writes args_out [item_off[nq], entity_dim]: per
 *      item (0 = the true entity, then the listed candidates) the K phase sums
 *      θh + (θr − θt) (head-batch) or (θh + θr) − θt (tail-batch) the reference
 *      takes the sin of (model.py:236-245; IEEE divisions and adds,
 *      host-independent).
 *   3. the caller evaluates sin_values = sin(args) with the reference's own
 *      library call (torch.sin on the host CPU) and kge_rank_finish_sin
 *      re-scores every item from those values in the reference's order
 *      (abs, ATen sum(dim=2), × modulus, γ −) and writes ranks / ties / listed
 *      as kge_rank_filtered_ex does.
 * Steps 2-3 may be repeated over disjoint subsets of the queries (a query
 * outside the subset gets 0 items) to bound the caller's buffers; ranks are
 * final once every query with items has been delivered once.  A query whose
 * non-empty item range does not hold exactly 1 + listed_out[q] items, a second
 * delivery of a query, or a call whose mode / nq / entity table differ from the
 * list stage's (or after another ranking call used the workspace) sets
 * KGE_DEVERR_ARG.
 */
/*
 * Self-test of the bound the pRotatE list stage's interval screen relies on:
 * writes to max_dist_out (device int32, zeroed by the caller) the largest
 * distance, in representable floats, between the device's sinf and the
 * correctly rounded sin over every float x with |x| <= range (where the double
 * sin lies next to a float midpoint, against both floats it may round to).
 * The screen assumes at most 1 for |x| <= 16 and 2 for |x| <= 65536
 * (kge_rank_ref.h SIN_FAST_*); tests/test_rank_parity_gpu.py checks both on
 * each GPU.
 */
int kge_selftest_sin(float range, int32_t *max_dist_out, void *stream);

int kge_rank_sin_args(const kge_model_desc *m, int32_t mode, int64_t nq, const int64_t *item_off, float *args_out,
                      void *workspace, size_t workspace_bytes, int32_t *err_flag, void *stream);
int kge_rank_finish_sin(const kge_model_desc *m, int32_t mode, int64_t nq, const int64_t *item_off,
                        const float *sin_values, int64_t *ranks_out, int32_t *ties_out, int32_t *listed_out,
                        void *workspace, size_t workspace_bytes, int32_t *err_flag, void *stream);

/*
 * Live stage timing for benchmarks (no reference counterpart): when enabled,
 * kge_train_step_grads records a hipEvent on its stream before and after each
 * stage of the caller's stream — 0 q build, 1 fused negative scoring +
 * self-adversarial loss (the gather loop), 2 positive score + chain rule,
 * 3 wait for the occurrence CSR (built on an internal side stream in parallel
 * with stages 0-2), 4 entity-major gradient pass (+ fused Adam), 5 wait for the
 * relation pass (side stream, parallel with 4) + loss finalisation.
 *   command 1: enable and reset, timing one call in every n_out (n_out <= 0:
 *              every call) — sampling keeps the event records' own cost
 *              (~4 % of a step when every call is timed) out of the throughput;
 *   command 0: disable and reset;
 *   command 2: synchronise the recorded events and write the summed
 *              milliseconds per stage to stage_ms_out[0..5] and the number of
 *              timed calls to stage_ms_out[6] (n_out >= 7);
 *   command 3: the same per timed call: stage_ms_out[7c .. 7c+5] the call's
 *              stage times, stage_ms_out[7c+6] its start (ms after the first
 *              timed call's start); n_out >= 7 × timed calls.
 *   command 4: enable and reset the RANKING timer: every kge_rank_filtered* call
 *              (and pRotatE's three-call form, list → finish) records events
 *              at its start, around its fast counting pass and after its ranks
 *              are written (every finish call of the three-call form marks
 *              "ranks written"; the last one before the next call counts)
 *              (command 0 disables it too);
 *   command 5: synchronise them and write the summed milliseconds of its
 *              KGE_RANK_TIMER_STAGES stages — 0 query / filter / table
 *              preparation and windows, 1 the fast counting pass (MFMA tile,
 *              register tile or wave scan), 2 near-tie refinement and rank
 *              emission (pRotatE's three-call form: including the caller's
 *              host sin between the calls) — then the number of DIRECTIONS
 *              ranked (a kge_rank_filtered_both call counts 2) (n_out >= 4).
 * Not graph-capturable while enabled.
 */
#define KGE_TIMER_STAGES 6
#define KGE_RANK_TIMER_STAGES 3
int kge_stage_timer(int32_t command, float *stage_ms_out, int32_t n_out);

/*
 * Device negative sampler: one training batch as TrainDataset.__getitem__ +
 * collate_fn build it (dataloader.py:34-66, sampling loop :44-61), for the
 * triples `batch[0..batch_size)` (ids into `triples`).
 *   pos_out[i] = triples[batch[i]], w_out[i] = weights[batch[i]]
 *     (weights = sqrt(1 / (count(h,r) + count(t,-r-1))), dataloader.py:40-42)
 *   neg_out[i, :] = the first negative_sample_size draws of row i's uniform
 *     stream over [0, nentity) that are NOT in the row's true list — the true
 *     heads of (r, t) for head-batch, the true tails of (h, r) for tail-batch
 *     (dataloader.py:47-56): true_ids[true_off[t] .. + true_len[t]), sorted.
 * Row i's stream is a splitmix64 sequence keyed by (key, i); the caller
 * advances `key` every batch.  The reference draws with numpy's global
 * MT19937, so parity is distributional and bit-exact against
 * the restatement of this generator in oracle/kge_oracle.py.
 * A row still short after max_draws draws sets KGE_DEVERR_SAMPLER (the
 * reference would loop forever) and is zero-padded.
 */
int kge_sample_negatives(const int64_t *triples, int64_t ntriples, const int64_t *batch, int64_t batch_size,
                         int64_t nentity, int64_t negative_sample_size, const int64_t *true_off,
                         const int32_t *true_len, const int64_t *true_ids, const float *weights, uint64_t key,
                         int64_t max_draws, int64_t *pos_out, int64_t *neg_out, float *w_out, int32_t *err_flag,
                         void *stream);

#ifdef __cplusplus
}
#endif

#endif /* KGE_HIP_H */
