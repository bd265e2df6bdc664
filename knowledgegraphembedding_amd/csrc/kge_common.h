// kge_common.h — argument blocks and launchers of the model-independent kernels.
#pragma once
#include "kge_internal.h"

namespace kge {

struct CsrArgs {
  const int64_t* pos;
  const int64_t* neg;
  int64_t neg_stride;
  int64_t B, n, Bn, E, R;
  int32_t* keys;  // [Bn + 3B]
  int32_t* cnt;   // [E + R + 1]  (last slot stays 0: the scan's total)
  int32_t* off;   // [E + R + 1]
  int32_t* tmp;   // [Bn + 3B]
  int32_t* occ;   // [Bn + 3B]
  int32_t* err;
  int64_t e_lo, e_hi;  // entity buckets built: [e_lo, e_hi) (an owner's rows); the others stay empty
  void* scan_tmp;  // rocPRIM scan scratch (csr_scan_temp_bytes)
  size_t scan_tmp_bytes;
};



int launch_rank_mfma(int gather, const float* q, const float* ent, int64_t nq, int64_t E, int K,
                     const int64_t* true_id, float* s_true, const uint32_t* bits, int32_t* gt, const RankWin& win,
                     hipStream_t s);
// split-bf16 MFMA tile (path "mfma"): operands split once per call into bf16 hi | lo pieces
int64_t xsplit_nslab(int K);
// (three bf16 MFMAs per fp32 product: the lo·lo products are dropped, +258.1·u·P
// on the error bound — kge_rank_mfma.hip, kge_capi.hip rank_impl)
int64_t xsplit_elems(int64_t rows, int K);
int launch_split_bf16(const float* src, int64_t rows, int K, uint16_t* dst, hipStream_t s,
                      const int64_t* skip = nullptr);
int launch_rank_mfma_x(int gather, const uint16_t* qs, const uint16_t* es, int64_t nq, int64_t E, int K,
                       const int64_t* true_id, float* s_true, const uint32_t* bits, int32_t* gt, const RankWin& win,
                       hipStream_t s);
constexpr int TS_BLOCKS = 2048;  // k_table_stats / k_split_stats grid bound
constexpr int TS_NSTAT = 4;      // max ‖e‖, max |x|, max ‖r_e‖, max ‖lo_e‖: stats holds TS_NSTAT·(1 + TS_BLOCKS) floats
int launch_table_stats(const float* ent, int64_t E, int Le, float* stats, hipStream_t s,
                       const int64_t* skip = nullptr);
// the entity table's split (launch_split_bf16) and statistics (launch_table_stats) in one read
int launch_split_stats(const float* ent, int64_t E, int K, uint16_t* dst, float* stats, hipStream_t s,
                       const int64_t* skip_stats, const int64_t* skip_split);
// the ranking workspace's table tag (KGE_RANK_REUSE_TABLE; kge_rank_mfma.hip k_rank_tag)
int launch_rank_tag(int64_t* tag, const float* ent, int64_t E, int Le, int reuse, int need_stats, int split_kind,
                    int64_t split_param, hipStream_t s);
// kge_selftest_sin (kge_rank_mfma.hip): max float distance of sinf from the correctly rounded sin on |x| ≤ range
int launch_selftest_sin(float range, int32_t* maxd, hipStream_t s);
// pRotatE's (cos, sin) / (sin, cos) phase table for the register tile ([rows][K][2]; kge_rank_mfma.hip)
int launch_prot_phase(const float* src, int64_t rows, int K, float kappa, int ent, float* dst, hipStream_t s,
                      const int64_t* skip = nullptr);
int launch_filter_bits_tab(const int64_t* queries, int head, const int64_t* tab, const int64_t* vals,
                           const int64_t* true_id, int64_t nq, int64_t E, int64_t R, uint32_t* bits, int32_t* err,
                           hipStream_t s);
// both directions in one launch (blocks nq.. tail-batch's): tab != 0 → off_* are the
// dense key tables, else per-query list offsets; -1 when the rows are too wide (per direction then)
int launch_filter_bits_both(const int64_t* queries, int tab, const int64_t* off_h, const int64_t* ids_h,
                            const int64_t* off_t, const int64_t* ids_t, const int64_t* true_id, int64_t nq,
                            int64_t E, int64_t R, uint32_t* bits, int32_t* err, hipStream_t s);
int launch_filter_bits(const int64_t* filt_off, const int64_t* filt_ids, const int64_t* true_id, int64_t nq,
                       int64_t E, uint32_t* bits, int32_t* err, hipStream_t s);
struct EmitArgs {
  const int32_t *gt, *eq, *gtx, *eqx, *ucnt;
  const int64_t* true_id;
  int64_t nq;
  int cap;
  int64_t* ranks;
  int32_t* ties;    // may be null
  int32_t* listed;  // may be null: near-ties listed per query (diagnostics)
  int64_t* ltag;    // non-null (pRotatE's list stage): the list tag written for the later stages
  int64_t ltag_v[3];
};
int launch_rank_emit(const EmitArgs& a, hipStream_t s);
size_t csr_scan_temp_bytes(int64_t nb);
int launch_csr(const CsrArgs& a, hipStream_t s);
int launch_rel_rows(const RelArgs& a, hipStream_t s);
int launch_finalize(const FinArgs& a, hipStream_t s);
int launch_weight_sum(const float* w, int64_t n, float* out, hipStream_t s);
int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float b1, float b2, float eps,
                float step_size, float bc2s, hipStream_t s);

}  // namespace kge
