// kge_capi.hip — the extern "C" boundary declared in include/kge_hip.h.
// Host-side argument checks, workspace carving and launch sequencing; no
// allocation, no synchronisation (graph-capturable).
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "kge_common.h"

namespace kge {
namespace {

struct Geom {
  int vec, ns;
  RowGeom eg;
  bool cplx;
};

const ModelOps& ops_for(int model) {
  static const ModelOps tbl[5] = {model_ops_transe(), model_ops_distmult(), model_ops_complex(),
                                  model_ops_rotate(), model_ops_protate()};
  return tbl[model];
}

int hip_status(hipError_t e) { return e == hipSuccess ? KGE_OK : (KGE_ERR_HIP_BASE + (int)e); }
int launch_status(int e) { return e == 0 ? KGE_OK : (e < 0 ? KGE_ERR_DIM : KGE_ERR_HIP_BASE + e); }

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// model.py:63-70 plus the broadcast rules of the plug-ins.
int check_model(const kge_model_desc* m, Geom* g) {
  if (!m) return KGE_ERR_ARG;
  // a caller built against another layout of this struct (KGE_ABI_VERSION)
  if (m->struct_size != (int32_t)sizeof(kge_model_desc)) return KGE_ERR_ABI;
  if (m->model < KGE_TRANSE || m->model > KGE_PROTATE) return KGE_ERR_MODEL;
  if (!m->entity_embedding || !m->relation_embedding) return KGE_ERR_ARG;
  if (m->nentity <= 0 || m->nrelation <= 0 || m->entity_dim <= 0 || m->relation_dim <= 0) return KGE_ERR_ARG;
  if (m->nentity >= (int64_t)1 << 31 || m->nrelation >= (int64_t)1 << 30) return KGE_ERR_DIM;
  const int Le = m->entity_dim, Lr = m->relation_dim;
  g->cplx = (m->model == KGE_COMPLEX || m->model == KGE_ROTATE);
  int span;
  if (m->model == KGE_ROTATE) {
    if (Le != 2 * Lr) return KGE_ERR_SHAPE;  // RotatE: -de, not -dr
    span = Lr;
  } else if (m->model == KGE_COMPLEX) {
    if (Le != Lr || (Le & 1)) return KGE_ERR_SHAPE;  // ComplEx: -de and -dr
    span = Le / 2;
  } else {
    if (Le != Lr) return KGE_ERR_SHAPE;
    span = Le;
  }
  if (m->model == KGE_PROTATE && !m->modulus) return KGE_ERR_ARG;
  const bool v4 = (span % 4 == 0) && aligned16(m->entity_embedding) && aligned16(m->relation_embedding);
  g->vec = v4 ? 4 : 1;
  const int S = span / g->vec;
  int ns = 1;
  while (64 * ns < S) ns *= 2;
  if (ns > (g->vec == 4 ? 8 : 32)) {
    // (half-)rows over 2048 floats: the run-time-looped kernels of
    // kge_wide.inc (single-float elements, ns = 0)
    g->vec = 1;
    g->ns = 0;
    g->eg.S = span;
    g->eg.half = g->cplx ? span : 0;
    return KGE_OK;
  }
  g->ns = ns;
  g->eg.S = S;
  g->eg.half = g->cplx ? span : 0;
  return KGE_OK;
}

// Fast counting pass of the filtered ranking (path 0 = auto): the split-bf16
// MFMA tile for DistMult / ComplEx (path 1; the fp32 MFMA tile, path 4, when
// the split operands would pass 32-bit buffer offsets), the register tile for
// the others when the reduction length is a multiple of 4, the wave scan
// otherwise.  Every path ends in the same reference-order refinement, so all
// give the same ranks.
enum RankPath : int { RP_AUTO = 0, RP_MFMA = 1, RP_TILE = 2, RP_SCAN = 3, RP_MFMA32 = 4 };
int rank_path(const kge_model_desc* m, int requested) {
  const bool bil = (m->model == KGE_DISTMULT || m->model == KGE_COMPLEX);
  const bool cplx = (m->model == KGE_ROTATE || m->model == KGE_COMPLEX);
  const int K = cplx ? m->entity_dim / 2 : m->entity_dim;
  const bool al = aligned16(m->entity_embedding);
  // (the MFMA tiles address their operands through 32-bit buffer offsets)
  const bool x_ok = bil && (uint64_t)xsplit_elems(m->nentity, m->entity_dim) * 2u < 0x7FFFFFF0ull;
  const bool mfma_ok = bil && (m->entity_dim % 4 == 0) && al &&
                       (uint64_t)m->nentity * (uint64_t)m->entity_dim * 4u < 0xFFFFFF00ull;
  // (the register tile's counting pass reads a block's 64 rows — pRotatE:
  // their 2K-float phase rows — through one buffer descriptor)
  const bool tile_ok = (K % 4 == 0) && al && (uint64_t)64 * 2 * (uint64_t)m->entity_dim * 4u < 0x7FFFFFF0ull;
  if (requested == RP_MFMA) return x_ok ? RP_MFMA : -1;
  if (requested == RP_MFMA32) return mfma_ok ? RP_MFMA32 : -1;
  if (requested == RP_TILE) return tile_ok ? RP_TILE : -1;
  if (requested == RP_SCAN) return RP_SCAN;
  return x_ok ? RP_MFMA : mfma_ok ? RP_MFMA32 : (tile_ok ? RP_TILE : RP_SCAN);
}
constexpr int RANK_CAP = KGE_RANK_LIST_CAP;  // listed near-ties per query before the exact rescan takes over
static_assert(RANK_CAP <= 1024, "k_rank_refine's pRotatE screen holds 4 list entries per thread of 256");

Consts consts_of(const kge_model_desc* m) {
  Consts c;
  c.gamma = m->gamma;
  c.kappa = m->phase_divisor;
  c.kappa_p = m->phase_divisor_p;
  c.modulus = 0.f;
  return c;
}

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* p) : base((char*)p) {}
  template <typename T>
  T* take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T* p = base ? (T*)(base + off) : nullptr;
    off += count * sizeof(T);
    return p;
  }
};

struct GradWs {
  float *g, *q, *dq, *ent_contrib, *rel_contrib, *row_stats, *reg_partial, *wsum;
  int32_t *keys, *cnt, *off, *tmp, *occ;
  float* q_sl;  // slice-major q for the sliced entity pass (single-call steps with even slices)
  void* scan_tmp;
  size_t scan_tmp_bytes;
};

GradWs carve_grad(void* ws, const kge_model_desc* m, int64_t B, int64_t n, size_t* bytes) {
  Carver c(ws);
  GradWs w;
  const int64_t Bn = B * n, N = Bn + 3 * B, nb = m->nentity + m->nrelation;
  w.g = c.take<float>(Bn);
  w.q = c.take<float>(B * (int64_t)m->entity_dim);
  w.dq = c.take<float>(B * (int64_t)m->entity_dim);
  w.ent_contrib = c.take<float>(2 * B * (int64_t)m->entity_dim);
  w.rel_contrib = c.take<float>(B * (int64_t)m->relation_dim);
  w.row_stats = c.take<float>(B * 4);
  w.reg_partial = c.take<float>(8 * m->nentity + m->nrelation);  // per (entity, column slice) + per relation
  w.wsum = c.take<float>(4);
  w.keys = c.take<int32_t>(N);
  w.cnt = c.take<int32_t>(nb + 1);
  w.off = c.take<int32_t>(nb + 1);
  w.tmp = c.take<int32_t>(N);
  w.occ = c.take<int32_t>(N);
  w.q_sl = c.take<float>(8 * B * 512);  // up to 8 slices × B rows × (64 + 64) float4 slots
  w.scan_tmp_bytes = csr_scan_temp_bytes(nb);
  w.scan_tmp = c.take<uint8_t>((int64_t)w.scan_tmp_bytes);
  *bytes = c.off + 256;
  return w;
}

hipStream_t as_stream(void* s) { return (hipStream_t)s; }

// ---- stage timer (bench instrumentation; see kge_stage_timer in the header)
struct StageTimer {
  bool on = false;
  int period = 1;              // time one train call in `period`
  size_t seen = 0;             // train calls since enabled
  std::vector<hipEvent_t> ev;  // (KGE_TIMER_STAGES + 1) events per timed call
  size_t used = 0;             // events recorded so far
  hipEvent_t next(hipStream_t) {
    if (used == ev.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      ev.push_back(e);
    }
    return ev[used++];
  }
  void mark(hipStream_t s) {
    if (!on) return;
    hipEvent_t e = next(s);
    if (e) hipEventRecord(e, s);
  }
};
StageTimer g_timer;
void timer_mark(hipStream_t s) { g_timer.mark(s); }
// the ranking's stage timer (kge_stage_timer commands 4 / 5): marks tagged by
// slot — 0 the call starts (with the call's number of directions), 1 fast pass
// begins, 2 fast pass ends, 3 ranks written.  A call is the marks from one
// slot-0 mark to the next; a stage is the time between the call's first mark of
// its slot and its last mark of the next slot, so a call that writes ranks in
// several pieces (pRotatE's per-chunk finish calls each mark slot 3) is timed to
// its last piece, and the list stage's own calls need no padding.
struct RankTimer {
  bool on = false;
  std::vector<hipEvent_t> ev;
  std::vector<int> slot, ndir;
  size_t used = 0;
  void mark(hipStream_t s, int sl, int nd = 1) {
    if (!on) return;
    if (used == ev.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      ev.push_back(e);
      slot.push_back(0);
      ndir.push_back(0);
    }
    if (hipEventRecord(ev[used], s) != hipSuccess) return;
    slot[used] = sl;
    ndir[used] = nd;
    ++used;
  }
};
RankTimer g_rank_timer;

// ---- side stream: the index-only work (occurrence CSR) and the relation
// pass run beside the gather kernels of the caller's stream.  Fork/join via
// events (a pattern stream capture records as graph edges); the caller's
// stream never runs ahead of anything the side stream still reads or writes.
struct Side {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, csr_done = nullptr, epi_done = nullptr, rel_done = nullptr;
  hipEvent_t rk_fork = nullptr, rk_join = nullptr;  // ranking: the entity table's statistics / split beside the queries' stages
};
// Diagnostic switches, read per call so a test can flip them between calls;
// none changes a result bit (each selects between paths that are tested
// bitwise equal): KGE_ENT_SLICES (force the entity pass's column-slice count;
// 0 = the row-per-wave k_entity), KGE_FIN_SEPARATE (the loss finalisation as
// its own launch), KGE_RANK_SIN_SCREEN=0 (pRotatE: send every listed
// near-tie to the caller's sin, no device screen).
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

Side* side_for_device() {
  static Side sides[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  Side& sd = sides[dev];
  if (!sd.s) {
    if (hipStreamCreateWithFlags(&sd.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    hipEventCreateWithFlags(&sd.fork, hipEventDisableTiming);
    hipEventCreateWithFlags(&sd.csr_done, hipEventDisableTiming);
    hipEventCreateWithFlags(&sd.epi_done, hipEventDisableTiming);
    hipEventCreateWithFlags(&sd.rel_done, hipEventDisableTiming);
    hipEventCreateWithFlags(&sd.rk_fork, hipEventDisableTiming);
    hipEventCreateWithFlags(&sd.rk_join, hipEventDisableTiming);
  }
  return &sd;
}

// Data-parallel factor exchange (kge_train_rows_slice / kge_train_step_from_rows)
// XS_CSR_ONLY: the occurrence CSR of a batch alone, on the caller's stream;
// XS_FROM_ROWS_CSR: XS_FROM_ROWS with that CSR already in the workspace
enum XStage : int { XS_NONE = 0, XS_ROWS_ONLY = 1, XS_FROM_ROWS = 2, XS_CSR_ONLY = 3, XS_FROM_ROWS_CSR = 4 };

// entity pass variant: column slices (k_entity_sl) when the row fits one
// 16-B slot per lane per slice (returns the slice count); 0 selects the
// row-per-wave pass (also forced by KGE_ENT_SLICES=0)
int entity_slices(const Geom& geo, int64_t B, int Le) {
  const int forced = env_int("KGE_ENT_SLICES", -1);  // read per call (tests switch it)
  const int S = geo.eg.S;
  auto fits = [&](int k) { return (S + k - 1) / k <= 64; };
  if (geo.vec != 4 || forced == 0) return 0;
  int k = forced;
  if (k < 0) {
    // smallest power of two that fits; doubled further while the q column
    // slice exceeds 2 MiB (half an XCD L2) only if the waves stay >= 3/4
    // busy (measured: a larger slice beats half-empty waves — global batch
    // of 2048 rows, 4 slices 0.54 ms vs 8 slices 0.73 ms)
    const double qslice = (double)B * Le * sizeof(float);
    k = 1;
    while (k < 8 && !fits(k)) k *= 2;
    while (k < 8 && qslice / k > 2.0 * 1024 * 1024 && (S + 2 * k - 1) / (2 * k) >= 48) k *= 2;
  }
  return ((k == 1 || k == 2 || k == 4 || k == 8) && fits(k)) ? k : 0;
}

// Line-aligned slicing for k_entity_sl (align_sl): the inner slice boundaries
// of a row move by the row's 16-B phase within its 128-B line so they fall on
// line boundaries of the row's first half.  Only when every stream of the pass
// (table = Adam param, gradient, moments) has the same phase, every row's
// phase is one the 64-slot slices absorb (last slice ≤ 64 slots) — d = 1000:
// phases 0 and 4.
int entity_slice_align(int nsl, int S, int Le, const float* ent, const float* grad, const AdamT& ad) {
  if (nsl < 2) return 0;
  const uintptr_t base = (uintptr_t)ent & 127;
  if (base & 15) return 0;
  for (const float* p : {grad, (const float*)ad.p, (const float*)ad.m, (const float*)ad.v})
    if (p && ((uintptr_t)p & 127) != base) return 0;
  if (S <= 64 * (nsl - 1)) return 0;
  int max_sh = 0;
  for (int e = 0; e < 8; ++e) {
    const int sh = (int)(((base + (uintptr_t)e * (uintptr_t)Le * 4u) >> 4) & 7);
    max_sh = sh > max_sh ? sh : max_sh;
  }
  return (S - 64 * (nsl - 1) + max_sh <= 64) ? 1 : 0;
}

// Shared body of backward and train.  Caller's stream: q build → gather loop →
// epilogue → entity pass → finalise; side stream: CSR ∥ row pass, relation pass ∥ entity pass.
int run_grad(const kge_model_desc* m, const Geom& geo, int mode, const int64_t* pos, const int64_t* neg,
             int64_t neg_stride, int64_t B, int64_t n, RowArgs ra, GradWs w, float* grad_entity,
             float* grad_relation, float* grad_modulus, float reg, FinArgs fa, const kge_adam_desc* adam,
             int32_t* err, hipStream_t s, int phases = KGE_PHASE_ALL, int64_t e_begin = 0, int64_t e_end = -1,
             int xstage = XS_NONE, int reg_relations = 1, int64_t csr_lo = 0, int64_t csr_hi = -1) {
  const ModelOps& op = ops_for(m->model);
  AdamK ak;
  ak.b1 = adam ? adam->beta1 : 0.f;
  ak.b2 = adam ? adam->beta2 : 0.f;
  ak.eps = adam ? adam->eps : 0.f;
  auto adam_t = [&](const kge_adam_tensor* t) {
    AdamT o;
    o.p = (adam && t && t->param) ? t->param : nullptr;
    o.m = o.p ? t->exp_avg : nullptr;
    o.v = o.p ? t->exp_avg_sq : nullptr;
    o.step_size = o.p ? t->step_size : 0.f;
    o.bc2s = o.p ? t->bias_correction2_sqrt : 1.f;
    return o;
  };
  const int write_grad = (!adam || adam->write_grad) ? 1 : 0;
  const Consts c = consts_of(m);
  const int Le = m->entity_dim, Lr = m->relation_dim;
  // k_row's LDS: q (2 padded halves), the merge buffer, the raw scores, the
  // wave states and, with the fused epilogue, the positive's element terms
  const bool wide = (geo.ns == 0);  // rows over 2048 floats (kge_wide.inc)
  const size_t lds = wide ? wide_row_lds(n)
                          : sizeof(float) * (2 * 64 * (size_t)geo.ns * geo.vec + (size_t)vb_floats(Le) + (size_t)ra.n_lds +
                                             32 + (ra.fuse_epi ? 64 * (size_t)geo.ns * geo.vec : 0));
  if (lds > 64 * 1024) return KGE_ERR_DIM;
  const bool all = (phases == KGE_PHASE_ALL);
  if (e_end < 0) e_end = m->nentity;
  // stage timing: a full call records all 7 marks; a phased ROWS call (the
  // data-parallel path) records the row-pass marks and pads the rest, so the
  // row pass is timed live on every rank either way
  const bool from_rows = (xstage == XS_FROM_ROWS || xstage == XS_FROM_ROWS_CSR);
  const bool csr_ready = (xstage == XS_FROM_ROWS_CSR);
  const bool timed = (phases & KGE_PHASE_ROWS) && !from_rows && xstage != XS_CSR_ONLY && g_timer.on && ra.op == ROW_TRAIN &&
                     (g_timer.seen++ % (size_t)g_timer.period) == 0;
  ra.timer_mid = timed ? &timer_mark : nullptr;
  Side* sd = side_for_device();
  hipStream_t ss = sd ? sd->s : s;
  int st;

  // wide rows: WIDE_PARTS column parts per entity (k_entity_w)
  const int nsl = wide ? WIDE_PARTS : entity_slices(geo, B, Le);
  const int64_t ent_parts = m->nentity * (int64_t)(nsl > 0 ? nsl : 1);
  // relation pass: as trailing blocks of the sliced entity launch (one call,
  // no stream join); else beside the entity pass on the side stream (always
  // so in phased calls, and for wide rows)
  const bool rel_fused = all && nsl > 0 && !wide;
  // slice-major q: k_row also writes q as [slice][row][re | im] so each of
  // the entity pass's q reads is 2 KB contiguous and line-aligned (0.240 ->
  // 0.234 ms at the FB15k shape); the single-call step with even slices only
  // (the line-aligned slices shift a row's columns by its phase, so they are
  // off here)
  const bool q_slm = all && nsl > 0 && geo.vec == 4 && xstage == XS_NONE && ra.op == ROW_TRAIN &&
                     (geo.eg.S + nsl - 1) / nsl <= 64;
  ra.q_sl = q_slm ? w.q_sl : nullptr;
  ra.q_sl_w = q_slm ? (geo.eg.S + nsl - 1) / nsl : 0;
  const bool rel_side = sd && !rel_fused;
  RelArgs rl;
  memset(&rl, 0, sizeof(rl));
  rl.rel = m->relation_embedding; rl.R = m->nrelation; rl.E = m->nentity; rl.B = B; rl.Bn = B * n; rl.Lr = Lr;
  rl.off = w.off; rl.occ = w.occ; rl.rel_contrib = w.rel_contrib; rl.reg3 = 3.f * reg;
  rl.reg_partial = w.reg_partial + ent_parts; rl.grad_rel = grad_relation;
  rl.write_grad = write_grad;
  rl.adam = adam_t(adam ? &adam->relation : nullptr);
  rl.adamk = ak;

  if (xstage == XS_ROWS_ONLY) {
    // the negative-row pass alone (q build + k_row), dL/dq to global memory for
    // the exchange; no epilogue, CSR or relation pass (kge_train_rows_slice)
    ra.fuse_epi = 0;
    if (timed) g_timer.mark(s);
    st = launch_status(op.row(mode, geo.vec, geo.ns, 0, ra, lds, s));
    if (st) return st;
    if (timed)
      for (int k = 0; k < 5; ++k) g_timer.mark(s);  // row-pass end + the stages not in this call
    return KGE_OK;
  }
  CsrArgs ca;
  ca.pos = pos; ca.neg = neg; ca.neg_stride = neg_stride;
  ca.B = B; ca.n = n; ca.Bn = B * n; ca.E = m->nentity; ca.R = m->nrelation;
  ca.keys = w.keys; ca.cnt = w.cnt; ca.off = w.off; ca.tmp = w.tmp; ca.occ = w.occ; ca.err = err;
  ca.e_lo = csr_lo; ca.e_hi = csr_hi < 0 ? m->nentity : csr_hi;
  ca.scan_tmp = w.scan_tmp; ca.scan_tmp_bytes = w.scan_tmp_bytes;
  if (xstage == XS_CSR_ONLY) return launch_status(launch_csr(ca, s));  // kge_train_csr
  if (from_rows) ra.fuse_epi = 0;  // the epilogue reads the gathered dL/dq (k_row_epi)

  // KGE_CSR_SERIAL=1 (diagnostic, same bits): the CSR on the caller's stream
  // before the row pass instead of beside it — what k_row gains without the
  // side stream's kernels competing for its CU slots
  const bool csr_serial = !csr_ready && env_int("KGE_CSR_SERIAL", 0) != 0;
  const bool use_csr = !csr_ready && !csr_serial;
  if (phases & KGE_PHASE_ROWS) {
  if (csr_serial) {
    st = launch_status(launch_csr(ca, s));
    if (st) return st;
  }
  // fork point: the occurrence CSR needs only the batch indices (recorded
  // before anything else is queued, so the side stream never waits for the
  // row pass)
  if (sd && use_csr) hipEventRecord(sd->fork, s);

  // q build + gather loop on the caller's stream, launched first so the GPU
  // is on the long kernel while the host queues everything else
  if (timed) g_timer.mark(s);
  // (XS_FROM_ROWS: the row pass ran on the ranks; only q is rebuilt here)
  st = launch_status(op.row(mode, geo.vec, geo.ns, from_rows ? 2 : 0, ra, lds, s));
  if (st) return st;
  if (timed) g_timer.mark(s);

  if (use_csr) {
    if (sd) hipStreamWaitEvent(ss, sd->fork, 0);
    st = launch_status(launch_csr(ca, ss));
    if (st) return st;
    if (sd) hipEventRecord(sd->csr_done, ss);
  }

  // epilogue (positive score, chain rule)
  st = launch_status(op.row(mode, geo.vec, geo.ns, 1, ra, lds, s));
  if (st) return st;
  if (timed) g_timer.mark(s);

  // relation pass on the side stream once the epilogue's contributions exist
  if (rel_side) {
    hipEventRecord(sd->epi_done, s);
    hipStreamWaitEvent(ss, sd->epi_done, 0);
    st = launch_status(launch_rel_rows(rl, ss));
    if (st) return st;
    hipEventRecord(sd->rel_done, ss);
  } else if (!all) {
    st = launch_status(launch_rel_rows(rl, s));
    if (st) return st;
  }
  if (timed && !all)
    for (int k = 0; k < 3; ++k) g_timer.mark(s);  // stages 3-5 not in this call
  }  // KGE_PHASE_ROWS

  fa.row_stats = w.row_stats;
  fa.reg_partial = (reg != 0.f) ? w.reg_partial : nullptr;
  {
    // entity rows [e_begin, e_end) (all of them unless an owner's range) and,
    // unless the caller counts them elsewhere, the relation rows
    const int64_t per = ent_parts / (m->nentity > 0 ? m->nentity : 1);
    fa.reg_a0 = e_begin * per;
    fa.reg_a1 = e_end * per;
    fa.reg_b0 = ent_parts;
    fa.reg_b1 = ent_parts + (reg_relations ? m->nrelation : 0);
  }
  fa.regularization = reg;
  fa.grad_modulus = grad_modulus;
  fa.adam = adam_t((adam && m->model == KGE_PROTATE) ? &adam->modulus : nullptr);
  fa.adamk = ak;
  // the loss finalisation rides in the entity launch's last block when that
  // launch is the whole rest of the step and writes nothing the finalisation
  // reads (no regulariser partials, no pRotatE modulus update)
  const bool fin_wanted = (phases & KGE_PHASE_FINALIZE) && (fa.losses || grad_modulus);
  const bool fin_fused = fin_wanted && all && rel_fused && e_end > e_begin && !fa.reg_partial && !fa.adam.p &&
                         env_int("KGE_FIN_SEPARATE", 0) == 0;

  if (phases & KGE_PHASE_ENTITY) {
  if (sd && use_csr)
    hipStreamWaitEvent(s, sd->csr_done, 0);  // join 1: the entity pass reads the CSR
  if (timed) g_timer.mark(s);

  EntArgs ea;
  memset(&ea, 0, sizeof(ea));
  ea.ent = m->entity_embedding; ea.modulus = m->modulus; ea.E = m->nentity; ea.Le = Le; ea.eg = geo.eg;
  ea.e_begin = e_begin; ea.e_end = e_end;
  ea.c = c; ea.off = w.off; ea.occ = w.occ; ea.Bn = B * n; ea.n = n;
  ea.g = (ra.op == ROW_TRAIN) ? w.g : ra.g_in;
  ea.q = w.q; ea.ent_contrib = w.ent_contrib; ea.reg3 = 3.f * reg; ea.reg_partial = w.reg_partial;
  ea.grad_ent = grad_entity;
  ea.write_grad = write_grad;
  ea.nsl = nsl;
  ea.slice_w = nsl > 0 ? (geo.eg.S + nsl - 1) / nsl : 0;  // (wide: elements per part)
  ea.adam = adam_t(adam ? &adam->entity : nullptr);
  ea.adamk = ak;
  ea.align_sl = (q_slm || wide) ? 0 : entity_slice_align(nsl, geo.eg.S, Le, m->entity_embedding, write_grad ? grad_entity : nullptr, ea.adam);
  ea.q_sl = q_slm ? w.q_sl : nullptr;
  ea.rel = rl;
  ea.B = B;
  ea.rel_blocks = rel_fused ? (m->nrelation + 3) / 4 : 0;
  ea.fin = fa;
  ea.fin_fused = fin_fused ? 1 : 0;
  if (e_end > e_begin) {
    st = launch_status(op.entity(mode, geo.vec, geo.ns, ea, s));
    if (st) return st;
  } else if (rel_fused) {
    // an owner with no entity rows (a trailing rank of a small table) still
    // owes the relation pass the entity launch would have carried
    st = launch_status(launch_rel_rows(rl, s));
    if (st) return st;
  }
  if (timed) g_timer.mark(s);
  }  // KGE_PHASE_ENTITY

  if (!(phases & KGE_PHASE_FINALIZE)) return KGE_OK;
  if (rel_side) {
    hipStreamWaitEvent(s, sd->rel_done, 0);  // join 2: everything the side stream wrote
  } else if (all && !rel_fused) {
    st = launch_status(launch_rel_rows(rl, s));
    if (st) return st;
  }
  if (fin_wanted && !fin_fused) {
    st = launch_status(launch_finalize(fa, s));
    if (st) return st;
  }
  if (timed) g_timer.mark(s);
  return KGE_OK;
}

RowArgs row_args(const kge_model_desc* m, const Geom& geo, const int64_t* pos, const int64_t* neg, int64_t ns,
                 int64_t B, int64_t n, GradWs w, int32_t* err) {
  RowArgs ra;
  memset(&ra, 0, sizeof(ra));
  ra.ent = m->entity_embedding; ra.rel = m->relation_embedding; ra.modulus = m->modulus;
  ra.pos = pos; ra.neg = neg; ra.neg_stride = ns;
  ra.B = B; ra.n = n; ra.E = m->nentity; ra.R = m->nrelation;
  ra.Le = m->entity_dim; ra.Lr = m->relation_dim; ra.eg = geo.eg; ra.c = consts_of(m);
  ra.g_out = w.g; ra.q_out = w.q; ra.dq_out = w.dq; ra.ent_contrib = w.ent_contrib; ra.rel_contrib = w.rel_contrib;
  ra.row_stats = w.row_stats; ra.err = err;
  ra.fuse_epi = 1;  // measured +1 % over the separate k_row_epi launch
  return ra;
}

}  // namespace
}  // namespace kge

using namespace kge;

extern "C" {

const char* kge_version(void) { return "knowledgegraphembedding_amd " KGE_ABI_VERSION " gfx950"; }

const char* kge_status_string(int status) {
  switch (status) {
    case KGE_OK: return "ok";
    case KGE_ERR_MODEL: return "model not supported";
    case KGE_ERR_MODE: return "mode not supported";
    case KGE_ERR_SHAPE: return "entity/relation dims inconsistent with the model";
    case KGE_ERR_ARG: return "invalid argument";
    case KGE_ERR_WORKSPACE: return "workspace too small";
    case KGE_ERR_DIM: return "size outside the kernels' range (negatives per row, queries per call, LDS; wide rows under query shipping)";
    case KGE_ERR_ABI: return "kge_model_desc.struct_size does not match this library (built against another kge_hip.h)";
    default:
      if (status >= KGE_ERR_HIP_BASE) return hipGetErrorString((hipError_t)(status - KGE_ERR_HIP_BASE));
      return "unknown";
  }
}

int kge_score(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg, int64_t batch,
              int64_t nneg, float* out, int32_t* err_flag, void* stream) {
  Geom geo;
  int st = check_model(m, &geo);
  if (st) return st;
  if (mode != KGE_SINGLE && mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH) return KGE_ERR_MODE;
  if (batch == 0 && nneg >= 1) return KGE_OK;  // empty batch: nothing to score (buffers may be empty/NULL)
  if (!pos || !out || !err_flag || batch < 0 || nneg < 1) return KGE_ERR_ARG;
  ScoreArgs a;
  a.ent = m->entity_embedding; a.rel = m->relation_embedding; a.modulus = m->modulus;
  a.pos = pos;
  if (mode == KGE_SINGLE) {
    if (nneg != 1) return KGE_ERR_ARG;
    a.neg = pos + 2;  // 'single' scores (h, r, t) with the tail-batch formulas, t in place of a negative
    a.neg_stride = 3;
  } else {
    if (!neg) return KGE_ERR_ARG;
    a.neg = neg;
    a.neg_stride = nneg;
  }
  a.B = batch; a.n = nneg; a.E = m->nentity; a.R = m->nrelation;
  a.Le = m->entity_dim; a.Lr = m->relation_dim; a.eg = geo.eg; a.c = consts_of(m);
  a.jpw = nneg < 16 ? nneg : 16;
  a.out = out; a.err = err_flag;
  const int64_t units = batch * ((nneg + a.jpw - 1) / a.jpw);
  const int kmode = (mode == KGE_HEAD_BATCH) ? HEAD_BATCH : TAIL_BATCH;
  return launch_status(ops_for(m->model).score(kmode, geo.vec, geo.ns, a, units, as_stream(stream)));
}

size_t kge_backward_workspace_bytes(const kge_model_desc* m, int32_t mode, int64_t batch, int64_t nneg) {
  (void)mode;
  size_t b = 0;
  carve_grad(nullptr, m, batch, nneg, &b);
  return b;
}

int kge_score_backward(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg, int64_t batch,
                       int64_t nneg, const float* grad_scores, float* grad_entity, float* grad_relation,
                       float* grad_modulus, void* workspace, size_t workspace_bytes, int32_t* err_flag,
                       void* stream) {
  Geom geo;
  int st = check_model(m, &geo);
  if (st) return st;
  if (mode != KGE_SINGLE && mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH) return KGE_ERR_MODE;
  if (!pos || !grad_scores || !grad_entity || !grad_relation || !err_flag || batch < 1 || nneg < 1)
    return KGE_ERR_ARG;
  const int64_t* negp = neg;
  int64_t ns = nneg;
  if (mode == KGE_SINGLE) {
    if (nneg != 1) return KGE_ERR_ARG;
    negp = pos + 2;
    ns = 3;
  } else if (!neg) {
    return KGE_ERR_ARG;
  }
  size_t need = 0;
  GradWs w = carve_grad(workspace, m, batch, nneg, &need);
  if (!workspace || workspace_bytes < need) return KGE_ERR_WORKSPACE;
  RowArgs ra = row_args(m, geo, pos, negp, ns, batch, nneg, w, err_flag);
  ra.op = ROW_GIVEN;
  ra.g_in = grad_scores;
  ra.n_lds = 0;
  FinArgs fa;
  memset(&fa, 0, sizeof(fa));
  fa.B = batch;
  fa.uni_weight = 1;
  fa.uni_n = 1.f;
  fa.losses = nullptr;
  const int kmode = (mode == KGE_HEAD_BATCH) ? HEAD_BATCH : TAIL_BATCH;
  return run_grad(m, geo, kmode, pos, negp, ns, batch, nneg, ra, w, grad_entity, grad_relation,
                  m->model == KGE_PROTATE ? grad_modulus : nullptr, 0.f, fa, nullptr, err_flag, as_stream(stream));
}

size_t kge_train_workspace_bytes(const kge_model_desc* m, int64_t batch, int64_t nneg) {
  size_t b = 0;
  carve_grad(nullptr, m, batch, nneg, &b);
  return b;
}

static int train_impl(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg, int64_t batch,
                      int64_t nneg, const float* subsampling_weight, const float* weight_sum, int32_t uni_weight,
                      int64_t uni_batch, int32_t adversarial, float adversarial_temperature, float regularization,
                      const kge_adam_desc* adam, float* grad_entity, float* grad_relation, float* grad_modulus,
                      float* losses_out, void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream,
                      int32_t phases = KGE_PHASE_ALL, int64_t e_begin = 0, int64_t e_end = -1, int xstage = XS_NONE,
                      float* rows_g = nullptr, float* rows_dq = nullptr, float* rows_stats = nullptr,
                      int reg_relations = 1, int64_t csr_lo = 0, int64_t csr_hi = -1) {
  Geom geo;
  int st = check_model(m, &geo);
  if (st) return st;
  if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH) return KGE_ERR_MODE;
  if (xstage == XS_NONE && (!grad_entity || !grad_relation || !losses_out)) return KGE_ERR_ARG;
  const bool csr_only = (xstage == XS_CSR_ONLY);
  const bool from_rows = (xstage == XS_FROM_ROWS || xstage == XS_FROM_ROWS_CSR);
  if (xstage != XS_NONE && !csr_only && (!rows_g || !rows_dq || !rows_stats)) return KGE_ERR_ARG;
  if (from_rows && (!grad_entity || !grad_relation || !losses_out)) return KGE_ERR_ARG;
  if (!pos || !neg || !err_flag || batch < 1 || nneg < 1) return KGE_ERR_ARG;
  if (adam) {
    if (!adam->entity.param || !adam->entity.exp_avg || !adam->entity.exp_avg_sq || !adam->relation.param ||
        !adam->relation.exp_avg || !adam->relation.exp_avg_sq)
      return KGE_ERR_ARG;
    if (adam->entity.param != m->entity_embedding || adam->relation.param != m->relation_embedding)
      return KGE_ERR_ARG;  // the update is in place on the model's own tables
    if (m->model == KGE_PROTATE && adam->modulus.param && adam->modulus.param != m->modulus) return KGE_ERR_ARG;
  }
  if (!uni_weight && !subsampling_weight) return KGE_ERR_ARG;
  if (m->model == KGE_PROTATE && !grad_modulus && xstage != XS_ROWS_ONLY && !csr_only) return KGE_ERR_ARG;
  if (xstage != XS_NONE && !csr_only && !uni_weight && !weight_sum) return KGE_ERR_ARG;  // the global Σw comes from the caller
  size_t need = 0;
  GradWs w = carve_grad(workspace, m, batch, nneg, &need);
  if (!workspace || workspace_bytes < need) return KGE_ERR_WORKSPACE;
  if (xstage != XS_NONE && !csr_only) {  // the exchanged per-row factors live in the caller's (gathered) buffers
    w.g = rows_g;
    w.dq = rows_dq;
    w.row_stats = rows_stats;
  }
  hipStream_t s = as_stream(stream);
  const float* wsum = weight_sum;
  float* wsum_out = nullptr;
  if (!uni_weight && !wsum) {
    wsum_out = w.wsum;  // computed by k_build_q's first block, before k_row reads it
    wsum = w.wsum;
  }
  const int64_t ub = uni_batch > 0 ? uni_batch : batch;
  RowArgs ra = row_args(m, geo, pos, neg, nneg, batch, nneg, w, err_flag);
  ra.op = ROW_TRAIN;
  ra.adversarial = adversarial ? 1 : 0;
  ra.adv_T = adversarial_temperature;
  ra.uni_weight = uni_weight ? 1 : 0;
  ra.uni_inv = 1.f / (float)ub;
  ra.sub_w = subsampling_weight;
  ra.w_sum = wsum;
  ra.wsum_out = wsum_out;
  ra.n_lds = (int)nneg;
  if (nneg > 8192) return KGE_ERR_DIM;
  FinArgs fa;
  memset(&fa, 0, sizeof(fa));
  fa.sub_w = subsampling_weight;
  fa.w_sum = wsum;
  fa.B = batch;
  fa.uni_weight = uni_weight ? 1 : 0;
  fa.uni_n = (float)ub;
  fa.losses = losses_out;
  fa.err = err_flag;
  if (phases < 1 || phases > KGE_PHASE_ALL) return KGE_ERR_ARG;
  if (e_end < 0) e_end = m->nentity;
  if (e_begin < 0 || e_begin > e_end || e_end > m->nentity) return KGE_ERR_ARG;
  return run_grad(m, geo, mode, pos, neg, nneg, batch, nneg, ra, w, grad_entity, grad_relation,
                  m->model == KGE_PROTATE ? grad_modulus : nullptr, regularization, fa, adam, err_flag, s, phases,
                  e_begin, e_end, xstage, reg_relations, csr_lo, csr_hi);
}

int kge_train_rows_slice(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                         int64_t nrows, int64_t nneg, const float* subsampling_weight, const float* weight_sum,
                         int32_t uni_weight, int64_t uni_batch, int32_t adversarial, float adversarial_temperature,
                         float* g_out, float* dq_out, float* stats_out, void* workspace, size_t workspace_bytes,
                         int32_t* err_flag, void* stream) {
  return train_impl(m, mode, pos, neg, nrows, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, adversarial,
                    adversarial_temperature, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr, workspace,
                    workspace_bytes, err_flag, stream, KGE_PHASE_ROWS, 0, -1, XS_ROWS_ONLY, g_out, dq_out, stats_out);
}

int kge_train_step_from_rows(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                             int64_t batch, int64_t nneg, const float* subsampling_weight, const float* weight_sum,
                             int32_t uni_weight, int64_t uni_batch, float regularization, const float* g_in,
                             const float* dq_in, float* stats_inout, const kge_adam_desc* adam, float* grad_entity,
                             float* grad_relation, float* grad_modulus, float* losses_out, void* workspace,
                             size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return train_impl(m, mode, pos, neg, batch, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, 1, 1.f,
                    regularization, adam, grad_entity, grad_relation, grad_modulus, losses_out, workspace,
                    workspace_bytes, err_flag, stream, KGE_PHASE_ALL, 0, -1, XS_FROM_ROWS, const_cast<float*>(g_in),
                    const_cast<float*>(dq_in), stats_inout);
}

int kge_train_step_from_rows_range(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                                   int64_t batch, int64_t nneg, const float* subsampling_weight,
                                   const float* weight_sum, int32_t uni_weight, int64_t uni_batch,
                                   float regularization, const float* g_in, const float* dq_in, float* stats_inout,
                                   const kge_adam_desc* adam, float* grad_entity, float* grad_relation,
                                   float* grad_modulus, float* losses_out, void* workspace, size_t workspace_bytes,
                                   int32_t* err_flag, void* stream, int64_t entity_begin, int64_t entity_end,
                                   int32_t csr_ready, int32_t reg_relations) {
  if (entity_begin < 0 || entity_end < entity_begin || entity_end > (m ? m->nentity : 0)) return KGE_ERR_ARG;
  return train_impl(m, mode, pos, neg, batch, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, 1, 1.f,
                    regularization, adam, grad_entity, grad_relation, grad_modulus, losses_out, workspace,
                    workspace_bytes, err_flag, stream, KGE_PHASE_ALL, entity_begin, entity_end,
                    csr_ready ? XS_FROM_ROWS_CSR : XS_FROM_ROWS, const_cast<float*>(g_in), const_cast<float*>(dq_in),
                    stats_inout, reg_relations ? 1 : 0);
}

int kge_train_step_from_rows_phased(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                                    int64_t batch, int64_t nneg, const float* subsampling_weight,
                                    const float* weight_sum, int32_t uni_weight, int64_t uni_batch,
                                    float regularization, const float* g_in, const float* dq_in, float* stats_inout,
                                    const kge_adam_desc* adam, float* grad_entity, float* grad_relation,
                                    float* grad_modulus, float* losses_out, void* workspace, size_t workspace_bytes,
                                    int32_t* err_flag, void* stream, int32_t phases, int64_t entity_begin,
                                    int64_t entity_end, int32_t csr_ready, int32_t reg_relations) {
  if (phases <= 0 || phases > KGE_PHASE_ALL) return KGE_ERR_ARG;
  if (entity_begin < 0 || entity_end < entity_begin || entity_end > (m ? m->nentity : 0)) return KGE_ERR_ARG;
  return train_impl(m, mode, pos, neg, batch, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, 1, 1.f,
                    regularization, adam, grad_entity, grad_relation, grad_modulus, losses_out, workspace,
                    workspace_bytes, err_flag, stream, phases, entity_begin, entity_end,
                    csr_ready ? XS_FROM_ROWS_CSR : XS_FROM_ROWS, const_cast<float*>(g_in), const_cast<float*>(dq_in),
                    stats_inout, reg_relations ? 1 : 0);
}

int kge_ship_step(const kge_model_desc* m, int32_t mode, const kge_ship_desc* sh, int32_t stage,
                  const kge_adam_desc* adam, float* grad_entity, float* grad_relation, float* grad_modulus,
                  float* losses_out, void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  Geom geo;
  int st = check_model(m, &geo);
  if (st) return st;
  if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH) return KGE_ERR_MODE;
  if (!sh || stage < KGE_SHIP_Q || stage > KGE_SHIP_ENTITY || !err_flag) return KGE_ERR_ARG;
  const int64_t B = sh->batch, n = sh->nneg;
  if (!sh->pos || !sh->neg || B < 1 || n < 1 || n > 8192) return KGE_ERR_ARG;
  if (sh->world < 1 || sh->world > 4096 || sh->rank < 0 || sh->rank >= sh->world) return KGE_ERR_ARG;
  if (sh->own_begin < 0 || sh->own_end < sh->own_begin || sh->own_end > m->nentity) return KGE_ERR_ARG;
  if (!sh->uni_weight && (!sh->subsampling_weight || !sh->weight_sum)) return KGE_ERR_ARG;
  const bool head = (mode == KGE_HEAD_BATCH);
  if (!sh->q || !sh->part || !sh->parts || !sh->scores || !sh->g || !sh->dq || !sh->pstats || !sh->ent_contrib ||
      !sh->rel_contrib || !sh->row_stats || (head && (!sh->qp || !sh->pq)))
    return KGE_ERR_ARG;
  if (stage >= KGE_SHIP_CHAIN && !grad_relation) return KGE_ERR_ARG;
  if (stage == KGE_SHIP_ENTITY && (!grad_entity || !losses_out || (m->model == KGE_PROTATE && !grad_modulus)))
    return KGE_ERR_ARG;
  if (adam && (!adam->entity.param || !adam->entity.exp_avg || !adam->entity.exp_avg_sq ||
               adam->entity.param != m->entity_embedding))
    return KGE_ERR_ARG;
  size_t need = 0;
  GradWs w = carve_grad(workspace, m, B, n, &need);
  if (!workspace || workspace_bytes < need) return KGE_ERR_WORKSPACE;
  hipStream_t s = as_stream(stream);
  const ModelOps& op = ops_for(m->model);
  const int kmode = head ? HEAD_BATCH : TAIL_BATCH;
  const int Le = m->entity_dim, Lr = m->relation_dim;

  RowArgs ra = row_args(m, geo, sh->pos, sh->neg, n, B, n, w, err_flag);
  ra.op = ROW_TRAIN;
  ra.adversarial = sh->adversarial ? 1 : 0;
  ra.adv_T = sh->adversarial_temperature;
  ra.uni_weight = sh->uni_weight ? 1 : 0;
  ra.uni_inv = 1.f / (float)(sh->uni_batch > 0 ? sh->uni_batch : B);
  ra.sub_w = sh->subsampling_weight;
  ra.w_sum = sh->weight_sum;
  ra.q_out = sh->q; ra.dq_out = sh->dq; ra.g_out = sh->g;
  ra.ent_contrib = sh->ent_contrib; ra.rel_contrib = sh->rel_contrib; ra.row_stats = sh->row_stats;
  ra.n_lds = 0; ra.fuse_epi = 0;
  ra.sh.own_lo = sh->own_begin; ra.sh.own_hi = sh->own_end;
  ra.sh.world = sh->world; ra.sh.me = sh->rank;
  ra.sh.q_in = sh->q; ra.sh.qp_in = sh->qp; ra.sh.qp_out = sh->qp;
  ra.sh.part_out = sh->part; ra.sh.parts_in = sh->parts; ra.sh.s_out = sh->scores;
  ra.sh.pq = sh->pq; ra.sh.pstats = sh->pstats;
  Side* sd = side_for_device();

  if (stage == KGE_SHIP_Q) return launch_status(op.row(kmode, geo.vec, geo.ns, 3, ra, 0, s));
  if (stage == KGE_SHIP_ROWS) {
    // the occurrence CSR of the global batch beside the row pass (it needs only the ids)
    CsrArgs ca;
    ca.pos = sh->pos; ca.neg = sh->neg; ca.neg_stride = n;
    ca.B = B; ca.n = n; ca.Bn = B * n; ca.E = m->nentity; ca.R = m->nrelation;
    ca.keys = w.keys; ca.cnt = w.cnt; ca.off = w.off; ca.tmp = w.tmp; ca.occ = w.occ; ca.err = err_flag;
    ca.e_lo = sh->own_begin; ca.e_hi = sh->own_end;  // only this shard's rows are visited by its entity pass
    ca.scan_tmp = w.scan_tmp; ca.scan_tmp_bytes = w.scan_tmp_bytes;
    hipStream_t ss = sd ? sd->s : s;
    if (sd) {
      hipEventRecord(sd->fork, s);
      hipStreamWaitEvent(ss, sd->fork, 0);
    }
    st = launch_status(launch_csr(ca, ss));
    if (st) return st;
    if (sd) hipEventRecord(sd->csr_done, ss);
    const size_t lds = sizeof(float) * (2 * 64 * (size_t)geo.ns * geo.vec + (size_t)vb_floats(Le) + (size_t)ra.n_lds + 32);
    if (lds > 64 * 1024) return KGE_ERR_DIM;
    return launch_status(op.row(kmode, geo.vec, geo.ns, 4, ra, lds, s));
  }
  if (stage == KGE_SHIP_MERGE) return launch_status(op.row(kmode, geo.vec, geo.ns, 5, ra, 0, s));

  const int nsl = entity_slices(geo, B, Le);
  const int64_t ent_parts = m->nentity * (int64_t)(nsl > 0 ? nsl : 1);
  const float reg = sh->regularization;
  if (stage == KGE_SHIP_CHAIN) {
    st = launch_status(op.row(kmode, geo.vec, geo.ns, 6, ra, 0, s));
    if (st) return st;
    if (sd) hipStreamWaitEvent(s, sd->csr_done, 0);  // the relation pass reads the CSR
    RelArgs rl;
    memset(&rl, 0, sizeof(rl));
    rl.rel = m->relation_embedding; rl.R = m->nrelation; rl.E = m->nentity; rl.B = B; rl.Bn = B * n; rl.Lr = Lr;
    rl.off = w.off; rl.occ = w.occ; rl.rel_contrib = sh->rel_contrib;
    rl.reg3 = (sh->rank == 0) ? 3.f * reg : 0.f;  // the relation table is replicated: its regulariser once
    rl.reg_partial = w.reg_partial + ent_parts; rl.grad_rel = grad_relation;
    rl.write_grad = 1;
    return launch_status(launch_rel_rows(rl, s));
  }

  // KGE_SHIP_ENTITY
  AdamK ak;
  ak.b1 = adam ? adam->beta1 : 0.f;
  ak.b2 = adam ? adam->beta2 : 0.f;
  ak.eps = adam ? adam->eps : 0.f;
  auto adam_t = [&](const kge_adam_tensor* t) {
    AdamT o;
    o.p = (adam && t && t->param) ? t->param : nullptr;
    o.m = o.p ? t->exp_avg : nullptr;
    o.v = o.p ? t->exp_avg_sq : nullptr;
    o.step_size = o.p ? t->step_size : 0.f;
    o.bc2s = o.p ? t->bias_correction2_sqrt : 1.f;
    return o;
  };
  EntArgs ea;
  memset(&ea, 0, sizeof(ea));
  ea.ent = m->entity_embedding; ea.modulus = m->modulus; ea.E = m->nentity; ea.Le = Le; ea.eg = geo.eg;
  ea.e_begin = sh->own_begin; ea.e_end = sh->own_end;
  ea.c = consts_of(m); ea.off = w.off; ea.occ = w.occ; ea.Bn = B * n; ea.n = n;
  ea.g = sh->g; ea.q = sh->q; ea.ent_contrib = sh->ent_contrib; ea.reg3 = 3.f * reg; ea.reg_partial = w.reg_partial;
  ea.grad_ent = grad_entity;
  ea.write_grad = (!adam || adam->write_grad) ? 1 : 0;
  ea.nsl = nsl;
  ea.slice_w = nsl > 0 ? (geo.eg.S + nsl - 1) / nsl : 0;  // (wide: elements per part)
  ea.adam = adam_t(adam ? &adam->entity : nullptr);
  ea.adamk = ak;
  ea.B = B;
  ea.rel_blocks = 0;
  if (sh->own_end > sh->own_begin) {
    st = launch_status(op.entity(kmode, geo.vec, geo.ns, ea, s));
    if (st) return st;
  }
  FinArgs fa;
  memset(&fa, 0, sizeof(fa));
  fa.row_stats = sh->row_stats;
  fa.sub_w = sh->subsampling_weight;
  fa.w_sum = sh->weight_sum;
  fa.B = B;
  fa.uni_weight = sh->uni_weight ? 1 : 0;
  fa.uni_n = (float)(sh->uni_batch > 0 ? sh->uni_batch : B);
  fa.losses = losses_out;
  fa.err = err_flag;
  fa.reg_partial = (reg != 0.f) ? w.reg_partial : nullptr;
  const int64_t per = nsl > 0 ? nsl : 1;
  fa.reg_a0 = sh->own_begin * per;
  fa.reg_a1 = sh->own_end * per;
  fa.reg_b0 = ent_parts;
  fa.reg_b1 = ent_parts + (sh->rank == 0 ? m->nrelation : 0);
  fa.regularization = reg;
  fa.grad_modulus = (m->model == KGE_PROTATE) ? grad_modulus : nullptr;
  fa.adam = adam_t((adam && m->model == KGE_PROTATE) ? &adam->modulus : nullptr);
  fa.adamk = ak;
  return launch_status(launch_finalize(fa, s));
}

int kge_train_csr(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg, int64_t batch,
                  int64_t nneg, void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return train_impl(m, mode, pos, neg, batch, nneg, nullptr, nullptr, 1, 0, 1, 1.f, 0.f, nullptr, nullptr, nullptr,
                    nullptr, nullptr, workspace, workspace_bytes, err_flag, stream, KGE_PHASE_ALL, 0, -1, XS_CSR_ONLY);
}

int kge_train_csr_range(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                        int64_t batch, int64_t nneg, int64_t entity_begin, int64_t entity_end, void* workspace,
                        size_t workspace_bytes, int32_t* err_flag, void* stream) {
  if (!m || entity_begin < 0 || entity_end < entity_begin || entity_end > m->nentity) return KGE_ERR_ARG;
  return train_impl(m, mode, pos, neg, batch, nneg, nullptr, nullptr, 1, 0, 1, 1.f, 0.f, nullptr, nullptr, nullptr,
                    nullptr, nullptr, workspace, workspace_bytes, err_flag, stream, KGE_PHASE_ALL, 0, -1, XS_CSR_ONLY,
                    nullptr, nullptr, nullptr, 1, entity_begin, entity_end);
}

int kge_train_step_from_rows_csr(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                                 int64_t batch, int64_t nneg, const float* subsampling_weight, const float* weight_sum,
                                 int32_t uni_weight, int64_t uni_batch, float regularization, const float* g_in,
                                 const float* dq_in, float* stats_inout, const kge_adam_desc* adam, float* grad_entity,
                                 float* grad_relation, float* grad_modulus, float* losses_out, void* workspace,
                                 size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return train_impl(m, mode, pos, neg, batch, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, 1, 1.f,
                    regularization, adam, grad_entity, grad_relation, grad_modulus, losses_out, workspace,
                    workspace_bytes, err_flag, stream, KGE_PHASE_ALL, 0, -1, XS_FROM_ROWS_CSR, const_cast<float*>(g_in),
                    const_cast<float*>(dq_in), stats_inout);
}

int kge_train_step_grads_phased(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                                int64_t batch, int64_t nneg, const float* subsampling_weight,
                                const float* weight_sum, int32_t uni_weight, int64_t uni_batch, int32_t adversarial,
                                float adversarial_temperature, float regularization, float* grad_entity,
                                float* grad_relation, float* grad_modulus, float* losses_out, void* workspace,
                                size_t workspace_bytes, int32_t* err_flag, void* stream, int32_t phases,
                                int64_t entity_begin, int64_t entity_end) {
  return train_impl(m, mode, pos, neg, batch, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, adversarial,
                    adversarial_temperature, regularization, nullptr, grad_entity, grad_relation, grad_modulus,
                    losses_out, workspace, workspace_bytes, err_flag, stream, phases, entity_begin, entity_end);
}

int kge_train_step_grads(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg,
                         int64_t batch, int64_t nneg, const float* subsampling_weight, const float* weight_sum,
                         int32_t uni_weight, int64_t uni_batch, int32_t adversarial,
                         float adversarial_temperature, float regularization, float* grad_entity,
                         float* grad_relation, float* grad_modulus, float* losses_out, void* workspace,
                         size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return train_impl(m, mode, pos, neg, batch, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, adversarial,
                    adversarial_temperature, regularization, nullptr, grad_entity, grad_relation, grad_modulus,
                    losses_out, workspace, workspace_bytes, err_flag, stream);
}

int kge_train_step(const kge_model_desc* m, int32_t mode, const int64_t* pos, const int64_t* neg, int64_t batch,
                   int64_t nneg, const float* subsampling_weight, const float* weight_sum, int32_t uni_weight,
                   int64_t uni_batch, int32_t adversarial, float adversarial_temperature, float regularization,
                   const kge_adam_desc* adam, float* grad_entity, float* grad_relation, float* grad_modulus,
                   float* losses_out, void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  if (!adam) return KGE_ERR_ARG;
  return train_impl(m, mode, pos, neg, batch, nneg, subsampling_weight, weight_sum, uni_weight, uni_batch, adversarial,
                    adversarial_temperature, regularization, adam, grad_entity, grad_relation, grad_modulus,
                    losses_out, workspace, workspace_bytes, err_flag, stream);
}

int kge_weight_sum(const float* w, int64_t n, float* out, void* stream) {
  if (!w || !out || n < 0) return KGE_ERR_ARG;
  return launch_status(launch_weight_sum(w, n, out, as_stream(stream)));
}

int kge_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t numel, float beta1,
                  float beta2, float eps, float step_size, float bias_correction2_sqrt, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || numel < 0) return KGE_ERR_ARG;
  if (numel == 0) return KGE_OK;
  if (!aligned16(param) || !aligned16(grad) || !aligned16(exp_avg) || !aligned16(exp_avg_sq)) return KGE_ERR_ARG;
  return launch_status(launch_adam(param, grad, exp_avg, exp_avg_sq, numel, beta1, beta2, eps, step_size,
                                   bias_correction2_sqrt, as_stream(stream)));
}

}  // extern "C"

namespace kge {
namespace {
struct RankWs {
  int64_t* tag;  // [8] what the table buffers below hold (k_rank_tag), then [3] the pRotatE list tag
  float *q, *qref, *s_true, *sref_true, *sref_hi, *delta, *stats;
  int64_t* true_id;
  int32_t *gt, *eq, *gtx, *eqx, *ucnt, *done, *ulist;
  uint32_t* bits;
  uint16_t *qs, *es;  // split-bf16 operands (DistMult / ComplEx)
  float *qph, *eph;   // pRotatE's phase tables for the register tile ([rows][K][2])
};
RankWs carve_rank(void* ws, const kge_model_desc* m, int64_t nq, size_t* bytes) {
  Carver c(ws);
  RankWs w;
  // the entity table's own buffers first, at offsets independent of nq, so a
  // later call on the same workspace can reuse them (KGE_RANK_REUSE_TABLE)
  w.tag = c.take<int64_t>(12);
  w.stats = c.take<float>(TS_NSTAT * (1 + TS_BLOCKS));  // [the TS_NSTAT maxima, per-block partials]
  // split-bf16 operands: only where the split tile can run (rank_path's x_ok)
  const bool xs = rank_path(m, RP_MFMA) == RP_MFMA;
  w.es = c.take<uint16_t>(xs ? xsplit_elems(m->nentity, m->entity_dim) : 0);
  // pRotatE's phase tables: only where its register tile can run
  const bool ph = m->model == KGE_PROTATE && rank_path(m, RP_TILE) == RP_TILE;
  w.eph = c.take<float>(ph ? 2 * m->nentity * (int64_t)m->entity_dim : 0);
  w.qs = c.take<uint16_t>(xs ? xsplit_elems(nq, m->entity_dim) : 0);
  w.qph = c.take<float>(ph ? 2 * nq * (int64_t)m->entity_dim : 0);
  w.q = c.take<float>(nq * (int64_t)m->entity_dim);
  w.qref = c.take<float>(nq * (int64_t)m->entity_dim);
  w.s_true = c.take<float>(nq);
  w.sref_true = c.take<float>(nq);
  w.sref_hi = c.take<float>(nq);
  w.delta = c.take<float>(nq);
  w.true_id = c.take<int64_t>(nq);
  w.gt = c.take<int32_t>(6 * nq);  // gt, eq, gtx, eqx, ucnt, done (zeroed by k_rank_prep)
  w.eq = w.gt ? w.gt + nq : nullptr;
  w.gtx = w.gt ? w.gt + 2 * nq : nullptr;
  w.eqx = w.gt ? w.gt + 3 * nq : nullptr;
  w.ucnt = w.gt ? w.gt + 4 * nq : nullptr;
  w.done = w.gt ? w.gt + 5 * nq : nullptr;
  w.ulist = c.take<int32_t>(nq * (int64_t)RANK_CAP);
  w.bits = c.take<uint32_t>(nq * ((m->nentity + 31) / 32));
  *bytes = c.off + 256;
  return w;
}
}  // namespace
}  // namespace kge

extern "C" {

size_t kge_rank_workspace_bytes(const kge_model_desc* m, int64_t nq) {
  size_t b = 0;
  carve_rank(nullptr, m, nq, &b);
  return b;
}

}  // extern "C"

namespace kge {
namespace {
// Stages of one filtered-ranking call (kge_rank_filtered_ex, and pRotatE's
// three-call form with the caller's sin): RS_LIST runs everything up to the
// fast pass's near-tie lists and writes only listed_out; RS_ARGS writes the
// pRotatE phase sums of the listed items; RS_FINISH refines them with the
// caller's sin values, rescans overflowed windows and writes the ranks.
enum { RS_ALL = 0, RS_LIST = 1, RS_ARGS = 2, RS_FINISH = 3 };

int rank_impl(const kge_model_desc* m, int32_t mode, const int64_t* queries, int64_t nq, const int64_t* filt_off,
              const int64_t* filt_ids, int64_t* ranks_out, int32_t* ties_out, int32_t* listed_out, int32_t path,
              void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream, int stage,
              const int64_t* item_off, const float* sins, float* args, const int64_t* filt_off2 = nullptr,
              const int64_t* filt_ids2 = nullptr, int both = 0) {
  Geom geo;
  int st = check_model(m, &geo);
  if (st) return st;
  // both: head-batch then tail-batch of the same queries in one pass (kge_rank_filtered_both);
  // per-query arrays hold 2·nq entries, the head direction's first
  if (!both && mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH) return KGE_ERR_MODE;
  if (!err_flag || nq < 0) return KGE_ERR_ARG;
  if (both && (stage != RS_ALL || !filt_off2)) return KGE_ERR_ARG;
  if (stage == RS_ALL || stage == RS_LIST) {
    if (!queries || !filt_off) return KGE_ERR_ARG;
  }
  if ((stage == RS_ALL || stage == RS_FINISH) && !ranks_out) return KGE_ERR_ARG;
  if (stage == RS_LIST && !listed_out) return KGE_ERR_ARG;
  if (stage == RS_ARGS && (!item_off || !args)) return KGE_ERR_ARG;
  if (stage == RS_FINISH && (!item_off || !sins)) return KGE_ERR_ARG;
  if (stage != RS_ALL && m->model != KGE_PROTATE) return KGE_ERR_MODEL;
  // KGE_RANK_REUSE_TABLE: the workspace already holds this entity table's
  // statistics and split operands from the previous call (the other direction)
  const bool reuse = (path & KGE_RANK_REUSE_TABLE) != 0;
  const bool ftab = (path & KGE_RANK_FILTER_TABLE) != 0;  // filt_off / filt_ids: the whole filter index
  path &= ~(KGE_RANK_REUSE_TABLE | KGE_RANK_STAGE_LIST | KGE_RANK_FILTER_TABLE);
  if (path < RP_AUTO || path > RP_MFMA32) return KGE_ERR_ARG;
  if (nq == 0) return KGE_OK;
  if (nq > 65535) return KGE_ERR_DIM;  // the bitmap launch puts queries on grid.y
  const int rp = rank_path(m, path);
  if (rp < 0) return KGE_ERR_ARG;  // the requested fast pass cannot take these rows
  // RotatE's reference cos | sin table (read with the row's slot geometry)
  const float* trig = (m->model == KGE_ROTATE) ? m->relation_trig : nullptr;
  if (trig && geo.vec == 4 && !aligned16(trig)) return KGE_ERR_ARG;
  const int ndir = both ? 2 : 1;
  const int64_t nqt = ndir * nq;  // queries in the workspace
  const int modes[2] = {both ? (int)KGE_HEAD_BATCH : (int)mode, (int)KGE_TAIL_BATCH};
  const int64_t* const foff[2] = {filt_off, filt_off2};
  const int64_t* const fids[2] = {filt_ids, filt_ids2};
  size_t need = 0;
  RankWs w = carve_rank(workspace, m, nqt, &need);
  if (!workspace || workspace_bytes < need) return KGE_ERR_WORKSPACE;
  hipStream_t s = as_stream(stream);
  // (gt, eq, gtx, eqx, ucnt are zeroed by k_rank_prep: RankArgs.zero_counts)
  const ModelOps& ops = ops_for(m->model);
  const bool cplx = (m->model == KGE_ROTATE || m->model == KGE_COMPLEX);
  const int K = cplx ? m->entity_dim / 2 : m->entity_dim;
  const int64_t Le = m->entity_dim, W = (m->nentity + 31) / 32;
  RankWin win;
  win.delta = w.delta; win.ucnt = w.ucnt; win.ulist = w.ulist; win.cap = RANK_CAP;
  // the per-query arrays of direction d start o = d·nq entries in
  auto win_at = [&](int64_t o) {
    RankWin x = win;
    x.delta += o; x.ucnt += o; x.ulist += o * RANK_CAP;
    return x;
  };

  // 1. q, true ids (and, for the wave scan, s_true)
  RankArgs a;
  memset(&a, 0, sizeof(a));
  a.ent = m->entity_embedding; a.rel = m->relation_embedding; a.modulus = m->modulus;
  a.queries = queries; a.nq = nq; a.E = m->nentity; a.R = m->nrelation;
  a.Le = m->entity_dim; a.Lr = m->relation_dim; a.eg = geo.eg; a.c = consts_of(m);
  a.filt_off = filt_off; a.filt_ids = filt_ids;
  a.cpw = 64;
  a.q = w.q; a.s_true = w.s_true; a.true_id = w.true_id; a.gt = w.gt;
  a.fbits = w.bits; a.W = W; a.win = win; a.err = err_flag;
  a.prep_only = 1;
  a.zero_counts = 1;
  a.cstride = nqt;
  a.trig = trig;
  auto rank_at = [&](int d) {
    RankArgs x = a;
    const int64_t o = d * nq;
    x.q += o * Le; x.s_true += o; x.true_id += o; x.gt += o; x.fbits += o * W; x.win = win_at(o);
    x.filt_off = foff[d]; x.filt_ids = fids[d];
    return x;
  };
  // the refinement's arguments (stages 4 and 6)
  RefArgs ra;
  memset(&ra, 0, sizeof(ra));
  ra.ent = m->entity_embedding; ra.rel = m->relation_embedding; ra.modulus = m->modulus;
  ra.queries = queries; ra.nq = nq; ra.E = m->nentity; ra.R = m->nrelation;
  ra.Le = m->entity_dim; ra.Lr = m->relation_dim; ra.K = K; ra.c = a.c;
  ra.q = w.q; ra.qref = w.qref; ra.true_id = w.true_id; ra.s_true = w.s_true; ra.sref_true = w.sref_true;
  ra.s_true_w = w.s_true;
  ra.delta = w.delta; ra.stats = w.stats;
  ra.exact_fast = (m->model == KGE_TRANSE && rp == RP_TILE) ? 1 : 0;
  ra.ucnt = w.ucnt; ra.ulist = w.ulist; ra.cap = RANK_CAP;
  ra.fbits = w.bits; ra.W = a.W; ra.gt = w.gt; ra.eq = w.eq; ra.gtx = w.gtx; ra.eqx = w.eqx; ra.err = err_flag;
  ra.trig = trig;
  ra.item_off = item_off; ra.sins = sins; ra.args = args;
  ra.lib_sin = (stage != RS_ALL) ? 1 : 0;
  ra.sref_hi = w.sref_hi; ra.done = w.done;
  // the list tag of pRotatE's three-call form: the later stages must name the
  // list stage's mode, nq and table (a reused or switched
  // workspace gave wrong ranks with no error)
  const int64_t ltag_v[3] = {(int64_t)0x4B47454C00000000ll | (int64_t)mode, nq,
                             (int64_t)(uintptr_t)m->entity_embedding};
  ra.ltag = w.tag ? w.tag + 8 : nullptr;
  for (int k = 0; k < 3; ++k) ra.ltag_v[k] = ltag_v[k];
  // the split-bf16 tile's arithmetic error in units of u·‖q‖·max‖e‖ (kge_rank_mfma.hip): the
  // final add 1.2, the slab's three chained MFMAs 97.6, the running sum 1.02·nslab; the
  // split's own error is added per query from the pieces' norms (k_rank_window)
  const int64_t xns = xsplit_nslab(m->entity_dim);
  ra.fast_u = (rp != RP_MFMA) ? 0.f : (float)(98.8 + 1.02 * xns);
  // a refinement stage: both directions' queries in one launch when both
  // (each block wholly in one direction, kge_kernels.inc ref_dir)
  auto ref_stage = [&](int stage_) -> int { return launch_status(ops.rank_ref(both ? BOTH_DIRS : mode, stage_, ra, s)); };
  // one launch per direction of a mode-dependent stage (one direction unless both)
  auto per_dir = [&](auto&& launch) -> int {
    for (int d = 0; d < ndir; ++d) {
      const int r = launch(d, modes[d]);
      if (r) return r;
    }
    return KGE_OK;
  };
  if (stage == RS_ARGS) return launch_status(ops.rank_ref(mode, 3, ra, s));
  EmitArgs ea;
  ea.gt = w.gt; ea.eq = w.eq; ea.gtx = w.gtx; ea.eqx = w.eqx; ea.ucnt = w.ucnt; ea.true_id = w.true_id;
  ea.nq = nqt; ea.cap = RANK_CAP; ea.ranks = ranks_out; ea.ties = ties_out; ea.listed = listed_out;
  ea.ltag = nullptr;
  for (int k = 0; k < 3; ++k) ea.ltag_v[k] = ltag_v[k];

  if (stage != RS_FINISH) {
    g_rank_timer.mark(s, 0, ndir);  // (rank timer) 0: the call starts
    // the entity table's work (tag, statistics, split or phase table) depends
    // on the table alone.  KGE_RANK_SIDE=1 (diagnostic, same bits) runs it on
    // the side stream beside the queries' q / bitmap / split (forked here,
    // joined before the windows read the statistics): measured 1-2 % SLOWER
    // than one stream (a ~130 µs dispatch gap before the counting tile after
    // the cross-stream join; profiles/r06/rank), so the default is the
    // caller's stream, the table's work queued first
    Side* rsd = env_int("KGE_RANK_SIDE", 0) != 0 ? side_for_device() : nullptr;
    hipStream_t ts = rsd ? rsd->s : s;
    if (rsd) hipEventRecord(rsd->rk_fork, s);
    // the table's statistics and split operands: reused only where the tag
    // says this workspace already holds them for this table (k_rank_tag)
    const bool need_stats = (m->model == KGE_DISTMULT || m->model == KGE_COMPLEX || m->model == KGE_PROTATE);
    // the derived table: split-bf16 operands (kind 1) or pRotatE's phase table
    // (kind 2, tagged with its divisor's bits)
    const bool prot_tile = m->model == KGE_PROTATE && rp == RP_TILE;
    const float kappa = a.c.kappa_p;
    int64_t kbits = 0;
    memcpy(&kbits, &kappa, sizeof(kappa));
    if (rsd) hipStreamWaitEvent(ts, rsd->rk_fork, 0);
    st = launch_status(launch_rank_tag(w.tag, m->entity_embedding, m->nentity, m->entity_dim, reuse ? 1 : 0,
                                       need_stats ? 1 : 0, rp == RP_MFMA ? 1 : (prot_tile ? 2 : 0),
                                       prot_tile ? kbits : 0, ts));
    if (st) return st;
    if (rp == RP_MFMA && need_stats) {  // (DistMult, ComplEx) one read of the table for both
      st = launch_status(launch_split_stats(m->entity_embedding, m->nentity, m->entity_dim, w.es, w.stats, ts,
                                            w.tag + 5, w.tag + 6));
      if (st) return st;
    } else {
      if (need_stats) {
        st = launch_status(launch_table_stats(m->entity_embedding, m->nentity, m->entity_dim, w.stats, ts, w.tag + 5));
        if (st) return st;
      }
      if (rp == RP_MFMA) {
        st = launch_status(launch_split_bf16(m->entity_embedding, m->nentity, m->entity_dim, w.es, ts, w.tag + 6));
        if (st) return st;
      }
    }
    if (prot_tile) {
      st = launch_status(launch_prot_phase(m->entity_embedding, m->nentity, K, kappa, 1, w.eph, ts, w.tag + 6));
      if (st) return st;
    }
    if (rsd) hipEventRecord(rsd->rk_join, ts);
    if (both && geo.ns != 0) {  // both directions' q in one launch (rows ≤ 2048 floats)
      RankArgs x = a;
      x.both_dirs = 1;
      st = launch_status(ops.rank(KGE_HEAD_BATCH, geo.vec, geo.ns, x, s));
    } else {
      st = per_dir([&](int d, int md) { return launch_status(ops.rank(md, geo.vec, geo.ns, rank_at(d), s)); });
    }
    if (st) return st;
    // 2. excluded candidates (filtered ids + the true id) as a bitmap (both
    // directions in one launch where the row fits LDS)
    st = both ? launch_filter_bits_both(queries, ftab ? 1 : 0, foff[0], fids[0], foff[1], fids[1], w.true_id, nq,
                                        m->nentity, m->nrelation, w.bits, err_flag, s)
              : -1;
    if (st > 0) return launch_status(st);
    if (st < 0) st = per_dir([&](int d, int md) {
      const int64_t o = d * nq;
      if (ftab)
        return launch_status(launch_filter_bits_tab(queries, md == KGE_HEAD_BATCH ? 1 : 0, foff[d], fids[d],
                                                    w.true_id + o, nq, m->nentity, m->nrelation, w.bits + o * W,
                                                    err_flag, s));
      return launch_status(launch_filter_bits(foff[d], fids[d], w.true_id + o, nq, m->nentity, w.bits + o * W,
                                              err_flag, s));
    });
    if (st) return st;
    // 3. the fast pass's own s_true (same instruction sequence as its candidates)
    TileArgs ta;
    ta.q = w.q; ta.ent = m->entity_embedding; ta.modulus = m->modulus;
    ta.nq = nq; ta.E = m->nentity; ta.Le = m->entity_dim; ta.K = K;
    ta.c = a.c; ta.true_id = w.true_id; ta.s_true = w.s_true;
    ta.fbits = w.bits; ta.W = a.W; ta.gt = w.gt; ta.win = win;
    ta.qph = w.qph; ta.eph = w.eph;
    auto tile_at = [&](int d) {
      TileArgs x = ta;
      const int64_t o = d * nq;
      x.q += o * Le; x.true_id += o; x.s_true += o; x.fbits += o * W; x.gt += o; x.win = win_at(o);
      if (x.qph) x.qph += o * 2 * (int64_t)K;
      return x;
    };
    if (prot_tile) {
      st = launch_status(launch_prot_phase(w.q, nqt, K, 0.f, 0, w.qph, s));
      if (st) return st;
    }
    // s_true in the reference's order after the window (k_rank_true_ref):
    // the split-bf16 path (instead of its gather pass), RotatE and pRotatE on
    // the register tile (after its gather pass, whose fast s_true sizes the
    // window's S; pRotatE: a point of the reference score's interval, the
    // window widened by its width); the window then covers the candidate's
    // error only
    const bool true_ref = rp == RP_MFMA || (rp == RP_TILE && (m->model == KGE_ROTATE || prot_tile));
    if (rp == RP_MFMA) {
      // (q of both directions split in one launch: the tile is mode-independent)
      st = launch_status(launch_split_bf16(w.q, nqt, m->entity_dim, w.qs, s));
      if (rsd) hipStreamWaitEvent(s, rsd->rk_join, 0);  // join: everything below reads the table's work
      if (!st && !true_ref)
        st = launch_status(launch_rank_mfma_x(1, w.qs, w.es, nqt, m->nentity, m->entity_dim, w.true_id, w.s_true,
                                              w.bits, w.gt, win, s));
    } else {
      if (rsd) hipStreamWaitEvent(s, rsd->rk_join, 0);  // join: everything below reads the table's work
      if (rp == RP_MFMA32)
        st = launch_status(launch_rank_mfma(1, w.q, m->entity_embedding, nqt, m->nentity, m->entity_dim, w.true_id,
                                            w.s_true, w.bits, w.gt, win, s));
      else if (rp == RP_TILE)
        st = per_dir([&](int d, int md) { return launch_status(ops.rank_tile(md, 1, tile_at(d), s)); });
    }
    if (st) return st;
    // 4. near-tie windows and the reference-order q
    ra.true_exact = true_ref ? 1 : 0;
    st = ref_stage(0);
    if (st) return st;
    if (true_ref) {
      st = ref_stage(4);
      if (st) return st;
    }
    // 5. fast counting pass: clear cases counted, near-ties listed (the MFMA
    // tiles take both directions' queries in one launch)
    g_rank_timer.mark(s, 1);  // (rank timer) 1: fast pass begins
    if (rp == RP_MFMA) {
      st = launch_status(launch_rank_mfma_x(0, w.qs, w.es, nqt, m->nentity, m->entity_dim, w.true_id, w.s_true,
                                            w.bits, w.gt, win, s));
    } else if (rp == RP_MFMA32) {
      st = launch_status(launch_rank_mfma(0, w.q, m->entity_embedding, nqt, m->nentity, m->entity_dim, w.true_id,
                                          w.s_true, w.bits, w.gt, win, s));
    } else if (rp == RP_TILE) {
      st = per_dir([&](int d, int md) { return launch_status(ops.rank_tile(md, 0, tile_at(d), s)); });
    } else {
      st = per_dir([&](int d, int md) {
        RankArgs x = rank_at(d);
        x.prep_only = 0;
        x.zero_counts = 0;
        return launch_status(ops.rank(md, geo.vec, geo.ns, x, s));
      });
    }
    if (st) return st;
    g_rank_timer.mark(s, 2);  // (rank timer) 2: fast pass ends
    if (stage == RS_LIST) {  // the lists stay in the workspace for RS_ARGS / RS_FINISH
      // pRotatE: every listed candidate's score as an interval under any
      // library sin within one ulp, in the reference's order; those whose
      // interval clears the true score's are decided now, only the rest go to
      // the caller's sin.  Overflowed windows: the same over every candidate
      // (k_rank_exact_iv).  KGE_RANK_SIN_SCREEN=0 (diagnostic): decide nothing.
      RefArgs rs = ra;
      rs.screen = 1;
      rs.decide = env_int("KGE_RANK_SIN_SCREEN", 1) != 0 ? 1 : 0;
      rs.ucnt_w = w.ucnt;
      rs.ulist_w = w.ulist;
      st = launch_status(ops.rank_ref(mode, 1, rs, s));
      if (st) return st;
      st = launch_status(ops.rank_ref(mode, 5, rs, s));
      if (st) return st;
      ea.ranks = nullptr;
      ea.ties = nullptr;
      ea.ltag = w.tag + 8;
      return launch_status(launch_rank_emit(ea, s));
    }
  }
  // 6. refinement in the reference's operation order; exact rescan on overflow
  // (RS_FINISH: overflowed pRotatE windows were ranked by the list stage)
  st = ref_stage(1);
  if (st) return st;
  if (stage != RS_FINISH) {
    st = ref_stage(2);
    if (st) return st;
  }
  st = launch_status(launch_rank_emit(ea, s));
  if (!st) g_rank_timer.mark(s, 3);  // (rank timer) 3: ranks written (the last of a call's marks counts)
  return st;
}
}  // namespace
}  // namespace kge

extern "C" {

int kge_rank_filtered_ex(const kge_model_desc* m, int32_t mode, const int64_t* queries, int64_t nq,
                         const int64_t* filt_off, const int64_t* filt_ids, int64_t* ranks_out, int32_t* ties_out,
                         int32_t* listed_out, int32_t path, void* workspace, size_t workspace_bytes,
                         int32_t* err_flag, void* stream) {
  const int stage = (path & KGE_RANK_STAGE_LIST) ? RS_LIST : RS_ALL;
  return rank_impl(m, mode, queries, nq, filt_off, filt_ids, ranks_out, ties_out, listed_out, path, workspace,
                   workspace_bytes, err_flag, stream, stage, nullptr, nullptr, nullptr);
}

int kge_rank_filtered_both(const kge_model_desc* m, const int64_t* queries, int64_t nq,
                           const int64_t* filt_off_head, const int64_t* filt_ids_head, const int64_t* filt_off_tail,
                           const int64_t* filt_ids_tail, int64_t* ranks_out, int32_t* ties_out, int32_t* listed_out,
                           int32_t path, void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  if (path & KGE_RANK_STAGE_LIST) return KGE_ERR_ARG;  // pRotatE's three-call form is per direction
  return rank_impl(m, KGE_HEAD_BATCH, queries, nq, filt_off_head, filt_ids_head, ranks_out, ties_out, listed_out,
                   path, workspace, workspace_bytes, err_flag, stream, RS_ALL, nullptr, nullptr, nullptr,
                   filt_off_tail, filt_ids_tail, 1);
}

int kge_selftest_sin(float range, int32_t* max_dist_out, void* stream) {
  if (!max_dist_out) return KGE_ERR_ARG;
  return launch_status(launch_selftest_sin(range, max_dist_out, as_stream(stream)));
}

int kge_rank_sin_args(const kge_model_desc* m, int32_t mode, int64_t nq, const int64_t* item_off, float* args_out,
                      void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return rank_impl(m, mode, nullptr, nq, nullptr, nullptr, nullptr, nullptr, nullptr, RP_AUTO, workspace,
                   workspace_bytes, err_flag, stream, RS_ARGS, item_off, nullptr, args_out);
}

int kge_rank_finish_sin(const kge_model_desc* m, int32_t mode, int64_t nq, const int64_t* item_off,
                        const float* sin_values, int64_t* ranks_out, int32_t* ties_out, int32_t* listed_out,
                        void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return rank_impl(m, mode, nullptr, nq, nullptr, nullptr, ranks_out, ties_out, listed_out, RP_AUTO, workspace,
                   workspace_bytes, err_flag, stream, RS_FINISH, item_off, sin_values, nullptr);
}

int kge_rank_filtered(const kge_model_desc* m, int32_t mode, const int64_t* queries, int64_t nq,
                      const int64_t* filt_off, const int64_t* filt_ids, int64_t* ranks_out, int32_t* ties_out,
                      void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream) {
  return kge_rank_filtered_ex(m, mode, queries, nq, filt_off, filt_ids, ranks_out, ties_out, nullptr, RP_AUTO,
                              workspace, workspace_bytes, err_flag, stream);
}

int kge_stage_timer(int32_t command, float* stage_ms_out, int32_t n_out) {
  constexpr int NS_ = KGE_TIMER_STAGES + 1;
  if (command == 0 || command == 1) {
    g_timer.on = (command == 1);
    g_timer.used = 0;
    g_timer.seen = 0;
    g_timer.period = (command == 1 && n_out > 0) ? n_out : 1;
    if (command == 0) {
      g_rank_timer.on = false;
      g_rank_timer.used = 0;
    }
    return KGE_OK;
  }
  if (command == 4) {  // ranking calls: enable and reset
    g_rank_timer.on = true;
    g_rank_timer.used = 0;
    return KGE_OK;
  }
  if (command == 5) {  // ranking calls: summed stage times + the number of directions ranked
    constexpr int NR = KGE_RANK_TIMER_STAGES + 1;
    if (!stage_ms_out || n_out < NR) return KGE_ERR_ARG;
    for (int k = 0; k < NR; ++k) stage_ms_out[k] = 0.f;
    const RankTimer& t = g_rank_timer;
    size_t i = 0;
    int dirs = 0;
    while (i < t.used) {
      if (t.slot[i] != 0) {  // (marks before the first call start: none are recorded so)
        ++i;
        continue;
      }
      size_t j = i + 1;
      while (j < t.used && t.slot[j] != 0) ++j;
      // the call's marks [i, j): first and last event of each slot
      long first[NR], last[NR];
      for (int k = 0; k < NR; ++k) first[k] = last[k] = -1;
      for (size_t x = i; x < j; ++x) {
        const int sl = t.slot[x];
        if (sl < 0 || sl >= NR) continue;
        if (first[sl] < 0) first[sl] = (long)x;
        last[sl] = (long)x;
      }
      if (last[NR - 1] >= 0) {  // the call wrote its ranks
        hipError_t err = hipEventSynchronize(t.ev[last[NR - 1]]);
        if (err != hipSuccess) return hip_status(err);
        for (int k = 0; k < KGE_RANK_TIMER_STAGES; ++k) {
          if (first[k] < 0 || last[k + 1] < 0) continue;
          float ms = 0.f;
          err = hipEventElapsedTime(&ms, t.ev[first[k]], t.ev[last[k + 1]]);
          if (err != hipSuccess) return hip_status(err);
          stage_ms_out[k] += ms;
        }
        dirs += t.ndir[i];
      }
      i = j;
    }
    stage_ms_out[KGE_RANK_TIMER_STAGES] = (float)dirs;
    return KGE_OK;
  }
  const size_t calls = g_timer.used / NS_;
  if (command == 3) {
    // per timed call: the 6 stage times, then the call's start relative to the
    // first timed call's start (ms, device clock)
    if (!stage_ms_out || (size_t)n_out < calls * NS_) return KGE_ERR_ARG;
    for (size_t c = 0; c < calls; ++c) {
      hipEvent_t* e = &g_timer.ev[c * NS_];
      hipError_t err = hipEventSynchronize(e[NS_ - 1]);
      if (err != hipSuccess) return hip_status(err);
      for (int k = 0; k < KGE_TIMER_STAGES; ++k) {
        float ms = 0.f;
        err = hipEventElapsedTime(&ms, e[k], e[k + 1]);
        if (err != hipSuccess) return hip_status(err);
        stage_ms_out[c * NS_ + k] = ms;
      }
      float t0 = 0.f;
      err = hipEventElapsedTime(&t0, g_timer.ev[0], e[0]);
      if (err != hipSuccess) return hip_status(err);
      stage_ms_out[c * NS_ + KGE_TIMER_STAGES] = t0;
    }
    return KGE_OK;
  }
  if (command != 2 || !stage_ms_out || n_out < NS_) return KGE_ERR_ARG;
  for (int k = 0; k < NS_; ++k) stage_ms_out[k] = 0.f;
  for (size_t c = 0; c < calls; ++c) {
    hipEvent_t* e = &g_timer.ev[c * NS_];
    hipError_t err = hipEventSynchronize(e[NS_ - 1]);
    if (err != hipSuccess) return hip_status(err);
    for (int k = 0; k < KGE_TIMER_STAGES; ++k) {
      float ms = 0.f;
      err = hipEventElapsedTime(&ms, e[k], e[k + 1]);
      if (err != hipSuccess) return hip_status(err);
      stage_ms_out[k] += ms;
    }
  }
  stage_ms_out[KGE_TIMER_STAGES] = (float)calls;
  return KGE_OK;
}

}  // extern "C"
