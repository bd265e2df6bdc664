// kge_torch_ops.cpp — the `kge` PyTorch operator library:
// TORCH_LIBRARY(kge, m) over the C-ABI of include/kge_hip.h, built into
// libkge_torch.so and loaded with torch.ops.load_library (Python) or linked by
// a libtorch C++ caller — no Python in the call path.
//
//   kge::score             KGEModel.forward + plug-ins            model.py:72-249
//   kge::score_backward    its autograd (dense IndexSelectBackward + index_add_)
//   kge::train_step_grads  train_step up to loss.backward()       model.py:252-301
//   kge::rank_filtered     test_step's filtered ranking           model.py:383-418
//   kge::sample_negatives  TrainDataset.__getitem__ + collate_fn  dataloader.py:34-66
//   kge::error_flag        the device error flag the kernels OR into (IndexError on read)
//
// model / mode are the integer ids of include/kge_hip.h (kge_model_id,
// kge_mode_id).  Argument errors raise before any launch: ValueError
// (TORCH_CHECK_VALUE) with the reference's messages for an unknown model or
// mode (model.py:64-70, 149, 162), RuntimeError (TORCH_CHECK) for devices,
// dtypes and shapes.  CPU tensors are refused — there is no CPU path.  Every
// launch goes on the current HIP stream of the tensors' device; scratch comes
// from the caching allocator on that stream.
#include <cstdlib>
#include <ATen/ATen.h>
#include <ATen/core/op_registration/op_registration.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPStream.h>
#include <torch/autograd.h>
#include <torch/library.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "kge_hip.h"

namespace {

using at::Tensor;
using c10::optional;

constexpr double kPi = 3.14159265358979323846;      // model.py:202
constexpr double kPiTypo = 3.14159262358979323846;  // model.py:232 (pRotatE; reproduced on purpose)
const char* const kModelNames[5] = {"TransE", "DistMult", "ComplEx", "RotatE", "pRotatE"};
const char* const kModeNames[3] = {"single", "head-batch", "tail-batch"};

void check_model_mode(int64_t model, int64_t mode, bool train) {
  TORCH_CHECK_VALUE(model >= KGE_TRANSE && model <= KGE_PROTATE, "model ", model, " not supported");
  const bool ok = (mode == KGE_HEAD_BATCH || mode == KGE_TAIL_BATCH || (!train && mode == KGE_SINGLE));
  TORCH_CHECK_VALUE(ok, "mode ", (mode >= 0 && mode <= 2) ? kModeNames[mode] : std::to_string(mode).c_str(),
                    " not supported");
}

c10::Device require_device(std::initializer_list<const Tensor*> ts) {
  optional<c10::Device> dev;
  for (const Tensor* t : ts) {
    if (!t || !t->defined()) continue;
    TORCH_CHECK(t->is_cuda(), "knowledgegraphembedding_amd runs on MI355X (ROCm) only: got a tensor on ",
                t->device(), ". Move the model and batch to the GPU (run.py --cuda).");
    if (!dev) dev = t->device();
    TORCH_CHECK(t->device() == *dev, "tensors on different devices: ", *dev, " vs ", t->device());
  }
  TORCH_CHECK(dev.has_value(), "no tensor argument");
  return *dev;
}

void check_table(const Tensor& t, const char* what) {
  TORCH_CHECK(t.dim() == 2, what, " must be 2-D, got ", t.sizes());
  TORCH_CHECK(t.scalar_type() == at::kFloat, what, " must be float32 (model.py:45,52), got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), what, " must be contiguous");
}

Tensor as_index(const Tensor& t, c10::Device dev) {
  Tensor o = t.to(dev, at::kLong, /*non_blocking=*/true);
  return o.contiguous();
}

hipStream_t current_stream(c10::Device dev) { return c10::hip::getCurrentHIPStream(dev.index()).stream(); }

// Per-device int32 error flag (written only by atomic OR, so streams share it).
Tensor& error_flag_for(c10::Device dev) {
  static std::mutex mu;
  static std::array<Tensor, 64> flags;
  std::lock_guard<std::mutex> lock(mu);
  const int idx = dev.index() < 0 ? 0 : dev.index();
  TORCH_CHECK(idx < 64, "device index ", idx, " out of range");
  if (!flags[idx].defined()) flags[idx] = at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(dev));
  return flags[idx];
}

kge_model_desc make_desc(int64_t model, const Tensor& entity, const Tensor& relation, double gamma, double erange,
                         const optional<Tensor>& modulus) {
  check_table(entity, "entity_embedding");
  check_table(relation, "relation_embedding");
  kge_model_desc d;
  std::memset(&d, 0, sizeof(d));
  d.struct_size = (int32_t)sizeof(d);
  d.model = (int32_t)model;
  d.entity_dim = (int32_t)entity.size(1);
  d.relation_dim = (int32_t)relation.size(1);
  d.nentity = entity.size(0);
  d.nrelation = relation.size(0);
  d.gamma = (float)gamma;
  d.phase_divisor = (float)(erange / kPi);  // model.py:209, in double then rounded (as the Python mirror)
  d.phase_divisor_p = (float)(erange / kPiTypo);
  d.entity_embedding = entity.data_ptr<float>();
  d.relation_embedding = relation.data_ptr<float>();
  if (model == KGE_PROTATE) {
    TORCH_CHECK(modulus.has_value() && modulus->defined(), "pRotatE needs its modulus (model.py:59-60)");
    TORCH_CHECK(modulus->scalar_type() == at::kFloat && modulus->numel() == 1, "modulus must be a float32 [1, 1]");
    d.modulus = modulus->data_ptr<float>();
  }
  return d;
}

void check_status(int st, const char* what) {
  if (st == KGE_OK) return;
  const char* msg = kge_status_string(st);
  TORCH_CHECK_VALUE(st != KGE_ERR_MODEL && st != KGE_ERR_MODE, what, ": ", msg);
  TORCH_CHECK(false, what, " failed with status ", st, ": ", msg);
}

Tensor workspace(size_t bytes, c10::Device dev) {
  return at::empty({(int64_t)bytes + 256}, at::TensorOptions().dtype(at::kByte).device(dev));
}

// ------------------------------------------------------------------ score
Tensor score_cuda(const Tensor& entity, const Tensor& relation, const Tensor& pos, const optional<Tensor>& neg,
                  int64_t mode, int64_t model, double gamma, double erange, const optional<Tensor>& modulus) {
  check_model_mode(model, mode, false);
  const Tensor* negp = (mode != KGE_SINGLE && neg.has_value()) ? &*neg : nullptr;
  TORCH_CHECK(mode == KGE_SINGLE || negp, "mode ", kModeNames[mode], " needs the negative sample");
  const c10::Device dev = require_device({&entity, &relation, &pos, negp, modulus ? &*modulus : nullptr});
  c10::DeviceGuard guard(dev);
  const kge_model_desc d = make_desc(model, entity, relation, gamma, erange, modulus);
  const Tensor p = as_index(pos, dev);
  TORCH_CHECK(p.dim() == 2 && p.size(1) == 3, "positive sample must be [B, 3], got ", p.sizes());
  Tensor n;
  int64_t B = p.size(0), nn = 1;
  if (negp) {
    n = as_index(*negp, dev);
    TORCH_CHECK(n.dim() == 2 && n.size(0) == B, "negative sample must be [B, n] with B = ", B, ", got ", n.sizes());
    nn = n.size(1);
  }
  Tensor out = at::empty({B, nn}, entity.options());
  if (B == 0 || nn == 0) return out;
  check_status(kge_score(&d, (int32_t)mode, p.data_ptr<int64_t>(), negp ? n.data_ptr<int64_t>() : nullptr, B, nn,
                         out.data_ptr<float>(), error_flag_for(dev).data_ptr<int32_t>(), current_stream(dev)),
               "kge_score");
  return out;
}

Tensor score_meta(const Tensor& entity, const Tensor& relation, const Tensor& pos, const optional<Tensor>& neg,
                  int64_t mode, int64_t model, double gamma, double erange, const optional<Tensor>& modulus) {
  check_model_mode(model, mode, false);
  if (mode == KGE_SINGLE) return at::empty_symint({pos.sym_size(0), 1}, entity.options());
  TORCH_CHECK(neg.has_value(), "mode ", kModeNames[mode], " needs the negative sample");
  return at::empty_symint({neg->sym_size(0), neg->sym_size(1)}, entity.options());
}

std::tuple<Tensor, Tensor, Tensor> score_backward_cuda(const Tensor& grad, const Tensor& entity,
                                                       const Tensor& relation, const Tensor& pos,
                                                       const optional<Tensor>& neg, int64_t mode, int64_t model,
                                                       double gamma, double erange,
                                                       const optional<Tensor>& modulus) {
  check_model_mode(model, mode, false);
  const Tensor* negp = (mode != KGE_SINGLE && neg.has_value()) ? &*neg : nullptr;
  TORCH_CHECK(mode == KGE_SINGLE || negp, "mode ", kModeNames[mode], " needs the negative sample");
  const c10::Device dev =
      require_device({&grad, &entity, &relation, &pos, negp, modulus ? &*modulus : nullptr});
  c10::DeviceGuard guard(dev);
  const kge_model_desc d = make_desc(model, entity, relation, gamma, erange, modulus);
  const Tensor p = as_index(pos, dev);
  const int64_t B = p.size(0);
  Tensor n;
  int64_t nn = 1;
  if (negp) {
    n = as_index(*negp, dev);
    nn = n.size(1);
  }
  const Tensor g = grad.to(at::kFloat).contiguous();
  TORCH_CHECK(g.numel() == B * nn, "grad has ", g.numel(), " elements, expected ", B * nn);
  Tensor ge = at::empty_like(entity, at::MemoryFormat::Contiguous);
  Tensor gr = at::empty_like(relation, at::MemoryFormat::Contiguous);
  const bool has_mod = model == KGE_PROTATE;
  Tensor gm = has_mod ? at::empty_like(*modulus, at::MemoryFormat::Contiguous) : entity.new_empty({0});
  if (B == 0) {
    ge.zero_();
    gr.zero_();
    if (has_mod) gm.zero_();
    return {ge, gr, gm};
  }
  const size_t need = kge_backward_workspace_bytes(&d, (int32_t)mode, B, nn);
  Tensor ws = workspace(need, dev);
  check_status(kge_score_backward(&d, (int32_t)mode, p.data_ptr<int64_t>(), negp ? n.data_ptr<int64_t>() : nullptr,
                                  B, nn, g.data_ptr<float>(), ge.data_ptr<float>(), gr.data_ptr<float>(),
                                  has_mod ? gm.data_ptr<float>() : nullptr, ws.data_ptr(), (size_t)ws.numel(),
                                  error_flag_for(dev).data_ptr<int32_t>(), current_stream(dev)),
               "kge_score_backward");
  return {ge, gr, gm};
}

std::tuple<Tensor, Tensor, Tensor> score_backward_meta(const Tensor& grad, const Tensor& entity,
                                                       const Tensor& relation, const Tensor& pos,
                                                       const optional<Tensor>& neg, int64_t mode, int64_t model,
                                                       double gamma, double erange,
                                                       const optional<Tensor>& modulus) {
  check_model_mode(model, mode, false);
  return {at::empty_like(entity), at::empty_like(relation),
          modulus.has_value() ? at::empty_like(*modulus) : entity.new_empty({0})};
}

// autograd of kge::score: d/d(entity, relation, modulus) through kge::score_backward
class ScoreFunction : public torch::autograd::Function<ScoreFunction> {
 public:
  static Tensor forward(torch::autograd::AutogradContext* ctx, const Tensor& entity, const Tensor& relation,
                        const Tensor& pos, const optional<Tensor>& neg, int64_t mode, int64_t model, double gamma,
                        double erange, const optional<Tensor>& modulus) {
    at::AutoDispatchBelowADInplaceOrView guard;
    static auto op = c10::Dispatcher::singleton().findSchemaOrThrow("kge::score", "").typed<decltype(score_cuda)>();
    Tensor out = op.call(entity, relation, pos, neg, mode, model, gamma, erange, modulus);
    ctx->save_for_backward({entity, relation, pos, neg.has_value() ? *neg : Tensor(),
                            modulus.has_value() ? *modulus : Tensor()});
    ctx->saved_data["mode"] = mode;
    ctx->saved_data["model"] = model;
    ctx->saved_data["gamma"] = gamma;
    ctx->saved_data["erange"] = erange;
    return out;
  }

  static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx,
                                                 torch::autograd::variable_list grads) {
    const auto s = ctx->get_saved_variables();
    const optional<Tensor> neg = s[3].defined() ? optional<Tensor>(s[3]) : c10::nullopt;
    const optional<Tensor> mod = s[4].defined() ? optional<Tensor>(s[4]) : c10::nullopt;
    static auto op = c10::Dispatcher::singleton()
                         .findSchemaOrThrow("kge::score_backward", "")
                         .typed<decltype(score_backward_cuda)>();
    auto r = op.call(grads[0].contiguous(), s[0], s[1], s[2], neg, ctx->saved_data["mode"].toInt(),
                     ctx->saved_data["model"].toInt(), ctx->saved_data["gamma"].toDouble(),
                     ctx->saved_data["erange"].toDouble(), mod);
    return {std::get<0>(r), std::get<1>(r), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(),
            mod.has_value() ? std::get<2>(r) : Tensor()};
  }
};

Tensor score_autograd(const Tensor& entity, const Tensor& relation, const Tensor& pos, const optional<Tensor>& neg,
                      int64_t mode, int64_t model, double gamma, double erange, const optional<Tensor>& modulus) {
  return ScoreFunction::apply(entity, relation, pos, neg, mode, model, gamma, erange, modulus);
}

// ------------------------------------------------------------- train step
std::tuple<Tensor, Tensor, Tensor, Tensor> train_step_grads_cuda(
    const Tensor& entity, const Tensor& relation, const optional<Tensor>& modulus, const Tensor& pos,
    const Tensor& neg, const Tensor& subsampling_weight, int64_t mode, int64_t model, double gamma, double erange,
    bool adversarial, double temperature, bool uni_weight, double regularization) {
  check_model_mode(model, mode, true);
  const c10::Device dev =
      require_device({&entity, &relation, modulus ? &*modulus : nullptr, &pos, &neg, &subsampling_weight});
  c10::DeviceGuard guard(dev);
  const kge_model_desc d = make_desc(model, entity, relation, gamma, erange, modulus);
  const Tensor p = as_index(pos, dev), n = as_index(neg, dev);
  const Tensor w = subsampling_weight.to(at::kFloat).contiguous().view({-1});
  TORCH_CHECK(p.dim() == 2 && p.size(1) == 3 && n.dim() == 2 && n.size(0) == p.size(0) && w.numel() == p.size(0),
              "batch shapes: positive [B, 3], negative [B, n], subsampling_weight [B]; got ", p.sizes(), ", ",
              n.sizes(), ", ", w.sizes());
  const int64_t B = n.size(0), nn = n.size(1);
  Tensor ge = at::empty_like(entity, at::MemoryFormat::Contiguous);
  Tensor gr = at::empty_like(relation, at::MemoryFormat::Contiguous);
  const bool has_mod = model == KGE_PROTATE;
  Tensor gm = has_mod ? at::empty({1, 1}, entity.options()) : entity.new_empty({0});
  Tensor losses = at::empty({5}, entity.options());
  Tensor ws = workspace(kge_train_workspace_bytes(&d, B, nn), dev);
  check_status(kge_train_step_grads(&d, (int32_t)mode, p.data_ptr<int64_t>(), n.data_ptr<int64_t>(), B, nn,
                                    w.data_ptr<float>(), nullptr, uni_weight ? 1 : 0, 0, adversarial ? 1 : 0,
                                    (float)temperature, (float)regularization, ge.data_ptr<float>(),
                                    gr.data_ptr<float>(), has_mod ? gm.data_ptr<float>() : nullptr,
                                    losses.data_ptr<float>(), ws.data_ptr(), (size_t)ws.numel(),
                                    error_flag_for(dev).data_ptr<int32_t>(), current_stream(dev)),
               "kge_train_step_grads");
  return {losses.narrow(0, 0, 4).clone(), ge, gr, gm};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> train_step_grads_meta(
    const Tensor& entity, const Tensor& relation, const optional<Tensor>& modulus, const Tensor& pos,
    const Tensor& neg, const Tensor& subsampling_weight, int64_t mode, int64_t model, double gamma, double erange,
    bool adversarial, double temperature, bool uni_weight, double regularization) {
  check_model_mode(model, mode, true);
  return {entity.new_empty({4}), at::empty_like(entity), at::empty_like(relation),
          modulus.has_value() ? entity.new_empty({1, 1}) : entity.new_empty({0})};
}

// ------------------------------------------------------------------ ranking
std::tuple<Tensor, Tensor> rank_filtered_cuda(const Tensor& entity, const Tensor& relation,
                                              const optional<Tensor>& modulus, const Tensor& queries,
                                              const Tensor& filt_off, const Tensor& filt_ids, int64_t mode,
                                              int64_t model, double gamma, double erange, int64_t path,
                                              const optional<Tensor>& relation_trig) {
  check_model_mode(model, mode, true);
  TORCH_CHECK_VALUE(path >= 0 && path <= 4, "rank path ", path,
                    " not supported (0 auto, 1 mfma, 2 tile, 3 scan, 4 mfma32)");
  const c10::Device dev = require_device({&entity, &relation, modulus ? &*modulus : nullptr, &queries});
  c10::DeviceGuard guard(dev);
  kge_model_desc d = make_desc(model, entity, relation, gamma, erange, modulus);
  if (relation_trig.has_value() && relation_trig->defined() && model == KGE_ROTATE) {
    const Tensor& tr = *relation_trig;
    TORCH_CHECK(tr.device() == dev && tr.scalar_type() == at::kFloat && tr.is_contiguous() && tr.dim() == 3 &&
                    tr.size(0) == d.nrelation && tr.size(1) == 2 && tr.size(2) == d.relation_dim,
                "relation_trig: expected a contiguous float32 [", d.nrelation, ", 2, ", d.relation_dim,
                "] tensor on ", dev);
    d.relation_trig = tr.data_ptr<float>();
  }
  const Tensor q = as_index(queries, dev);
  TORCH_CHECK(q.dim() == 2 && q.size(1) == 3, "queries must be [nq, 3], got ", q.sizes());
  const int64_t nq = q.size(0);
  const Tensor off = as_index(filt_off, dev);
  TORCH_CHECK(off.numel() == nq + 1, "filt_off must hold nq + 1 = ", nq + 1, " offsets, got ", off.numel());
  const Tensor ids = filt_ids.numel() ? as_index(filt_ids, dev)
                                      : at::zeros({1}, at::TensorOptions().dtype(at::kLong).device(dev));
  Tensor ranks = at::empty({nq}, at::TensorOptions().dtype(at::kLong).device(dev));
  Tensor ties = at::empty({nq}, at::TensorOptions().dtype(at::kInt).device(dev));
  if (nq == 0) return {ranks, ties};
  Tensor ws = workspace(kge_rank_workspace_bytes(&d, nq), dev);
  int32_t* err = error_flag_for(dev).data_ptr<int32_t>();
  void* st = current_stream(dev);
  if (model == KGE_PROTATE) {
    // bit-exact pRotatE (kge_hip.h, three-call form): the device decides
    // every near-tie whose score interval under any 1-ulp sin clears the true
    // score's; the undecided ones' phase sums go through the reference's own
    // sin — ATen's CPU at::sin, the call model.py:245 makes — and come back for
    // the reference-order re-scoring, in chunks of ≤ 256 MB of arguments
    Tensor cnt = at::empty({nq}, at::TensorOptions().dtype(at::kInt).device(dev));
    check_status(kge_rank_filtered_ex(&d, (int32_t)mode, q.data_ptr<int64_t>(), nq, off.data_ptr<int64_t>(),
                                      ids.data_ptr<int64_t>(), ranks.data_ptr<int64_t>(), ties.data_ptr<int32_t>(),
                                      cnt.data_ptr<int32_t>(), (int32_t)path | KGE_RANK_STAGE_LIST, ws.data_ptr(),
                                      (size_t)ws.numel(), err, st),
                 "kge_rank_filtered_ex (list)");
    const Tensor c = cnt.to(at::kCPU);  // sync: the counts size the argument buffers
    const int32_t* cp = c.data_ptr<int32_t>();
    // KGE_SIN_CHUNK_BYTES: the chunk budget (tests force several chunks with a small one)
    const char* be = getenv("KGE_SIN_CHUNK_BYTES");
    const int64_t K = d.entity_dim, budget = (be && atoll(be) > 0) ? (int64_t)atoll(be) : ((int64_t)256 << 20);
    auto items_of = [&](int64_t i) -> int64_t {
      return (cp[i] >= 1 && cp[i] <= KGE_RANK_LIST_CAP) ? 1 + (int64_t)cp[i] : 0;
    };
    int64_t lo = 0;
    do {
      // the next chunk [lo, hi): consecutive queries with ≤ budget bytes of arguments
      int64_t hi = lo, bytes = 0;
      while (hi < nq && (bytes == 0 || bytes + items_of(hi) * K * 4 <= budget)) bytes += items_of(hi++) * K * 4;
      Tensor item_off = at::zeros({nq + 1}, at::TensorOptions().dtype(at::kLong));
      int64_t* io = item_off.data_ptr<int64_t>();
      for (int64_t i = 0; i < nq; ++i) io[i + 1] = io[i] + ((i >= lo && i < hi) ? items_of(i) : 0);
      const Tensor off_d = item_off.to(dev);
      Tensor args = at::empty({std::max<int64_t>(io[nq], 1), K}, entity.options());
      Tensor sins = args;
      if (io[nq]) {
        check_status(kge_rank_sin_args(&d, (int32_t)mode, nq, off_d.data_ptr<int64_t>(), args.data_ptr<float>(),
                                       ws.data_ptr(), (size_t)ws.numel(), err, st),
                     "kge_rank_sin_args");
        sins = at::sin(args.to(at::kCPU)).to(dev);
      }
      check_status(kge_rank_finish_sin(&d, (int32_t)mode, nq, off_d.data_ptr<int64_t>(), sins.data_ptr<float>(),
                                       ranks.data_ptr<int64_t>(), ties.data_ptr<int32_t>(), nullptr, ws.data_ptr(),
                                       (size_t)ws.numel(), err, st),
                   "kge_rank_finish_sin");
      lo = hi;
    } while (lo < nq);
    return {ranks, ties};
  }
  check_status(kge_rank_filtered_ex(&d, (int32_t)mode, q.data_ptr<int64_t>(), nq, off.data_ptr<int64_t>(),
                                    ids.data_ptr<int64_t>(), ranks.data_ptr<int64_t>(), ties.data_ptr<int32_t>(),
                                    nullptr, (int32_t)path, ws.data_ptr(), (size_t)ws.numel(), err, st),
               "kge_rank_filtered_ex");
  return {ranks, ties};
}

std::tuple<Tensor, Tensor> rank_filtered_meta(const Tensor& entity, const Tensor& relation,
                                              const optional<Tensor>& modulus, const Tensor& queries,
                                              const Tensor& filt_off, const Tensor& filt_ids, int64_t mode,
                                              int64_t model, double gamma, double erange, int64_t path,
                                              const optional<Tensor>& relation_trig) {
  check_model_mode(model, mode, true);
  auto o = queries.options();
  return {at::empty_symint({queries.sym_size(0)}, o.dtype(at::kLong)),
          at::empty_symint({queries.sym_size(0)}, o.dtype(at::kInt))};
}

// ------------------------------------------------------------------ sampler
void sample_negatives_cuda(const Tensor& triples, const Tensor& batch, int64_t nentity, int64_t negative_sample_size,
                           const Tensor& true_off, const Tensor& true_len, const Tensor& true_ids,
                           const Tensor& weights, int64_t key, int64_t max_draws, const Tensor& pos_out,
                           const Tensor& neg_out, const Tensor& w_out) {
  const c10::Device dev =
      require_device({&triples, &batch, &true_off, &true_len, &true_ids, &weights, &pos_out, &neg_out, &w_out});
  c10::DeviceGuard guard(dev);
  const int64_t B = batch.size(0);
  const std::pair<const Tensor*, at::ScalarType> want[] = {
      {&triples, at::kLong}, {&batch, at::kLong},   {&true_off, at::kLong}, {&true_len, at::kInt},
      {&true_ids, at::kLong}, {&weights, at::kFloat}, {&pos_out, at::kLong}, {&neg_out, at::kLong},
      {&w_out, at::kFloat}};
  for (const auto& tw : want)
    TORCH_CHECK(tw.first->scalar_type() == tw.second && tw.first->is_contiguous(),
                "sample_negatives: expected a contiguous ", tw.second, " tensor, got ", tw.first->scalar_type());
  TORCH_CHECK(pos_out.numel() == B * 3 && neg_out.numel() == B * negative_sample_size && w_out.numel() == B,
              "sample_negatives: output shapes do not match the batch");
  check_status(kge_sample_negatives(triples.data_ptr<int64_t>(), triples.size(0), batch.data_ptr<int64_t>(), B,
                                    nentity, negative_sample_size, true_off.data_ptr<int64_t>(),
                                    true_len.data_ptr<int32_t>(), true_ids.data_ptr<int64_t>(),
                                    weights.data_ptr<float>(), (uint64_t)key, max_draws, pos_out.data_ptr<int64_t>(),
                                    neg_out.data_ptr<int64_t>(), w_out.data_ptr<float>(),
                                    error_flag_for(dev).data_ptr<int32_t>(), current_stream(dev)),
               "kge_sample_negatives");
}

void sample_negatives_meta(const Tensor&, const Tensor&, int64_t, int64_t, const Tensor&, const Tensor&,
                           const Tensor&, const Tensor&, int64_t, int64_t, const Tensor&, const Tensor&,
                           const Tensor&) {}

Tensor error_flag(c10::Device device) {
  TORCH_CHECK(device.is_cuda(), "the error flag lives on a ROCm device, not ", device);
  return error_flag_for(device.has_index() ? device : c10::Device(c10::kCUDA, c10::hip::current_device()));
}

// CPU: no compute path — refuse with the Python mirror's message
template <typename R, typename... A>
R refuse_cpu(A...) {
  TORCH_CHECK(false, "knowledgegraphembedding_amd runs on MI355X (ROCm) only: got CPU tensors. "
                     "Move the model and batch to the GPU (run.py --cuda).");
}

Tensor score_cpu(const Tensor& e, const Tensor& r, const Tensor& p, const optional<Tensor>& n, int64_t mode,
                 int64_t model, double g, double er, const optional<Tensor>& m) {
  check_model_mode(model, mode, false);
  return refuse_cpu<Tensor>();
}
std::tuple<Tensor, Tensor, Tensor> score_backward_cpu(const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                                                      const optional<Tensor>&, int64_t mode, int64_t model, double,
                                                      double, const optional<Tensor>&) {
  check_model_mode(model, mode, false);
  return refuse_cpu<std::tuple<Tensor, Tensor, Tensor>>();
}
std::tuple<Tensor, Tensor, Tensor, Tensor> train_step_grads_cpu(const Tensor&, const Tensor&,
                                                                const optional<Tensor>&, const Tensor&,
                                                                const Tensor&, const Tensor&, int64_t mode,
                                                                int64_t model, double, double, bool, double, bool,
                                                                double) {
  check_model_mode(model, mode, true);
  return refuse_cpu<std::tuple<Tensor, Tensor, Tensor, Tensor>>();
}
std::tuple<Tensor, Tensor> rank_filtered_cpu(const Tensor&, const Tensor&, const optional<Tensor>&, const Tensor&,
                                             const Tensor&, const Tensor&, int64_t mode, int64_t model, double,
                                             double, int64_t, const optional<Tensor>&) {
  check_model_mode(model, mode, true);
  return refuse_cpu<std::tuple<Tensor, Tensor>>();
}
void sample_negatives_cpu(const Tensor&, const Tensor&, int64_t, int64_t, const Tensor&, const Tensor&,
                          const Tensor&, const Tensor&, int64_t, int64_t, const Tensor&, const Tensor&,
                          const Tensor&) {
  refuse_cpu<void>();
}

}  // namespace

TORCH_LIBRARY(kge, m) {
  m.def("score(Tensor entity, Tensor relation, Tensor pos, Tensor? neg, int mode, int model, float gamma, "
        "float embedding_range, Tensor? modulus) -> Tensor");
  m.def("score_backward(Tensor grad, Tensor entity, Tensor relation, Tensor pos, Tensor? neg, int mode, "
        "int model, float gamma, float embedding_range, Tensor? modulus) -> (Tensor, Tensor, Tensor)");
  m.def("train_step_grads(Tensor entity, Tensor relation, Tensor? modulus, Tensor pos, Tensor neg, "
        "Tensor subsampling_weight, int mode, int model, float gamma, float embedding_range, bool adversarial, "
        "float temperature, bool uni_weight, float regularization) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("rank_filtered(Tensor entity, Tensor relation, Tensor? modulus, Tensor queries, Tensor filt_off, "
        "Tensor filt_ids, int mode, int model, float gamma, float embedding_range, int path=0, "
        "Tensor? relation_trig=None) -> (Tensor, Tensor)");
  m.def("sample_negatives(Tensor triples, Tensor batch, int nentity, int negative_sample_size, Tensor true_off, "
        "Tensor true_len, Tensor true_ids, Tensor weights, int key, int max_draws, Tensor(a!) pos_out, "
        "Tensor(b!) neg_out, Tensor(c!) w_out) -> ()");
  m.def("error_flag(Device device) -> Tensor");
  m.impl("error_flag", &error_flag);
}

TORCH_LIBRARY_IMPL(kge, CUDA, m) {
  m.impl("score", &score_cuda);
  m.impl("score_backward", &score_backward_cuda);
  m.impl("train_step_grads", &train_step_grads_cuda);
  m.impl("rank_filtered", &rank_filtered_cuda);
  m.impl("sample_negatives", &sample_negatives_cuda);
}

TORCH_LIBRARY_IMPL(kge, Meta, m) {
  m.impl("score", &score_meta);
  m.impl("score_backward", &score_backward_meta);
  m.impl("train_step_grads", &train_step_grads_meta);
  m.impl("rank_filtered", &rank_filtered_meta);
  m.impl("sample_negatives", &sample_negatives_meta);
}

TORCH_LIBRARY_IMPL(kge, CPU, m) {
  m.impl("score", &score_cpu);
  m.impl("score_backward", &score_backward_cpu);
  m.impl("train_step_grads", &train_step_grads_cpu);
  m.impl("rank_filtered", &rank_filtered_cpu);
  m.impl("sample_negatives", &sample_negatives_cpu);
}

TORCH_LIBRARY_IMPL(kge, Autograd, m) { m.impl("score", &score_autograd); }
