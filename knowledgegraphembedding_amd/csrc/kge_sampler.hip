// kge_sampler.hip — device negative sampler (TrainDataset.__getitem__ +
// collate_fn, dataloader.py:34-66): for each positive of a batch, n negative
// heads (head-batch) or tails (tail-batch) drawn uniformly from [0, E) with
// the true heads of (r, t) / true tails of (h, r) rejected, plus the
// positive itself and its subsampling weight.
//
// One wave per positive.  Draw d of batch row i is the counter-based value
//   x = mix64(mix64(key ^ i·C1) + d·C2),   candidate = ⌊x·E / 2^64⌋
// (mix64 = the splitmix64 finaliser; C2 its Weyl increment, so each row walks
// its own splitmix64 sequence).  Each step the 64 lanes draw 64 consecutive
// d, test membership by binary search in the row's sorted true list, and
// keep the survivors in draw order (ballot + prefix popcount) until n are
// written — the first n survivors of an i.i.d. uniform stream, which is the
// distribution of the reference's "draw 2n, drop the true ones, repeat,
// truncate to n" loop (dataloader.py:44-61).
#include "kge_common.h"

namespace kge {

namespace {

constexpr uint64_t kRowMul = 0xD1B54A32D192ED03ull;
constexpr uint64_t kWeyl = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct SampleArgs {
  const int64_t* triples;   // [T, 3]
  int64_t T;
  const int64_t* batch;     // [B] triple ids
  int64_t B, E, n;
  const int64_t* true_off;  // [T] start of each triple's true list in true_ids
  const int32_t* true_len;  // [T]
  const int64_t* true_ids;  // sorted ascending inside each list
  const float* weights;     // [T] subsampling weights
  uint64_t key;
  int64_t max_draws;        // per row; beyond it the row is reported (KGE_DEVERR_SAMPLER)
  int64_t* pos_out;         // [B, 3]
  int64_t* neg_out;         // [B, n]
  float* w_out;             // [B]
  int32_t* err;
};

__global__ __launch_bounds__(256) void k_sample_neg(SampleArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + wave_id();
  if (i >= a.B) return;
  int64_t* out = a.neg_out + i * a.n;
  const int64_t ti = a.batch[i];
  if (ti < 0 || ti >= a.T) {
    if (lane == 0) atomicOr(a.err, KGE_DEVERR_INDEX);
    for (int64_t j = lane; j < a.n; j += 64) out[j] = 0;
    if (lane < 3) a.pos_out[i * 3 + lane] = 0;
    if (lane == 0) a.w_out[i] = 0.f;
    return;
  }
  if (lane < 3) a.pos_out[i * 3 + lane] = a.triples[ti * 3 + lane];
  if (lane == 0) a.w_out[i] = a.weights[ti];
  const int64_t* ids = a.true_ids + a.true_off[ti];
  const int len = a.true_len[ti];
  const uint64_t krow = mix64(a.key ^ ((uint64_t)i * kRowMul));
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int64_t filled = 0;
  for (int64_t d = 0; filled < a.n; d += 64) {
    if (d >= a.max_draws) {  // (almost) every entity is a true one: report, pad with the last draw
      if (lane == 0) atomicOr(a.err, KGE_DEVERR_SAMPLER);
      for (int64_t j = filled + lane; j < a.n; j += 64) out[j] = 0;
      break;
    }
    const uint64_t x = mix64(krow + (uint64_t)(d + lane) * kWeyl);
    const int64_t e = (int64_t)__umul64hi(x, (uint64_t)a.E);
    int lo = 0, hi = len;  // first index with ids[k] >= e
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ids[mid] < e) lo = mid + 1;
      else hi = mid;
    }
    const bool keep = !(lo < len && ids[lo] == e);
    const uint64_t m = __ballot(keep);
    const int64_t slot = filled + __popcll(m & below);
    if (keep && slot < a.n) out[slot] = e;
    filled += __popcll(m);
  }
}

}  // namespace

}  // namespace kge

extern "C" {

int kge_sample_negatives(const int64_t* triples, int64_t ntriples, const int64_t* batch, int64_t batch_size,
                         int64_t nentity, int64_t negative_sample_size, const int64_t* true_off,
                         const int32_t* true_len, const int64_t* true_ids, const float* weights, uint64_t key,
                         int64_t max_draws, int64_t* pos_out, int64_t* neg_out, float* w_out, int32_t* err_flag,
                         void* stream) {
  if (!triples || !batch || !true_off || !true_len || !true_ids || !weights || !pos_out || !neg_out || !w_out ||
      !err_flag)
    return KGE_ERR_ARG;
  if (ntriples < 0 || batch_size < 0 || nentity <= 0 || negative_sample_size < 0 || max_draws <= 0)
    return KGE_ERR_ARG;
  if (batch_size == 0) return KGE_OK;
  kge::SampleArgs a;
  a.triples = triples; a.T = ntriples; a.batch = batch; a.B = batch_size; a.E = nentity;
  a.n = negative_sample_size; a.true_off = true_off; a.true_len = true_len; a.true_ids = true_ids;
  a.weights = weights; a.key = key; a.max_draws = max_draws;
  a.pos_out = pos_out; a.neg_out = neg_out; a.w_out = w_out; a.err = err_flag;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(kge::k_sample_neg, dim3((unsigned)((batch_size + 3) / 4)), dim3(256), 0, s, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KGE_OK : KGE_ERR_HIP_BASE + (int)e;
}

}  // extern "C"
