// Feasibility of a column-sliced row pass: the negative gather served from the
// XCD's L2 instead of the Infinity Cache.  The FB15k RotatE table (14951 ×
// 2000 fp32, 119.6 MB) is cut into NSL column slices of 4-complex-column
// chunks; XCD x (workgroups are dealt to XCDs round-robin: blockIdx % 8) runs
// slices x, x+8, ... one after the other, so its L2 holds one slice of the
// table (3.8 MB at NSL = 32, 1.9 MB at 64) while every (row, negative) pair
// reads that slice's piece of the negative row.
//   mode 0: partial RotatE distances Σ|q - e| per (slice, row, negative)
//           (pass 1: score pieces, reduced across the pair's lanes)
//   mode 1: Σ_neg w · (q - e)/|q - e| per (slice, row) (pass 2: dL/dq pieces)
// Same 2.1 GB of table bytes per launch as k_row; compare with
// gather_ceiling.hip (the unsliced pattern, 0.287 ms).  One JSON line each.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sliced_row_ceiling tools/dbg/sliced_row_ceiling.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int E = 14951, D = 1000, LE = 2 * D, B = 1024, N = 256, NCH = D / 4;
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NSL>
struct Geo {
  static constexpr int J = NSL / 8;                                   // slices per XCD
  static constexpr int MAXC = (NCH + NSL - 1) / NSL;                  // chunks per slice (max)
  static constexpr int LPP = MAXC <= 4 ? 4 : (MAXC <= 8 ? 8 : 16);    // lanes per pair
  static constexpr int PPW = 64 / LPP;                                // pairs per wave step
};

template <int NSL, int MODE, int UNR>
__global__ __launch_bounds__(256) void k_slice(const float* __restrict__ tab, const float* __restrict__ q,
                                               const int* __restrict__ neg, const float* __restrict__ wgt,
                                               float* __restrict__ out) {
  using G = Geo<NSL>;
  const int xcd = blockIdx.x & 7;
  const int t = blockIdx.x >> 3;
  const int j = t / (B / 4), rb = t % (B / 4);
  const int sl = xcd + 8 * j;
  const int c0 = sl * NCH / NSL, c1 = (sl + 1) * NCH / NSL;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = rb * 4 + w;
  const int sub = lane % G::LPP, grp = lane / G::LPP;
  const int ch = c0 + sub;
  const bool act = ch < c1;
  const int co = act ? ch * 4 : 0;
  f4 qa = act ? *(const f4*)(q + (size_t)row * LE + co) : f4{0, 0, 0, 0};
  f4 qb = act ? *(const f4*)(q + (size_t)row * LE + D + co) : f4{0, 0, 0, 0};
  f4 ar = {0, 0, 0, 0}, ai = {0, 0, 0, 0};
  const int* nb = neg + row * N;
  for (int n0 = 0; n0 < N; n0 += G::PPW * UNR) {
    f4 ea[UNR], eb[UNR];
    float wv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int e = nb[n0 + u * G::PPW + grp];
      const float* er = tab + (size_t)e * LE + co;
      ea[u] = act ? *(const f4*)er : f4{0, 0, 0, 0};
      eb[u] = act ? *(const f4*)(er + D) : f4{0, 0, 0, 0};
      if (MODE == 1) wv[u] = wgt[row * N + n0 + u * G::PPW + grp];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const f4 dr = qa - ea[u], di = qb - eb[u];
      const f4 s2 = dr * dr + di * di;
      if (MODE == 0) {
        float s = act ? (sqrtf(s2.x) + sqrtf(s2.y)) + (sqrtf(s2.z) + sqrtf(s2.w)) : 0.f;
#pragma unroll
        for (int m = 1; m < G::LPP; m <<= 1) s += __shfl_xor(s, m);
        if (sub == 0) out[((size_t)sl * B + row) * N + n0 + u * G::PPW + grp] = s;
      } else {
        const f4 inv = {s2.x > 0.f ? __frsqrt_rn(s2.x) : 0.f, s2.y > 0.f ? __frsqrt_rn(s2.y) : 0.f,
                        s2.z > 0.f ? __frsqrt_rn(s2.z) : 0.f, s2.w > 0.f ? __frsqrt_rn(s2.w) : 0.f};
        ar += wv[u] * (dr * inv);
        ai += wv[u] * (di * inv);
      }
    }
  }
  if (MODE == 1) {
    // the pair groups of a wave hold partial sums of the same row: fold them
#pragma unroll
    for (int m = G::LPP; m < 64; m <<= 1) {
      ar.x += __shfl_xor(ar.x, m); ar.y += __shfl_xor(ar.y, m); ar.z += __shfl_xor(ar.z, m); ar.w += __shfl_xor(ar.w, m);
      ai.x += __shfl_xor(ai.x, m); ai.y += __shfl_xor(ai.y, m); ai.z += __shfl_xor(ai.z, m); ai.w += __shfl_xor(ai.w, m);
    }
    if (grp == 0 && act) {
      *(f4*)(out + (size_t)row * LE + co) = ar;
      *(f4*)(out + (size_t)row * LE + D + co) = ai;
    }
  }
}

template <int NSL, int MODE, int UNR>
static int run(const float* tab, const float* q, const int* neg, const float* wgt, float* out, const float* h_tab,
               const float* h_q, const int* h_neg, const float* h_w) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = NSL * (B / 4);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_slice<NSL, MODE, UNR>), dim3(grid), dim3(256), 0, 0, tab, q, neg, wgt, out);
  CK(hipDeviceSynchronize());
  const int reps = 50;
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_slice<NSL, MODE, UNR>), dim3(grid), dim3(256), 0, 0, tab, q, neg, wgt, out);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  // spot check one (row, negative) / one row against the host
  double err = 0.0;
  const int row = 777, nn = 131;
  if (MODE == 0) {
    std::vector<float> part((size_t)NSL * B * N);
    CK(hipMemcpy(part.data(), out, part.size() * 4, hipMemcpyDeviceToHost));
    double ref = 0.0, got = 0.0;
    const int e = h_neg[row * N + nn];
    for (int c = 0; c < D; ++c) {
      const double dr = h_q[(size_t)row * LE + c] - h_tab[(size_t)e * LE + c];
      const double di = h_q[(size_t)row * LE + D + c] - h_tab[(size_t)e * LE + D + c];
      ref += std::sqrt(dr * dr + di * di);
    }
    for (int s = 0; s < NSL; ++s) got += part[((size_t)s * B + row) * N + nn];
    err = std::fabs(got - ref) / ref;
  } else {
    std::vector<float> dq((size_t)B * LE);
    CK(hipMemcpy(dq.data(), out, dq.size() * 4, hipMemcpyDeviceToHost));
    for (int c = 0; c < D; c += 97) {
      double rr = 0.0;
      for (int k = 0; k < N; ++k) {
        const int e = h_neg[row * N + k];
        const double dr = h_q[(size_t)row * LE + c] - h_tab[(size_t)e * LE + c];
        const double di = h_q[(size_t)row * LE + D + c] - h_tab[(size_t)e * LE + D + c];
        const double m = std::sqrt(dr * dr + di * di);
        rr += h_w[row * N + k] * (m > 0 ? dr / m : 0.0);
      }
      err = std::fmax(err, std::fabs(dq[(size_t)row * LE + c] - rr) / (std::fabs(rr) + 1e-3));
    }
  }
  const double bytes = (double)B * N * LE * 4;
  printf("{\"kernel\": \"sliced_row\", \"mode\": \"%s\", \"nsl\": %d, \"unroll\": %d, \"ms\": %.4f, \"table_GBps\": %.1f, "
         "\"rel_err\": %.2e}\n",
         MODE ? "dq pieces" : "score pieces", NSL, UNR, ms, bytes / (ms * 1e-3) / 1e9, err);
  fflush(stdout);
  return 0;
}

int main() {
  std::mt19937_64 g(7);
  std::vector<float> h_tab((size_t)E * LE), h_q((size_t)B * LE), h_w((size_t)B * N);
  std::uniform_real_distribution<float> U(-0.05f, 0.05f);
  for (auto& x : h_tab) x = U(g);
  for (auto& x : h_q) x = U(g);
  for (auto& x : h_w) x = U(g) + 0.06f;
  std::vector<int> h_neg((size_t)B * N);
  for (auto& x : h_neg) x = (int)(g() % E);
  float *tab, *q, *wgt, *out;
  int* neg;
  CK(hipMalloc(&tab, h_tab.size() * 4));
  CK(hipMalloc(&q, h_q.size() * 4));
  CK(hipMalloc(&wgt, h_w.size() * 4));
  CK(hipMalloc(&neg, h_neg.size() * 4));
  CK(hipMalloc(&out, (size_t)64 * B * N * 4));
  CK(hipMemcpy(tab, h_tab.data(), h_tab.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(q, h_q.data(), h_q.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wgt, h_w.data(), h_w.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(neg, h_neg.data(), h_neg.size() * 4, hipMemcpyHostToDevice));
#define R(NSL, MODE, UNR) \
  if (run<NSL, MODE, UNR>(tab, q, neg, wgt, out, h_tab.data(), h_q.data(), h_neg.data(), h_w.data())) return 1;
  R(32, 0, 2) R(32, 0, 4) R(32, 0, 8) R(64, 0, 4) R(64, 0, 8) R(16, 0, 4)
  R(32, 1, 2) R(32, 1, 4) R(32, 1, 8) R(64, 1, 4) R(64, 1, 8) R(16, 1, 4)
  return 0;
}
