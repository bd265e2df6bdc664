// Practical ceiling of k_row's access pattern without its arithmetic: one
// 256-thread block per positive row, waves w = 0..3 stream negative rows
// j = w, w+4, ... (n = 256 per block, 1024 blocks), each 8000-B row read as
// two 4000-B halves through range-checked buffer loads, 16 B per lane — the
// same loads k_row issues — into a running sum (one float written per block).
// Table: FB15k RotatE shape, 14951 × 2000 fp32 (119.6 MB); ids uniform.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/gather_ceiling tools/dbg/gather_ceiling.hip
//   /tmp/gather_ceiling            → one JSON line
#include <hip/hip_runtime.h>

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

constexpr int E = 14951, LE = 2000, B = 1024, N = 256, NS = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)bytes, 0x00020000);
}

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_gather(const float* __restrict__ ent, const int64_t* __restrict__ neg,
                                                       float* __restrict__ out) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t* nb = neg + (int64_t)blockIdx.x * N;
  float acc = 0.f;
  for (int j = w; j < N; j += WAVES) {
    const float* row = ent + nb[j] * LE;
    const auto ra = rsrc(row, LE / 2 * 4), rb = rsrc(row + LE / 2, LE / 2 * 4);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const u4 a = __builtin_amdgcn_raw_buffer_load_b128(ra, (uint32_t)(lane + 64 * k) * 16u, 0, 0);
      const u4 b = __builtin_amdgcn_raw_buffer_load_b128(rb, (uint32_t)(lane + 64 * k) * 16u, 0, 0);
      acc += __uint_as_float(a.x) + __uint_as_float(a.y) + __uint_as_float(a.z) + __uint_as_float(a.w);
      acc += __uint_as_float(b.x) + __uint_as_float(b.y) + __uint_as_float(b.z) + __uint_as_float(b.w);
    }
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;  // keeps the loads live, never true for the test data
}

template <int WAVES>
static int run(const float* ent, const int64_t* neg, float* out, const char* tag) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_gather<WAVES>), dim3(B), dim3(64 * WAVES), 0, 0, ent, neg, out);
  CK(hipDeviceSynchronize());
  const int reps = 50;
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_gather<WAVES>), dim3(B), dim3(64 * WAVES), 0, 0, ent, neg, out);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double bytes = (double)B * N * LE * 4 + (double)B * N * 8;
  printf("{\"kernel\": \"gather_ceiling\", \"variant\": \"%s\", \"ms\": %.4f, \"bytes\": %.0f, \"GBps\": %.1f}\n", tag, ms,
         bytes, bytes / (ms * 1e-3) / 1e9);
  return 0;
}

int main() {
  std::mt19937_64 g(7);
  std::vector<float> h_ent((size_t)E * LE);
  for (auto& x : h_ent) x = (float)((g() >> 40) & 0xffff) * 1e-6f;
  std::vector<int64_t> h_neg((size_t)B * N);
  for (auto& x : h_neg) x = (int64_t)(g() % E);
  float* ent;
  int64_t* neg;
  float* out;
  CK(hipMalloc(&ent, h_ent.size() * 4));
  CK(hipMalloc(&neg, h_neg.size() * 8));
  CK(hipMalloc(&out, B * 4));
  CK(hipMemcpy(ent, h_ent.data(), h_ent.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(neg, h_neg.data(), h_neg.size() * 8, hipMemcpyHostToDevice));
  if (run<4>(ent, neg, out, "4 waves/block (k_row's shape)")) return 1;
  if (run<8>(ent, neg, out, "8 waves/block")) return 1;
  if (run<16>(ent, neg, out, "16 waves/block")) return 1;
  CK(hipFree(ent));
  CK(hipFree(neg));
  CK(hipFree(out));
  return 0;
}
