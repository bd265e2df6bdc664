// The early-step phase without the training step: does a
// pure Adam-shaped HBM stream — the entity pass's 837 MB per launch of
// p / m / v reads and p / m / v / grad writes over the FB15k table, nothing
// gathered — show the same rise over its first launches and decay over ~40
// launches after the GPU idled?  Each launch timed by its own events; bursts
// of 80 launches after an idle gap (host sleep), for the non-temporal stream
// (as the entity pass), the default-policy stream, and the non-temporal
// stream alternating with a 2.1 GB random-row read of a 120 MB table (k_row's
// gather shape, table resident in the Infinity Cache).  One JSON line per
// launch.  Variant 2 also times each gather launch (gather_us): a table kept
// in the Infinity Cache between launches would show a cold first gather after
// an idle gap if the cache were dropped while the GPU idles.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/stream_hump tools/dbg/stream_hump.hip
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr long N = 14951L * 2000;  // floats per array

template <bool NT>
__global__ __launch_bounds__(256) void k_adam_stream(f4* __restrict__ p, f4* __restrict__ m, f4* __restrict__ v,
                                                     f4* __restrict__ g, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    f4 pp, mm, vv;
    if (NT) {
      pp = __builtin_nontemporal_load(p + i);
      mm = __builtin_nontemporal_load(m + i);
      vv = __builtin_nontemporal_load(v + i);
    } else {
      pp = p[i]; mm = m[i]; vv = v[i];
    }
    const f4 gg = pp * 1e-3f;
    mm = 0.9f * mm + 0.1f * gg;
    vv = 0.999f * vv + 0.001f * gg * gg;
    pp = pp - 1e-4f * mm / (__builtin_elementwise_sqrt(vv) + 1e-8f);
    if (NT) {
      __builtin_nontemporal_store(pp, p + i);
      __builtin_nontemporal_store(mm, m + i);
      __builtin_nontemporal_store(vv, v + i);
      __builtin_nontemporal_store(gg, g + i);
    } else {
      p[i] = pp; m[i] = mm; v[i] = vv; g[i] = gg;
    }
  }
}

// k_row's gather shape: block i reads 256 random 8 KB rows of the table (one
// row per wave step, 4 waves), sums them into a small output
__global__ __launch_bounds__(256) void k_gather(const f4* __restrict__ tab, const int* __restrict__ ids,
                                                float* __restrict__ out, int nneg) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int j = w; j < nneg; j += 4) {
    const f4* row = tab + (long)ids[blockIdx.x * nneg + j] * 500;  // 2000 floats = 500 f4
    for (int k = lane; k < 500; k += 64) acc += row[k];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
  f4 *p, *m, *v, *g;
  CK(hipMalloc(&p, N * 4));
  CK(hipMalloc(&m, N * 4));
  CK(hipMalloc(&v, N * 4));
  CK(hipMalloc(&g, N * 4));
  CK(hipMemset(p, 0, N * 4));
  CK(hipMemset(m, 0, N * 4));
  CK(hipMemset(v, 0, N * 4));
  const int B = 1024, NNEG = 256;
  std::vector<int> hid((size_t)B * NNEG);
  unsigned s = 12345u;
  for (auto& x : hid) {
    s = s * 1664525u + 1013904223u;
    x = (int)((s >> 8) % 14951u);
  }
  int* ids;
  float* out;
  CK(hipMalloc(&ids, hid.size() * 4));
  CK(hipMalloc(&out, (size_t)B * 256 * 4));
  CK(hipMemcpy(ids, hid.data(), hid.size() * 4, hipMemcpyHostToDevice));
  const long n4 = N / 4;
  const int grid = 4096, launches = 80;
  std::vector<hipEvent_t> ev(2 * launches), evg(2 * launches);
  for (auto& e : evg) CK(hipEventCreate(&e));
  for (auto& e : ev) CK(hipEventCreate(&e));
  const char* names[3] = {"stream_nt", "stream_default", "stream_nt_after_gather"};
  for (int variant = 0; variant < 3; ++variant) {
    for (int idle_ms : {2000, 50}) {
      usleep(idle_ms * 1000);
      for (int r = 0; r < launches; ++r) {
        if (variant == 2) {
          CK(hipEventRecord(evg[2 * r], 0));
          hipLaunchKernelGGL(k_gather, dim3(B), dim3(256), 0, 0, (const f4*)p, ids, out, NNEG);
          CK(hipEventRecord(evg[2 * r + 1], 0));
        }
        CK(hipEventRecord(ev[2 * r], 0));
        if (variant == 1) hipLaunchKernelGGL((k_adam_stream<false>), dim3(grid), dim3(256), 0, 0, p, m, v, g, n4);
        else hipLaunchKernelGGL((k_adam_stream<true>), dim3(grid), dim3(256), 0, 0, p, m, v, g, n4);
        CK(hipEventRecord(ev[2 * r + 1], 0));
      }
      CK(hipDeviceSynchronize());
      for (int r = 0; r < launches; ++r) {
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, ev[2 * r], ev[2 * r + 1]));
        float gms = 0.f;
        if (variant == 2) CK(hipEventElapsedTime(&gms, evg[2 * r], evg[2 * r + 1]));
        printf("{\"variant\": \"%s\", \"idle_ms\": %d, \"launch\": %d, \"us\": %.1f, \"gather_us\": %.1f}\n",
               names[variant], idle_ms, r, ms * 1e3, gms * 1e3);
      }
      fflush(stdout);
    }
  }
  return 0;
}
