// Ceiling of the entity pass's HBM stream alone: a dense Adam-shaped update
// over the FB15k RotatE table (14951 × 2000 fp32 = 119.6 MB per array) —
// read p, m, v, write p, m, v and the gradient (7 × 119.6 MB = 837 MB, the
// 28 B per element k_entity_sl moves), 16 B per lane, non-temporal like the
// pass, no q gather.  Prints one JSON line per variant.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/stream_ceiling tools/dbg/stream_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
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

template <bool NT>
static int run(f4* p, f4* m, f4* v, f4* g, int grid, const char* tag) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const long n4 = N / 4;
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_adam_stream<NT>), dim3(grid), dim3(256), 0, 0, p, m, v, g, n4);
  CK(hipDeviceSynchronize());
  const int reps = 50;
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_adam_stream<NT>), dim3(grid), dim3(256), 0, 0, p, m, v, g, n4);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double bytes = 7.0 * N * 4;
  printf("{\"kernel\": \"adam_stream_ceiling\", \"variant\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"bytes\": %.0f, \"GBps\": %.1f}\n",
         tag, grid, ms, bytes, bytes / (ms * 1e-3) / 1e9);
  return 0;
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
  for (int grid : {1024, 2048, 4096, 8192}) {
    if (run<true>(p, m, v, g, grid, "non-temporal")) return 1;
    if (run<false>(p, m, v, g, grid, "default policy")) return 1;
  }
  CK(hipFree(p));
  CK(hipFree(m));
  CK(hipFree(v));
  CK(hipFree(g));
  return 0;
}
