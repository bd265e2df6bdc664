// Exhaustive distance, in representable floats, between the device sinf and
// the correctly rounded sin ((float)sin((double)x)) over every finite float
// with |x| <= 2^e_max (default 2^12).  Prints the maximum and a histogram.
//   hipcc --offload-arch=gfx950 -O3 sinf_ulp_scan.hip -o sinf_ulp_scan && ./sinf_ulp_scan [e_max]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ int64_t ord_of(float f) {
  const int32_t b = __float_as_int(f);
  return b >= 0 ? (int64_t)b : -(int64_t)(b & 0x7fffffff);
}

__global__ void scan(uint32_t lim, unsigned long long* hist, int* maxd) {
  // x ranges over bit patterns [0, lim) and their negatives
  const uint64_t n = (uint64_t)lim * 2;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t bits = (uint32_t)(i >> 1) | ((i & 1) ? 0x80000000u : 0u);
    const float x = __int_as_float((int32_t)bits);
    const float d = sinf(x);
    const float r = (float)sin((double)x);
    int64_t dist = ord_of(d) - ord_of(r);
    if (dist < 0) dist = -dist;
    const int c = dist > 7 ? 7 : (int)dist;
    atomicAdd(&hist[c], 1ull);
    if (dist > 0) atomicMax(maxd, (int)(dist > 1000000 ? 1000000 : dist));
  }
}

int main(int argc, char** argv) {
  const int emax = argc > 1 ? atoi(argv[1]) : 12;
  // bit pattern of 2^emax (exclusive upper limit of |x| patterns, plus one to include it)
  const uint32_t lim = ((uint32_t)(127 + emax) << 23) + 1u;
  unsigned long long* hist;
  int* maxd;
  hipMalloc(&hist, 8 * sizeof(unsigned long long));
  hipMalloc(&maxd, sizeof(int));
  hipMemset(hist, 0, 8 * sizeof(unsigned long long));
  hipMemset(maxd, 0, sizeof(int));
  scan<<<8192, 256>>>(lim, hist, maxd);
  unsigned long long h[8];
  int m;
  hipMemcpy(h, hist, sizeof(h), hipMemcpyDeviceToHost);
  hipMemcpy(&m, maxd, sizeof(m), hipMemcpyDeviceToHost);
  printf("{\"emax\": %d, \"max_ulp\": %d, \"hist\": [", emax, m);
  for (int i = 0; i < 8; ++i) printf("%llu%s", h[i], i < 7 ? ", " : "");
  printf("]}\n");
  return 0;
}
