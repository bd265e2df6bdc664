// In-kernel shader clock over time, beside a running workload (VERDICT r03
// #9, the early-step phase).  One 64-thread workgroup samples the shader-clock
// counter (s_memtime, one tick per shader cycle) and the 100 MHz constant
// counter (s_memrealtime) every few microseconds and stores the pairs with
// vector stores from lane 0 into its own buffer; the clock over any interval
// is Δtick / Δreal × 100 MHz (MI355X_MICROARCH.md, DVFS give-back item 6).
// It occupies one wave slot of one CU and reads nothing the workload writes.
// marker_stamp: one (real, tick) pair on the caller's stream, to place the
// workload's event-timed steps on the probe's real-time axis.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/dbg/libclock_probe.so tools/dbg/clock_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>

__global__ __launch_bounds__(64) void k_clock_probe(uint64_t* __restrict__ out, int n, int spin) {
  for (int i = 0; i < n; ++i) {
    const uint64_t real = __builtin_amdgcn_s_memrealtime();
    const uint64_t tick = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      out[2 * i] = real;
      out[2 * i + 1] = tick;
    }
    for (int k = 0; k < spin; ++k) __builtin_amdgcn_s_sleep(127);
  }
}

__global__ void k_marker(uint64_t* __restrict__ out) {
  const uint64_t real = __builtin_amdgcn_s_memrealtime();
  const uint64_t tick = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = real;
    out[1] = tick;
  }
}

extern "C" int clock_probe_launch(uint64_t* out, int n, int spin, void* stream) {
  if (n <= 0 || spin < 0) return -1;
  hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, out, n, spin);
  return (int)hipGetLastError();
}

extern "C" int marker_stamp(uint64_t* out, void* stream) {
  hipLaunchKernelGGL(k_marker, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  return (int)hipGetLastError();
}
