// parallel slice kernel, MODE_GENERATE (one translation unit per kernel: see avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_parallel_generate(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                    uint8_t* out, avr_slice_result* res, uint16_t* est, const int* order, uint32_t flags, hipStream_t stream) {
  hipLaunchKernelGGL((slices_parallel_kernel<MODE_GENERATE, false>), dim3(n), dim3(slice_threads<MODE_GENERATE>()), lds, stream, T, descs, n, in, out, res, est, order, flags);
  // field pictures / MBAFF frames: a second launch over the batch (its workgroups for progressive
  // slices return at once)
  if (flags & kFlagFields) {
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    hipLaunchKernelGGL((slices_parallel_kernel<MODE_GENERATE, true>), dim3(n), dim3(slice_threads<MODE_GENERATE>()), lds, stream, T, descs, n, in, out, res, est, order, flags);
  }
  return hipGetLastError();
}

// AVR_PROFILE builds: read (and clear) this kernel's section cycle counters; zeros otherwise.
hipError_t profile_parallel_generate(unsigned long long* out16) {
#if defined(AVR_PROFILE) || defined(AVR_WATCHDOG)
  hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(avr_prof), sizeof(unsigned long long) * 64);
  unsigned long long z[64] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(avr_prof), z, sizeof(z));
  return e;
#else
  for (int i = 0; i < 64; i++) out16[i] = 0;
  return hipSuccess;
#endif
}

}  // namespace avr
