// parallel slice kernel, MODE_COMPRESS (one translation unit per kernel: see avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_parallel_compress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                    uint8_t* out, avr_slice_result* res, uint16_t* est, const int* order, uint32_t flags, hipStream_t stream) {
  // the per-CU priority board of this kernel starts empty on every launch (cu_cell's slot counter
  // must not carry a previous launch's residue)
  if (hipError_t e = reset_cu_board(stream); e != hipSuccess) return e;
  hipLaunchKernelGGL((slices_parallel_kernel<MODE_COMPRESS, false>), dim3(n), dim3(slice_threads<MODE_COMPRESS>()), lds, stream, T, descs, n, in, out, res, est, order, flags);
  // field pictures / MBAFF frames: a second launch over the batch (its workgroups for progressive
  // slices return at once)
  if (flags & kFlagFields) {
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    if (hipError_t e = reset_cu_board(stream); e != hipSuccess) return e;
    hipLaunchKernelGGL((slices_parallel_kernel<MODE_COMPRESS, true>), dim3(n), dim3(slice_threads<MODE_COMPRESS>()), lds, stream, T, descs, n, in, out, res, est, order, flags);
  }
  return hipGetLastError();
}

// AVR_PROFILE builds: read (and clear) this kernel's section cycle counters; zeros otherwise.
hipError_t profile_parallel_compress(unsigned long long* out16) {
#ifdef AVR_PROFILE
  hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(avr_prof), sizeof(unsigned long long) * 64);
  unsigned long long z[64] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(avr_prof), z, sizeof(z));
  return e;
#else
  for (int i = 0; i < 64; i++) out16[i] = 0;
  return hipSuccess;
#endif
}

// AVR_PROFILE builds: per-slice wave placement (see avr_place); zeros otherwise.
hipError_t placement_parallel_compress(uint32_t* out, int n) {
  if (n > 4096) n = 4096;
#ifdef AVR_PROFILE
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(avr_place), sizeof(uint32_t) * 8 * n);
#else
  for (int i = 0; i < 8 * n; i++) out[i] = 0;
  return hipSuccess;
#endif
}

}  // namespace avr
