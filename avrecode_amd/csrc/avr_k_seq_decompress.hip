// sequential slice kernel, MODE_DECOMPRESS (one translation unit per kernel: see avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_sequential_decompress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                    uint8_t* out, avr_slice_result* res, uint16_t* est, uint8_t* frames, int* frame_meta,
                    const int* file_first, int n_files, uint64_t frame_stride, uint32_t flags,
                    hipStream_t stream) {
  if (flags & kFlagFields)
    hipLaunchKernelGGL((slices_sequential_kernel<MODE_DECOMPRESS, true>), dim3(n_files), dim3(slice_threads<MODE_DECOMPRESS>()), lds, stream, T, descs, n, in, out, res, est,
                     frames, frame_meta, file_first, frame_stride, flags);
  else
    hipLaunchKernelGGL((slices_sequential_kernel<MODE_DECOMPRESS, false>), dim3(n_files), dim3(slice_threads<MODE_DECOMPRESS>()), lds, stream, T, descs, n, in, out, res, est,
                     frames, frame_meta, file_first, frame_stride, flags);
  return hipGetLastError();
}

// AVR_PROFILE builds: read (and clear) this kernel's section cycle counters; zeros otherwise.
hipError_t profile_sequential_decompress(unsigned long long* out16) {
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
