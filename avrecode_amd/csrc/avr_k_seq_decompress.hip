// sequential slice kernel, MODE_DECOMPRESS (one translation unit per kernel: see avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_sequential_decompress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                    uint8_t* out, avr_slice_result* res, uint16_t* est, uint8_t* frames, int* frame_meta,
                    hipStream_t stream) {
  hipLaunchKernelGGL(slices_sequential_kernel<MODE_DECOMPRESS>, dim3(1), dim3(64), lds, stream, T, descs, n, in, out, res, est,
                     frames, frame_meta);
  return hipGetLastError();
}

}  // namespace avr
