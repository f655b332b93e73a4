// parallel slice kernel, MODE_DECOMPRESS (one translation unit per kernel: see avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_parallel_decompress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                    uint8_t* out, avr_slice_result* res, uint16_t* est, hipStream_t stream) {
  hipLaunchKernelGGL(slices_parallel_kernel<MODE_DECOMPRESS>, dim3(n), dim3(64), lds, stream, T, descs, n, in, out, res, est);
  return hipGetLastError();
}

}  // namespace avr
