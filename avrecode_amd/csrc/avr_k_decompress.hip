// parallel slice kernel, MODE_DECOMPRESS, the reference's arithmetic_code<uint64_t, uint8_t> coder (one
// translation unit per kernel: see avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_parallel_decompress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                    uint8_t* out, avr_slice_result* res, uint16_t* est, const int* order, uint32_t flags, hipStream_t stream, uint32_t* qhead, int qgrid, int qgrid_fld, size_t lds_fld, const FieldLane* lane) {
  return launch_parallel<MODE_DECOMPRESS, false>(T, descs, n, lds, in, out, res, est, order, flags, stream, QueueLaunch{qhead, qgrid, qgrid_fld, lds_fld, lane});
}

// AVR_PROFILE builds: read (and clear) this kernel's section cycle counters; zeros otherwise.
hipError_t profile_parallel_decompress(unsigned long long* out16) {
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

// AVR_PROFILE builds: per-slice wave placement (see avr_place); zeros otherwise.
hipError_t placement_parallel_decompress(uint32_t* out, int n) {
  if (n > 4096) n = 4096;
#ifdef AVR_PROFILE
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(avr_place), sizeof(uint32_t) * 8 * n);
#else
  for (int i = 0; i < 8 * n; i++) out[i] = 0;
  return hipSuccess;
#endif
}

}  // namespace avr
