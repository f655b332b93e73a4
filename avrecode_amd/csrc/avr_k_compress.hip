// parallel slice kernel, MODE_COMPRESS, the reference's arithmetic_code<uint64_t, uint8_t> coder (one
// translation unit per kernel: see avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_parallel_compress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                    uint8_t* out, avr_slice_result* res, uint16_t* est, const int* order, uint32_t flags, hipStream_t stream, uint32_t* qhead, int qgrid, int qgrid_fld, size_t lds_fld, const FieldLane* lane) {
  return launch_parallel<MODE_COMPRESS, false>(T, descs, n, lds, in, out, res, est, order, flags, stream, QueueLaunch{qhead, qgrid, qgrid_fld, lds_fld, lane});
}

// AVR_PROFILE builds: read (and clear) this kernel's section cycle counters; zeros otherwise.
hipError_t profile_parallel_compress(unsigned long long* out16) {
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

#ifdef AVR_QTRACE
// Queue trace builds: host-mapped coherent memory for the compress kernel's progress records (8
// u32 per workgroup, avr_walker.h QTRACE), returned to the caller; nwg workgroups at most.
extern "C" int avr_debug_qtrace(uint32_t** host, int nwg) {
  void* p = nullptr;
  if (hipHostMalloc(&p, (size_t)nwg * 32, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return -2;
  for (size_t i = 0; i < (size_t)nwg * 8; i++) ((uint32_t*)p)[i] = 0;
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) return -2;
  if (hipMemcpyToSymbol(HIP_SYMBOL(avr::avr_qtrace), &dp, sizeof(dp)) != hipSuccess) return -2;
  *host = (uint32_t*)p;
  return 0;
}
#endif
