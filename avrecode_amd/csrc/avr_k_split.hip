// The long-slice split's kernels (avr_walker.h slices_split_kernel, avr_kernels.h SplitArgs): the
// parallel model on arithmetic_code<uint64_t, uint8_t>, compress (whole slices, cut as they are
// walked) and decompress (the pieces), in one translation unit with its own CU board.
#include "avr_walker.h"

namespace avr {

int split_grid(int n, int max_mb_width) {
  const int cap = resident_slices(shared_bytes_progressive(max_mb_width, false));
  return cap <= 0 ? (n < 1 ? n : 1) : n < cap ? n : cap;
}

hipError_t launch_split(int mode, const EngineTables* T, const avr_slice_desc* descs, int n, int max_mb_width,
                        const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est, const SplitArgs& sp,
                        uint32_t flags, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (mode != MODE_COMPRESS && mode != MODE_DECOMPRESS) return hipErrorInvalidValue;
  const size_t lds = shared_bytes_progressive(max_mb_width, false);
  if (lds > 160 * 1024 || !sp.ctl || !sp.recs || sp.rec_stride < seam_rec_bytes(max_mb_width)) return hipErrorInvalidValue;
  flags = (flags & ~(kFlagMringGlobal | kFlagFields | kFlagP32 | (0xffffu << kFlagRingShift))) |
          (uint32_t)max_mb_width << kFlagRingShift;
  const int grid = split_grid(n, max_mb_width);
  if (hipError_t e = reset_cu_board(stream); e != hipSuccess) return e;
  if (mode == MODE_COMPRESS)
    hipLaunchKernelGGL((slices_split_kernel<MODE_COMPRESS>), dim3(grid), dim3(slice_threads<MODE_COMPRESS>()), lds,
                       stream, T, descs, n, in, out, res, est, sp, flags);
  else
    hipLaunchKernelGGL((slices_split_kernel<MODE_DECOMPRESS>), dim3(grid), dim3(slice_threads<MODE_DECOMPRESS>()), lds,
                       stream, T, descs, n, in, out, res, est, sp, flags);
  return hipGetLastError();
}

}  // namespace avr
