// parallel slice kernel, MODE_DECOMPRESS, P32 coder: the parallel model's optional 32-bit container coder
// (avr_engine.h PEncoder / PDecoder, tag avrecode-amd:P32; one translation unit per kernel, see
// avr_walker.h).
#include "avr_walker.h"

namespace avr {

hipError_t launch_parallel_decompress32(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                  const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                  const int* order, uint32_t flags, hipStream_t stream, uint32_t* qhead, int qgrid, int qgrid_fld, size_t lds_fld, const FieldLane* lane) {
  return launch_parallel<MODE_DECOMPRESS, true>(T, descs, n, lds, in, out, res, est, order, flags, stream, QueueLaunch{qhead, qgrid, qgrid_fld, lds_fld, lane});
}

}  // namespace avr
