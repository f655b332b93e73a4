// Host-visible entry points of avr_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#include "../../include/avrecode.h"

namespace avr {

struct EngineTables;

// Per model instance (u16 units): the dense SIG + NZ estimator table (kEstTable entries), then
// the write log that lets the next user clear only what was written (see avr_walker.h): a u32
// count at kEstLogN (kEstLogOverflow: clear the whole table) and kEstLogCap u32 entry indices.
constexpr int kEstTable = 294016;
constexpr int kEstLogN = kEstTable;
constexpr int kEstLog = kEstTable + 2;
constexpr int kEstLogCap = 8191;
constexpr uint32_t kEstLogOverflow = 0xffffffffu;
// then, for the progressive parallel kernels of wide launches (kFlagMringGlobal), the upper row's
// model bytes (Walker::mring: 28 B per macroblock column -- 52 reserved -- up to kMringCols columns)
constexpr int kEstMring = kEstLog + 2 * kEstLogCap;
constexpr int kMringCols = 288;
constexpr int kEstGlobal = kEstMring + kMringCols * 26;
static_assert(kEstGlobal % 8 == 0 && kEstTable % 8 == 0, "16-byte clears");

constexpr uint32_t kFlagBill = 1;   // launch flag: the coders bill per CodingType (avr_slice_result.bill)
// launch flags bits 16-31: EdgeRec slots of the LDS ring (max_mb_width of shared_bytes), set by
// launch_slices; an MBAFF slice needs 3 mb_width + 7 (Walker::pair_edge)
constexpr int kFlagRingShift = 16;
// launch flag: the batch may hold field pictures / MBAFF frames -- the parallel launches add a
// launch of the field-capable kernel for them, the sequential ones use it for every file
constexpr uint32_t kFlagFields = 2;
// launch flag: parallel model with the P32 container coder (avr_k_*32.hip) instead of the reference's
// arithmetic_code<uint64_t, uint8_t>
constexpr uint32_t kFlagP32 = 4;
// launch flag (set by launch_slices): the progressive parallel kernels keep the upper row's model
// bytes in global scratch instead of LDS, so that four workgroups of a wide picture fit a CU
constexpr uint32_t kFlagMringGlobal = 8;
// LDS of one slice workgroup: the field / reference-model walkers' layout (full EdgeRecs), and the
// progressive parallel kernels' (EdgeCore ring, plus the model row in LDS unless mring_global)
size_t shared_bytes(int max_mb_width);
size_t shared_bytes_progressive(int max_mb_width, bool mring_global);
// the progressive parallel kernels of a launch of this width keep the model row in global memory:
// it fits one more workgroup per CU (and the row fits the scratch)
bool mring_global_for(int max_mb_width);
// does workgroup b of a 4G-workgroup launch land on CU group b mod G (schedule_kernel's assumption)?
hipError_t probe_round_robin(size_t lds, bool* ok);
// mode: 0 compress, 1 decompress, 2 generate, 3 trace (decode-only bin trace).  sequential = reference model (single wavefront).
// Sequential (reference-model) launches walk n_files files at once, one workgroup each: file f is
// the slices [file_first[f], file_first[f + 1]) (device array; nullptr = one file of all n slices)
// with est + f kEstGlobal, frames + f frame_stride and frame_meta[f] of its own.
struct SeqFiles {
  const int* file_first = nullptr;
  int n_files = 1;
  uint64_t frame_stride = 0;
};
// The field-capable kernel of a parallel launch beside the progressive one instead of after it (a
// batch holding both, e.g. a corpus with interlaced files): launch_parallel records `fork` on the
// launch's stream once the shared setup (queue, CU board) is queued, runs the field kernel on
// `stream` after it, and makes the launch's stream wait for `join` recorded there.  The persistent
// field kernel then takes the estimator scratches after the progressive kernel's (est_slots with
// fields).  Null stream: the field kernel follows the progressive one on the launch's stream.
struct FieldLane {
  hipStream_t stream = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
// ------------------------------------------------------------------ the long-slice split
// The parallel model may cut a long progressive slice at macroblock-row starts into pieces re-coded
// with fresh models (the oracle's restatement in oracle/oracle_seams.c), so its
// decompress runs on one workgroup per piece.  One record per cut ("seam") in device memory:
struct SeamRec {
  uint32_t first_mb, last_dqp_nz;
  uint32_t cd_low, cd_range, cd_k, cd_next;   // compress: the CABAC decoder at the cut (CabacDecoder)
  uint32_t ce_low, ce_range, ce_outstanding, ce_cache;   // decompress: the re-encoder (CabacEncoder,
  int32_t ce_queue;                                     //   a cache byte always present)
  uint32_t q;                                 // the piece's first byte in the slice's CABAC bytes
  uint32_t pad[4];
  uint8_t state[1024];                        // CABAC context bytes
  // then the upper row's EdgeCore records (kEdgeBytes per macroblock column)
};
constexpr int kEdgeBytes = 40;
static_assert(sizeof(SeamRec) == 64 + 1024, "SeamRec layout");
inline size_t seam_rec_bytes(int max_mb_width) {
  return (sizeof(SeamRec) + (size_t)kEdgeBytes * max_mb_width + 15) & ~(size_t)15;
}
// per descriptor of a split launch
struct PieceCtl {
  int32_t seam;        // its start: record index in SplitArgs::recs, -1 = the slice's own start
  uint32_t n_mbs;      // macroblocks in the piece, 0 = to end_of_slice (the slice's last piece)
  int32_t snap;        // compress: the first record index for the cuts this slice may take (-1: none)
  uint32_t snap_cap;   // records from there
};
struct SplitArgs {
  const PieceCtl* ctl = nullptr;
  uint8_t* recs = nullptr;      // rec_stride bytes per record
  uint32_t rec_stride = 0;
  uint32_t split_bits = 0;      // compress: a cut candidate every split_bits decoded bits
  uint32_t* snap_n = nullptr;   // compress: cuts made (records written) per descriptor
  uint32_t* piece_end = nullptr;   // compress: the re-coded stream's length at the end of each piece,
                                   //   one entry per record (from PieceCtl::snap)
};
// compress (mode 0: whole long slices, cut as they are walked) / decompress (1: the pieces) with the
// parallel model on arithmetic_code<uint64_t, uint8_t> (avr_k_split.hip): one workgroup per
// descriptor, min(n, resident slots) workgroups; est holds that many estimator scratches
int split_grid(int n, int max_mb_width);
hipError_t launch_split(int mode, const EngineTables* T, const avr_slice_desc* descs, int n, int max_mb_width,
                        const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est, const SplitArgs& sp,
                        uint32_t flags, hipStream_t stream);
// flags: kFlagBill (1) = the coders bill per CodingType into avr_slice_result.bill
hipError_t launch_slices(int mode, bool sequential, const EngineTables* T, const avr_slice_desc* descs, int n,
                         int max_mb_width, const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                         uint8_t* frames, int* frame_meta, int* order, hipStream_t stream,
                         const SeqFiles& files = SeqFiles(), uint32_t flags = 0, void* qscratch = nullptr,
                         const FieldLane* lane = nullptr);
// Parallel compress / decompress batches larger than the chip holds at once (more than
// resident_slices) run as one persistent launch over a largest-first queue when launch_slices gets
// a queue scratch of queue_scratch_bytes(n) (device); est then needs est_slots(n, max_mb_width)
// estimator scratches of kEstGlobal u16 (one per resident workgroup), else n; with a FieldLane,
// est_slots(n, max_mb_width, true) (the field kernel's workgroups too).
size_t queue_scratch_bytes(int n);
int slots_per_cu(size_t lds);
int resident_slices(size_t lds);
int est_slots(int n, int max_mb_width, bool field_lane = false);
int parallel_kernel_kind(int mode, int n, int max_mb_width);
// one per kernel translation unit (avr_k_*.hip); lds = shared_bytes(max_mb_width)
hipError_t launch_parallel_compress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                    const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                    const int* order, uint32_t flags, hipStream_t stream,
                                    uint32_t* qhead = nullptr, int qgrid = 0, int qgrid_fld = 0,
                                    size_t lds_fld = 0, const FieldLane* lane = nullptr);
hipError_t launch_parallel_decompress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                      const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                      const int* order, uint32_t flags, hipStream_t stream,
                                    uint32_t* qhead = nullptr, int qgrid = 0, int qgrid_fld = 0,
                                    size_t lds_fld = 0, const FieldLane* lane = nullptr);
hipError_t launch_parallel_compress32(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                      const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                      const int* order, uint32_t flags, hipStream_t stream,
                                    uint32_t* qhead = nullptr, int qgrid = 0, int qgrid_fld = 0,
                                    size_t lds_fld = 0, const FieldLane* lane = nullptr);
hipError_t launch_parallel_decompress32(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                        const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                        const int* order, uint32_t flags, hipStream_t stream,
                                    uint32_t* qhead = nullptr, int qgrid = 0, int qgrid_fld = 0,
                                    size_t lds_fld = 0, const FieldLane* lane = nullptr);
hipError_t launch_parallel_generate(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                    const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                    const int* order, uint32_t flags, hipStream_t stream);
hipError_t launch_parallel_trace(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                 const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                 const int* order, uint32_t flags, hipStream_t stream);
hipError_t launch_sequential_compress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                      const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                      uint8_t* frames, int* frame_meta, const int* file_first, int n_files,
                                      uint64_t frame_stride, uint32_t flags, hipStream_t stream);
hipError_t launch_sequential_decompress(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                        const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                        uint8_t* frames, int* frame_meta, const int* file_first, int n_files,
                                      uint64_t frame_stride, uint32_t flags, hipStream_t stream);
// reference-model compress in parallel (avr_k_rmode.hip): scan (count: ops == nullptr; write),
// estimator chains over the op stream, per-slice coder
hipError_t launch_rscan(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds, const uint8_t* in,
                        uint8_t* frames, const int64_t* goff, uint32_t* counts, uint32_t* ops,
                        const uint64_t* op_off, avr_slice_result* res, int32_t* stop_ok, bool fields, hipStream_t stream);
// Several files in one pass (a corpus): file f's ops are [file_op_off[f], file_op_off[f + 1]) (device,
// n_files + 1 entries; ignored for one file), each file with estimators of its own.
size_t rmode_sort_temp_bytes(uint64_t N, int n_files);
int rmode_max_files_per_pass();
hipError_t launch_rmode_estimators(const uint32_t* ops, uint64_t N, const uint64_t* file_op_off, int n_files,
                                   uint32_t* keys, uint64_t* vals, uint32_t* skeys, uint64_t* svals, void* temp,
                                   size_t temp_bytes, uint32_t* rops, hipStream_t stream);
hipError_t launch_rcode(const EngineTables* T, const avr_slice_desc* descs, int n, const uint32_t* rops,
                        const uint64_t* op_off, const uint32_t* counts, uint8_t* out, avr_slice_result* res,
                        const int32_t* stop_ok, uint32_t flags, hipStream_t stream);
// section cycle counters of AVR_PROFILE builds (avr_walker.h); zeros otherwise
hipError_t profile_parallel_compress(unsigned long long* out16);
hipError_t placement_parallel_compress(uint32_t* out8n, int n);
hipError_t placement_parallel_decompress(uint32_t* out8n, int n);
hipError_t profile_parallel_decompress(unsigned long long* out16);
hipError_t profile_parallel_generate(unsigned long long* out16);
hipError_t profile_parallel_trace(unsigned long long* out16);
hipError_t profile_sequential_compress(unsigned long long* out16);
hipError_t profile_sequential_decompress(unsigned long long* out16);
hipError_t launch_derive_decompress(const avr_slice_desc* descs, const avr_slice_result* rc, int n,
                                    avr_slice_desc* dd, hipStream_t stream);
hipError_t launch_verify(const avr_slice_desc* descs, const avr_slice_result* rc, const avr_slice_result* rd, int n,
                         const uint8_t* in, const uint8_t* regen, int32_t* verdict, hipStream_t stream);
hipError_t launch_pack(const avr_slice_desc* descs, const avr_slice_result* res, int n, const uint8_t* out,
                       uint8_t* packed, uint64_t* offsets, hipStream_t stream);

}  // namespace avr
