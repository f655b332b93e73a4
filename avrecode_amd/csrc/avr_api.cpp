// C ABI of avrecode-amd (include/avrecode.h): host orchestration around the device kernels.
//
//   compress file   demux + headers (avr_front.cpp) -> payload arena in HBM -> slice kernel
//                   (one wavefront per slice) -> segmentation + Recoded protobuf
//                   (recode.cpp:1102-1132, 1275-1297)
//   decompress file Recoded -> literal + surrogate stream (recode.cpp:1359-1409, 1527-1544) ->
//                   headers -> slice kernel -> last-byte patch (recode.cpp:1345-1356)
//
// The hot path has no host implementation: without a GPU every entry point fails with
// AVR_ERR_DEVICE.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <zlib.h>

#include "../../include/avrecode.h"
#include "avr_engine.h"
#include "avr_front.h"
#include "avr_synth.h"
#include "avr_kernels.h"
#include "h264_tables.h"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  // zero: a fresh allocation starts zeroed (the estimator tables rely on it, see kEstLogN)
  hipError_t reserve(size_t n, bool zero = false) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess && zero) e = hipMemset(p, 0, n);
    if (e == hipSuccess && zero) e = hipDeviceSynchronize();
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  ~DevBuf() { release(); }
  template <class T>
  T* as() const {
    return (T*)p;
  }
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct avr_ctx {
  int device = 0;
  std::string err;
  hipStream_t stream = nullptr;
  DevBuf tables, est, frames, frame_meta, in, out, descs, res, packed, offsets, order;
  DevBuf queue;                                          // largest-first slice queue (launch_slices)
  DevBuf rm_goff, rm_counts, rm_stop, rm_off, rm_ops;   // parallel reference-model compress
  DevBuf regen, dec_descs, res_d, verdict;               // compress-side roundtrip check
  DevBuf file_first, file_op_off;                        // reference model over several files
  // the parallel model's long-slice split (split_compress / split_decompress): its own stream, so the
  // long slices' first pass overlaps the rest of the batch, and its own estimator scratch
  hipStream_t split_stream = nullptr;
  DevBuf sp_in, sp_out, sp_descs, sp_res, sp_ctl, sp_recs, sp_snapn, sp_est, sp_in2, sp_out2;
  size_t split_bytes = 0;   // avr_set_split_bytes / AVR_SPLIT_BYTES (0: no split)
  // a batch holding both progressive and field slices runs its field kernel beside the progressive
  // one (avr::FieldLane); AVR_FIELD_LANE=0 keeps the two in one stream, one after the other
  hipStream_t fld_stream = nullptr;
  hipEvent_t fld_ev[2] = {nullptr, nullptr};
  avr::FieldLane field_lane() const {
    avr::FieldLane l;
    if (fld_stream) l.stream = fld_stream, l.fork = fld_ev[0], l.join = fld_ev[1];
    return l;
  }
  bool round_robin = false;   // placement probe passed: the CU schedule (order) may be used
  int* order_or_null() { return round_robin ? order.as<int>() : nullptr; }
  // phase breakdown of the current / last whole-file call (avr_phase_times): run_plan adds the
  // device phases (HIP events ev[0..3] around its uploads, kernels and downloads) and its own wall
  // time (plan_wall); the file paths add the host phases
  avr_phase_times phase{};
  double plan_wall = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  ~avr_ctx() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (split_stream) (void)hipStreamDestroy(split_stream);
    for (auto& e : fld_ev)
      if (e) (void)hipEventDestroy(e);
    if (fld_stream) (void)hipStreamDestroy(fld_stream);
  }
};

namespace {

// Model modes (include/avrecode.h): the reference model, and the parallel model on the reference's
// arithmetic_code<uint64_t, uint8_t> (PARALLEL) or on the optional 32-bit P32 coder (PARALLEL32).
bool valid_model(int m) {
  return m == AVR_MODEL_REFERENCE || m == AVR_MODEL_PARALLEL || m == AVR_MODEL_PARALLEL32 || m == AVR_MODEL_CHAINED;
}
bool parallel_model(int m) { return m == AVR_MODEL_PARALLEL || m == AVR_MODEL_PARALLEL32; }
// the reference model over a whole file, or in chains of AVR_CHAIN_SLICES coded slices
bool reference_model(int m) { return m == AVR_MODEL_REFERENCE || m == AVR_MODEL_CHAINED; }
// models whose per-slice outputs come from several ranks and are assembled on one: the parallel
// models (slice ranges) and the chained model (chain ranges); the reference model is one unit
bool assemblable(int m) { return parallel_model(m) || m == AVR_MODEL_CHAINED; }
uint32_t coder_flag(int m) { return m == AVR_MODEL_PARALLEL32 ? avr::kFlagP32 : 0u; }
constexpr size_t kLdsBudget = 160 * 1024;   // LDS per workgroup (one slice) on gfx950
constexpr uint64_t kMaxSynthBytes = (uint64_t)1 << 35;   // avr_synthesize_stream's output cap (32 GiB)

int fail(avr_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
// No C++ exception crosses the C ABI: the entry points that build host containers run their body
// through guarded(), which turns an allocation failure into AVR_ERR_OUT_OF_MEMORY.
template <class F>
int guarded(avr_ctx* c, F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return fail(c, AVR_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(c, AVR_ERR_DEVICE, std::string("internal error: ") + e.what());
  }
}
#define HIP_TRY(c, expr)                                                                              \
  do {                                                                                                \
    hipError_t _e = (expr);                                                                           \
    if (_e != hipSuccess) return fail(c, AVR_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

// Engine tables: FFmpeg-layout CABAC tables, (m,n) init, exact reciprocals for the recoded
// coder's (range/(pos+neg)) and the model's neighbour geometry.
void build_tables(avr::EngineTables* t) {
  memset(t, 0, sizeof(*t));
  // FFmpeg-layout LPS range [q*128 + state] and transitions ([128+s] MPS, [127-s] LPS), state =
  // 2*pStateIdx + valMPS; packed per state into one 64-bit record (HotTables::cabac)
  uint8_t lps[512], mlps[256];
  for (int q = 0; q < 4; q++)
    for (int i = 0; i < 64; i++) lps[q * 128 + 2 * i] = lps[q * 128 + 2 * i + 1] = avr::kRangeTabLPS[i][q];
  for (int i = 0; i < 64; i++) {
    int mps = i < 62 ? i + 1 : i;
    mlps[128 + 2 * i] = (uint8_t)(2 * mps);
    mlps[128 + 2 * i + 1] = (uint8_t)(2 * mps + 1);
    mlps[127 - 2 * i] = (uint8_t)(i == 0 ? 1 : 2 * avr::kTransIdxLPS[i]);
    mlps[127 - (2 * i + 1)] = (uint8_t)(i == 0 ? 0 : 2 * avr::kTransIdxLPS[i] + 1);
  }
  for (int st = 0; st < 128; st++) {
    uint64_t r = 0;
    for (int q = 0; q < 4; q++) r |= (uint64_t)lps[q * 128 + st] << (8 * q);
    r |= (uint64_t)mlps[128 + st] << 32;
    r |= (uint64_t)mlps[127 - st] << 40;
    t->hot.cabac[st] = r;
  }
  for (int tbl = 0; tbl < 4; tbl++)
    for (int c = 0; c < 1024; c++) {
      int m, n;
      avr::mn_for_ctx(tbl - 1, c, &m, &n);
      t->mn[tbl][c][0] = (int8_t)m;
      t->mn[tbl][c][1] = (int8_t)n;
    }
  for (uint32_t d = 2; d < 128; d++) {
    int l = 0;
    while ((1u << l) < d) l++;
    unsigned __int128 num = (unsigned __int128)1 << (63 + l);
    t->hot.div[d][0] = (uint64_t)((num + d - 1) / d);
    t->hot.div[d][1] = (uint64_t)(l - 1);
    t->hot.rcp32[d] = (uint32_t)((1ull << 32) / d);   // P-format coder (avr_engine.h, PEncoder)
  }
  // reverse_scan_8 neighbours (recode.cpp:279-312, 444-447)
  static const uint8_t scan8[48] = {
    4 + 1 * 8,  5 + 1 * 8,  4 + 2 * 8,  5 + 2 * 8,  6 + 1 * 8,  7 + 1 * 8,  6 + 2 * 8,  7 + 2 * 8,
    4 + 3 * 8,  5 + 3 * 8,  4 + 4 * 8,  5 + 4 * 8,  6 + 3 * 8,  7 + 3 * 8,  6 + 4 * 8,  7 + 4 * 8,
    4 + 6 * 8,  5 + 6 * 8,  4 + 7 * 8,  5 + 7 * 8,  6 + 6 * 8,  7 + 6 * 8,  6 + 7 * 8,  7 + 7 * 8,
    4 + 8 * 8,  5 + 8 * 8,  4 + 9 * 8,  5 + 9 * 8,  6 + 8 * 8,  7 + 8 * 8,  6 + 9 * 8,  7 + 9 * 8,
    4 + 11 * 8, 5 + 11 * 8, 4 + 12 * 8, 5 + 12 * 8, 6 + 11 * 8, 7 + 11 * 8, 6 + 12 * 8, 7 + 12 * 8,
    4 + 13 * 8, 5 + 13 * 8, 4 + 14 * 8, 5 + 14 * 8, 6 + 13 * 8, 7 + 13 * 8, 6 + 14 * 8, 7 + 14 * 8};
  auto cell_block = [&](int row, int col, bool* crossed) {
    const int top = row <= 4 ? 1 : row <= 9 ? 6 : 11;
    *crossed = false;
    if (row == top - 1) row = top + 3, *crossed = true;
    if (col == 3) col = 7, *crossed = true;
    for (int k = 0; k < 48; k++)
      if (scan8[k] == row * 8 + col) return k;
    return 0;
  };
  for (int n = 0; n < 48; n++) {
    bool cr;
    int s = scan8[n];
    int l = cell_block(s >> 3, (s & 7) - 1, &cr);
    t->hot.nb_left[n] = (uint8_t)(l | (cr ? 128 : 0));
    int u = cell_block((s >> 3) - 1, s & 7, &cr);
    t->hot.nb_up[n] = (uint8_t)(u | (cr ? 128 : 0));
  }
  // ctxIdx bases per ctxBlockCat (9.3.3.1.1.9, frame coded) and the 8x8 ctxIdxInc maps
  static const int16_t cbf[14] = {85, 89, 93, 97, 101, 1012, 460, 464, 468, 1016, 472, 476, 480, 1020};
  static const int16_t sig[14] = {105, 120, 134, 149, 152, 402, 484, 499, 513, 660, 528, 543, 557, 718};
  static const int16_t last[14] = {166, 181, 195, 210, 213, 417, 572, 587, 601, 690, 616, 631, 645, 748};
  static const int16_t abs_[14] = {227, 237, 247, 257, 266, 426, 952, 962, 972, 708, 982, 992, 1002, 766};
  // dense SIG estimator base per ctxBlockCat: 4096 per 4x4-class cat, 61440 for 8x8 cats (5, 9, 13)
  static const int32_t seb[14] = {0, 4096, 8192, 12288, 16384, 20480, 81920, 86016, 90112,
                                  94208, 155648, 159744, 163840, 167936};
  static const uint8_t sig8[63] = {
    0, 1, 2, 3, 4, 5, 5, 4, 4, 3, 3, 4, 4, 4, 5, 5, 4, 4, 4, 4, 3, 3, 6, 7, 7, 7, 8, 9, 10, 9, 8, 7,
    7, 6, 11, 12, 13, 11, 6, 7, 8, 9, 14, 10, 9, 8, 6, 11, 12, 13, 11, 6, 9, 14, 10, 9, 11, 12, 13, 11, 14, 10, 12};
  static const uint8_t last8[63] = {
    0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
    3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8};
  for (int c = 0; c < 14; c++) {
    t->hot.cbf_base[c] = cbf[c];
    t->hot.sig_base[c] = sig[c];
    t->hot.last_base[c] = last[c];
    t->hot.abs_base[c] = abs_[c];
    t->hot.sig_est_base[c] = seb[c];
  }
  for (int i = 0; i < 63; i++) {
    t->hot.sig8x8[i] = sig8[i];
    t->hot.last8x8[i] = last8[i];
  }
  // field coded (FFmpeg significant_coeff_flag_offset[1], last_coeff_flag_offset[1],
  // significant_coeff_flag_offset_8x8[1] == recode.cpp:691-694)
  static const int16_t sig_f[14] = {277, 292, 306, 321, 324, 436, 776, 791, 805, 675, 820, 835, 849, 733};
  static const int16_t last_f[14] = {338, 353, 367, 382, 385, 451, 864, 879, 893, 699, 908, 923, 937, 757};
  static const uint8_t sig8_f[63] = {
    0, 1, 1, 2, 2, 3, 3, 4, 5, 6, 7, 7, 7, 8, 4, 5, 6, 9, 10, 10, 8, 11, 12, 11, 9, 9, 10, 10, 8, 11, 12, 11,
    9, 9, 10, 10, 8, 11, 12, 11, 9, 9, 10, 10, 8, 13, 13, 9, 9, 10, 10, 8, 13, 13, 9, 9, 10, 10, 14, 14, 14, 14, 14};
  for (int c = 0; c < 14; c++) {
    t->sig_base_fld[c] = sig_f[c];
    t->last_base_fld[c] = last_f[c];
  }
  for (int i = 0; i < 63; i++) t->sig8x8_fld[i] = sig8_f[i];
  const double alpha = std::pow(0.01875 / 0.5, 1.0 / 63.0);
  for (int s = 0; s < 64; s++) t->gen_plps[s] = (uint16_t)std::lround(65536.0 * 0.5 * std::pow(alpha, s));
}

bool check_reciprocals(const avr::EngineTables& t) {
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (uint32_t d = 2; d < 128; d++) {
    auto q = [&](uint64_t v) -> uint64_t {
      return (uint64_t)(((unsigned __int128)v * t.hot.div[d][0]) >> 64) >> t.hot.div[d][1];
    };
    const uint64_t edge[] = {0, 1, d - 1, d, d + 1, (1ull << 63) - 1, 1ull << 63, (1ull << 62) + 12345};
    for (uint64_t v : edge)
      if (q(v) != v / d) return false;
    for (int k = 0; k < 4000; k++) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      uint64_t v = x >> 1;
      uint64_t m = (v / d) * d;
      if (q(v) != v / d || q(m) != m / d || (m && q(m - 1) != (m - 1) / d)) return false;
    }
  }
  return true;
}

// A byte vector whose resize() leaves new bytes uninitialised (multi-GB buffers that are written
// right after: no memset pass first).
template <class T>
struct DefaultInit : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = DefaultInit<U>;
  };
  DefaultInit() = default;
  template <class U>
  DefaultInit(const DefaultInit<U>&) {}
  template <class U>
  void construct(U* p) {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};
typedef std::vector<uint8_t, DefaultInit<uint8_t>> Bytes;

struct Plan {
  std::vector<avr_slice_desc> descs;
  Bytes arena;   // payloads (compress) or recoded streams (decompress)
  // decompress_setup with layout_only: the arena is not built; its byte copies are listed in
  // arena_copies (dst in the arena, source in the container) and its length in arena_end
  bool layout_only = false;
  std::vector<avr::PbCopy> arena_copies;
  uint64_t arena_end = 0;
  int max_w = 1;
  // sequential (reference-model) plans over several files: file f is descs[file_first[f] ..
  // file_first[f + 1]); empty = one file
  std::vector<int> file_first;
  int n_files() const { return file_first.empty() ? 1 : (int)file_first.size() - 1; }
  int file_begin(int f) const { return file_first.empty() ? 0 : file_first[f]; }
  int file_end(int f) const { return file_first.empty() ? (int)descs.size() : file_first[f + 1]; }
  // field pictures / MBAFF frames present: launches add the field-capable kernels (kFlagFields)
  bool fields() const {
    for (const auto& d : descs)
      if (d.structure != AVR_STRUCT_FRAME) return true;
    return false;
  }
  // both kinds of slice: the field kernel has work beside the progressive one (avr::FieldLane)
  bool mixed() const {
    bool f = false, p = false;
    for (const auto& d : descs) (d.structure != AVR_STRUCT_FRAME ? f : p) = true;
    return f && p;
  }
};

template <class V>
void append_aligned(V* arena, const uint8_t* p, size_t n, size_t extra, uint64_t* off) {
  size_t o = (arena->size() + 15) & ~(size_t)15;
  arena->resize(o + n + extra, 0);
  if (n) memcpy(arena->data() + o, p, n);
  *off = o;
}

// EdgeRec slots of the LDS ring a slice needs (launch max_mb_width): an MBAFF slice keeps its pair
// edges and records there too (Walker::pair_edge)
int ring_cols(const avr_slice_desc& d) { return d.structure == AVR_STRUCT_MBAFF ? 3 * d.mb_width + 7 : d.mb_width; }

avr_slice_desc desc_from_header(const avr::SliceInfo& s) {
  avr_slice_desc d;
  memset(&d, 0, sizeof(d));
  d.slice_type = s.h.slice_type == 3 ? 0 : s.h.slice_type == 4 ? 2 : s.h.slice_type;
  d.slice_qp = s.h.slice_qp;
  d.cabac_init_idc = s.h.cabac_init_idc;
  d.first_mb = s.h.first_mb;
  d.mb_width = s.h.mb_width;
  d.mb_height = s.h.mb_height;
  d.num_ref_idx_l0 = s.h.num_ref_idx[0];
  d.num_ref_idx_l1 = s.h.num_ref_idx[1];
  d.chroma_array_type = s.h.chroma_array_type;
  d.transform_8x8_mode = s.h.transform_8x8_mode;
  d.direct_8x8_inference = s.h.direct_8x8_inference;
  d.x264_build = s.h.x264_build;
  d.picture_id = s.picture_id;
  d.coded = 1;
  d.file_offset = ~(uint64_t)0;
  d.structure = s.h.field_pic ? (s.h.bottom_field ? AVR_STRUCT_BOTTOM_FIELD : AVR_STRUCT_TOP_FIELD)
              : s.h.mbaff ? AVR_STRUCT_MBAFF : AVR_STRUCT_FRAME;
  return d;
}

constexpr int kRModeFallback = 1;

// Does the parallel reference-model compress beat one workgroup per file on this plan?  Its time is
// its largest slice's: the scan twice (count, write) and the recoded coder, one after the other;
// the sequential kernel's is its largest file's, with walker, modeler and coder overlapped on three
// waves.  Measured per payload byte of the chain (profiles/r05_rcode_ab.txt and
// r05m_rmode_files_before.log: a 4K 4:4:4 slice of 1.38 MB, scan 1.3-1.8 s per pass, coder ~1.5 s
// per MB; the per-file kernel's compress of a 2-slice such file 1.4 s per MB): the parallel pass
// pays when the largest file's payload exceeds ~3.7 times the largest slice's (cockatoo.mp4: 280
// slices; a 1-2-slice-per-picture 4K file does not).
// AVR_RMODE_PARALLEL=1 forces the parallel pass (tests), AVR_RMODE_SEQUENTIAL=1 the sequential kernel.
bool rmode_parallel_pays(const Plan& plan) {
  if (getenv("AVR_RMODE_PARALLEL")) return true;
  const int nf = plan.n_files(), n = (int)plan.descs.size();
  uint64_t max_slice = 0, max_file = 0;
  for (int f = 0; f < nf; f++) {
    const int e = f + 1 < nf ? plan.file_begin(f + 1) : n;
    uint64_t fs = 0;
    for (int k = plan.file_begin(f); k < e; k++) {
      const uint64_t s = plan.descs[k].coded ? plan.descs[k].payload_size : 0;
      fs += s;
      max_slice = std::max(max_slice, s);
    }
    max_file = std::max(max_file, fs);
  }
  return max_file * 10 > max_slice * 37;
}

// Reference-model compress of a plan (file order) in parallel over slices (avr_k_rmode.hip).
// Frame metadata generations mirror update_frame_spec (recode.cpp:824-843) as
// slices_sequential_kernel implements it; a stream whose frame size changes with a stale other
// frame is left to the sequential kernel (kRModeFallback), as is a plan too large for one pass.
int run_rmode_compress(avr_ctx* c, Plan& plan, uint64_t out_total, uint32_t flags) {
  const int n = (int)plan.descs.size();
  const int nf = plan.n_files();
  if (nf > avr::rmode_max_files_per_pass()) return kRModeFallback;
  struct Fb { int gen = -1, w = 0, h = 0, fid = 0; } fb[2];
  std::vector<uint8_t> gen_parity;   // field parities (1 top, 2 bottom) seen per frame generation
  int cur = 0;
  std::vector<int64_t> gen_off, goff(2 * (size_t)n);
  int64_t fbytes = 0;
  std::vector<char> file_start(n + 1, 0);
  for (int f = 0; f < nf; f++) file_start[plan.file_begin(f)] = 1;
  for (int k = 0; k < n; k++) {
    if (file_start[k]) {   // a new file: a fresh model, frames of its own
      fb[0] = Fb();
      fb[1] = Fb();
      cur = 0;
    }
    const avr_slice_desc& d = plan.descs[k];
    const int W = d.mb_width, H = d.mb_height;
    if (fb[cur].w != W || fb[cur].h != H || !(fb[cur].fid == d.picture_id && fb[cur].w && fb[cur].h)) {
      cur = 1 - cur;
      Fb& nw = fb[cur];
      Fb& ot = fb[1 - cur];
      const bool reinit_other = (nw.w != W || nw.h != H) && (ot.w != W || ot.h != H);
      nw.gen = (int)gen_off.size();
      gen_off.push_back(fbytes);
      gen_parity.push_back(0);
      fbytes += (int64_t)W * H * 52;
      if (reinit_other) {
        ot.gen = -1;
        ot.w = W;
        ot.h = H;
      }
      nw.w = W;
      nw.h = H;
      nw.fid = d.picture_id;
    }
    const Fb& ot = fb[1 - cur];
    if (ot.gen >= 0 && (ot.w != W || ot.h != H)) return kRModeFallback;
    goff[2 * k] = gen_off[fb[cur].gen];
    goff[2 * k + 1] = ot.gen < 0 ? -1 : gen_off[ot.gen];
    // a field whose frame has no slice of the other parity yet (its rows are still zero in the
    // sequential model, but filled in the buffer the parallel scan reads): offsets are 4-aligned
    if (d.structure == AVR_STRUCT_TOP_FIELD || d.structure == AVR_STRUCT_BOTTOM_FIELD) {
      uint8_t& seen = gen_parity[fb[cur].gen];
      if (!(seen & (d.structure == AVR_STRUCT_TOP_FIELD ? 2 : 1))) goff[2 * k] |= 1;
      seen |= (uint8_t)(d.structure == AVR_STRUCT_TOP_FIELD ? 1 : 2);
    }
  }
  if (fbytes > ((int64_t)4 << 30)) return kRModeFallback;
  const size_t lds = avr::shared_bytes(plan.max_w);
  HIP_TRY(c, c->frames.reserve((size_t)fbytes + 64));
  HIP_TRY(c, hipMemsetAsync(c->frames.p, 0, (size_t)fbytes + 64, c->stream));
  HIP_TRY(c, c->rm_goff.reserve(sizeof(int64_t) * goff.size()));
  HIP_TRY(c, hipMemcpyAsync(c->rm_goff.p, goff.data(), sizeof(int64_t) * goff.size(), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, c->rm_counts.reserve(sizeof(uint32_t) * n));
  HIP_TRY(c, c->rm_stop.reserve(sizeof(int32_t) * n));
  HIP_TRY(c, c->rm_off.reserve(sizeof(uint64_t) * (n + 1)));
  // 1) count the model ops (and fill the frame metadata)
  HIP_TRY(c, avr::launch_rscan(c->tables.as<avr::EngineTables>(), c->descs.as<avr_slice_desc>(), n, lds,
                               c->in.as<uint8_t>(), c->frames.as<uint8_t>(), c->rm_goff.as<int64_t>(),
                               c->rm_counts.as<uint32_t>(), nullptr, nullptr, c->res.as<avr_slice_result>(),
                               c->rm_stop.as<int32_t>(), plan.fields(), c->stream));
  std::vector<uint32_t> counts(n);
  HIP_TRY(c, hipMemcpyAsync(counts.data(), c->rm_counts.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  std::vector<uint64_t> off(n + 1, 0);
  for (int k = 0; k < n; k++) off[k + 1] = off[k] + counts[k];
  const uint64_t N = off[n];
  if (getenv("AVR_RMODE_STATS")) {
    uint64_t pay = 0;
    uint32_t mx = 0;
    double mxr = 0;
    for (int k = 0; k < n; k++) {
      pay += plan.descs[k].payload_size;
      mx = std::max(mx, counts[k]);
      if (plan.descs[k].payload_size > 0) mxr = std::max(mxr, (double)counts[k] / plan.descs[k].payload_size);
    }
    fprintf(stderr, "rmode: %d slices, %llu ops, %llu payload bytes (%.2f ops/B, max slice %u ops, max %.1f ops/B)\n",
            n, (unsigned long long)N, (unsigned long long)pay, pay ? (double)N / pay : 0.0, mx, mxr);
  }
  if (N >= (1ull << 31) - 1) return kRModeFallback;   // hipCUB's item count is an int
  HIP_TRY(c, hipMemcpyAsync(c->rm_off.p, off.data(), sizeof(uint64_t) * (n + 1), hipMemcpyHostToDevice, c->stream));
  std::vector<uint64_t> fop(nf + 1);
  for (int f = 0; f <= nf; f++) fop[f] = off[f < nf ? plan.file_begin(f) : n];
  HIP_TRY(c, c->file_op_off.reserve(sizeof(uint64_t) * (nf + 1)));
  HIP_TRY(c, hipMemcpyAsync(c->file_op_off.p, fop.data(), sizeof(uint64_t) * (nf + 1), hipMemcpyHostToDevice,
                            c->stream));
  const size_t tb = avr::rmode_sort_temp_bytes(N, nf);
  // ops, keys, skeys, rops: 4 B per op; vals, svals: 8 B (op index << 2 | flags)
  HIP_TRY(c, c->rm_ops.reserve(sizeof(uint32_t) * (N + 1) * 8 + tb + 256));
  uint32_t* ops = c->rm_ops.as<uint32_t>();
  uint32_t* keys = ops + (N + 1);
  uint32_t* skeys = keys + (N + 1);
  uint32_t* rops = skeys + (N + 1);
  uint64_t* vals = (uint64_t*)(rops + (N + 1));
  uint64_t* svals = vals + (N + 1);
  void* temp = (void*)(((uintptr_t)(svals + (N + 1)) + 255) & ~(uintptr_t)255);
  // 2) write the ops, 3) estimator chains, 4) per-slice coder
  HIP_TRY(c, avr::launch_rscan(c->tables.as<avr::EngineTables>(), c->descs.as<avr_slice_desc>(), n, lds,
                               c->in.as<uint8_t>(), c->frames.as<uint8_t>(), c->rm_goff.as<int64_t>(),
                               c->rm_counts.as<uint32_t>(), ops, c->rm_off.as<uint64_t>(),
                               c->res.as<avr_slice_result>(), c->rm_stop.as<int32_t>(), plan.fields(), c->stream));
  HIP_TRY(c, avr::launch_rmode_estimators(ops, N, c->file_op_off.as<uint64_t>(), nf, keys, vals, skeys, svals, temp,
                                          tb, rops, c->stream));
  HIP_TRY(c, avr::launch_rcode(c->tables.as<avr::EngineTables>(), c->descs.as<avr_slice_desc>(), n, rops,
                               c->rm_off.as<uint64_t>(), c->rm_counts.as<uint32_t>(), c->out.as<uint8_t>(),
                               c->res.as<avr_slice_result>(), c->rm_stop.as<int32_t>(), flags, c->stream));
  (void)out_total;
  return AVR_OK;
}

// Device scratch of a parallel launch of n slices: the estimator tables (one per slice of a resident
// batch, one per workgroup of a persistent one: avr::est_slots), the CU schedule and the slice queue.
hipError_t reserve_parallel(avr_ctx* c, int n, int max_w, bool field_lane = false) {
  const int slots = std::max(1, avr::est_slots(n, max_w, field_lane));
  hipError_t e = c->est.reserve(sizeof(uint16_t) * (size_t)avr::kEstGlobal * slots, true);
  if (e == hipSuccess) e = c->order.reserve(sizeof(int) * (size_t)std::max(1, n));
  if (e == hipSuccess) e = c->queue.reserve(std::max<size_t>(256, avr::queue_scratch_bytes(n)));
  return e;
}

// Upload plan, run the slice kernel over it (one launch, see launch_slices), download results and outputs.
// verify (parallel compress only): also decompress every slice's output on the device, apply the
// last-byte rule and compare with the payload (avr_roundtrip_slices); a slice whose output does not
// regenerate its payload gets status kStatusNoRoundtrip, so no container ever holds a block that
// cannot be decompressed.
constexpr int32_t kStatusNoRoundtrip = AVR_SLICE_NO_ROUNDTRIP;
// out_host: a std::vector<uint8_t> or a Bytes (not zero-filled first: the download overwrites it)
template <class HostBuf>
int run_plan(avr_ctx* c, int mode, bool sequential, Plan& plan, std::vector<avr_slice_result>* res,
             HostBuf* out_host, bool verify = false, uint32_t flags = 0) {
  const int n = (int)plan.descs.size();
  if (plan.fields()) flags |= avr::kFlagFields;
  // a parallel batch of progressive and field slices: the two kernels side by side
  const avr::FieldLane lane = !sequential && plan.mixed() ? c->field_lane() : avr::FieldLane();
  res->assign(n, avr_slice_result{0, 0, 0, 0, {0, 0, 0, 0, 0, 0}});
  uint64_t out_total = 0;
  for (auto& d : plan.descs) {
    d.out_offset = out_total;
    out_total += ((uint64_t)d.out_capacity + 15) & ~15ull;
  }
  out_host->resize(out_total);
  if (!n) return AVR_OK;
  const double t_wall = now_s();
  HIP_TRY(c, c->in.reserve(plan.arena.size() + 4096));
  HIP_TRY(c, c->out.reserve(out_total + 4096));
  HIP_TRY(c, c->descs.reserve(sizeof(avr_slice_desc) * n));
  HIP_TRY(c, c->res.reserve(sizeof(avr_slice_result) * n));
  for (auto& e : c->ev)
    if (!e) HIP_TRY(c, hipEventCreate(&e));
  HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->in.p, plan.arena.data(), plan.arena.size(), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->descs.p, plan.descs.data(), sizeof(avr_slice_desc) * n, hipMemcpyHostToDevice,
                            c->stream));
  HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
  int rm = kRModeFallback;
  if (sequential && mode == 0 && !getenv("AVR_RMODE_SEQUENTIAL") && rmode_parallel_pays(plan)) {
    rm = run_rmode_compress(c, plan, out_total, flags);
    if (rm < 0) return rm;
  }
  if (sequential && rm == AVR_OK) {
    // done: the parallel reference-model compress
  } else if (sequential) {
    // one workgroup per file (the reference model is sequential within a file only)
    const int nf = plan.n_files();
    avr::SeqFiles sf;
    sf.n_files = nf;
    size_t fbytes = 0;
    for (auto& d : plan.descs) fbytes = std::max(fbytes, (size_t)2 * d.mb_width * d.mb_height * 52);
    sf.frame_stride = (fbytes + 255) & ~(size_t)255;
    HIP_TRY(c, c->est.reserve(sizeof(uint16_t) * avr::kEstGlobal * (size_t)nf, true));
    HIP_TRY(c, c->frames.reserve(sf.frame_stride * nf + 64));
    HIP_TRY(c, c->frame_meta.reserve(sizeof(int) * (size_t)nf + 64));
    if (!plan.file_first.empty()) {
      HIP_TRY(c, c->file_first.reserve(sizeof(int) * plan.file_first.size()));
      HIP_TRY(c, hipMemcpyAsync(c->file_first.p, plan.file_first.data(), sizeof(int) * plan.file_first.size(),
                                hipMemcpyHostToDevice, c->stream));
      sf.file_first = c->file_first.as<int>();
    }
    HIP_TRY(c, avr::launch_slices(mode, true, c->tables.as<avr::EngineTables>(), c->descs.as<avr_slice_desc>(), n,
                                  plan.max_w, c->in.as<uint8_t>(), c->out.as<uint8_t>(), c->res.as<avr_slice_result>(),
                                  c->est.as<uint16_t>(), c->frames.as<uint8_t>(), c->frame_meta.as<int>(), nullptr,
                                  c->stream, sf, flags));
  } else {
    HIP_TRY(c, reserve_parallel(c, n, plan.max_w, lane.stream != nullptr));
    HIP_TRY(c, avr::launch_slices(mode, false, c->tables.as<avr::EngineTables>(), c->descs.as<avr_slice_desc>(), n,
                                  plan.max_w, c->in.as<uint8_t>(), c->out.as<uint8_t>(), c->res.as<avr_slice_result>(),
                                  c->est.as<uint16_t>(), nullptr, nullptr, c->order_or_null(), c->stream,
                                  avr::SeqFiles(), flags, c->queue.p, &lane));
  }
  std::vector<int32_t> verdict;
  if (verify && mode == 0 && !sequential) {
    HIP_TRY(c, c->regen.reserve(plan.arena.size() + 4096));
    HIP_TRY(c, c->dec_descs.reserve(sizeof(avr_slice_desc) * n));
    HIP_TRY(c, c->res_d.reserve(sizeof(avr_slice_result) * n));
    HIP_TRY(c, c->verdict.reserve(sizeof(int32_t) * n));
    avr_slice_desc* dd = c->dec_descs.as<avr_slice_desc>();
    avr_slice_result* rd = c->res_d.as<avr_slice_result>();
    HIP_TRY(c, avr::launch_derive_decompress(c->descs.as<avr_slice_desc>(), c->res.as<avr_slice_result>(), n, dd,
                                             c->stream));
    HIP_TRY(c, avr::launch_slices(1, false, c->tables.as<avr::EngineTables>(), dd, n, plan.max_w, c->out.as<uint8_t>(),
                                  c->regen.as<uint8_t>(), rd, c->est.as<uint16_t>(), nullptr, nullptr,
                                  c->order_or_null(), c->stream, avr::SeqFiles(),
                                  (plan.fields() ? avr::kFlagFields : 0u) | (flags & avr::kFlagP32), c->queue.p,
                                  &lane));
    HIP_TRY(c, avr::launch_verify(c->descs.as<avr_slice_desc>(), c->res.as<avr_slice_result>(), rd, n,
                                  c->in.as<uint8_t>(), c->regen.as<uint8_t>(), c->verdict.as<int32_t>(), c->stream));
    verdict.resize(n);
    HIP_TRY(c, hipMemcpyAsync(verdict.data(), c->verdict.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipEventRecord(c->ev[2], c->stream));
  HIP_TRY(c, hipMemcpyAsync(res->data(), c->res.p, sizeof(avr_slice_result) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(out_host->data(), c->out.p, out_total, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  float ms[3] = {0, 0, 0};
  for (int i = 0; i < 3; i++) HIP_TRY(c, hipEventElapsedTime(&ms[i], c->ev[i], c->ev[i + 1]));
  c->phase.upload_s += 1e-3 * ms[0];
  c->phase.kernel_s += 1e-3 * ms[1];
  c->phase.download_s += 1e-3 * ms[2];
  c->plan_wall += now_s() - t_wall;
  for (int k = 0; k < (int)verdict.size(); k++)
    if ((*res)[k].status == 0 && verdict[k] != 1) (*res)[k].status = kStatusNoRoundtrip;
  return AVR_OK;
}

// ------------------------------------------------------------------------ the long-slice split
// The parallel model (on arithmetic_code<uint64_t, uint8_t>) cuts a long progressive slice at
// macroblock-row starts into pieces re-coded with fresh models, so its decompress runs one workgroup
// per piece instead of one chain (the reference decodes a slice as one chain, recode.cpp:1411-1520).
// The format is this library's own, restated and checked by the oracle (oracle/oracle_seams.c,
// avr_oracle.h):
//   - a cut candidate every 8 split_bytes CABAC bits decoded (at a row start, half a piece still
//     ahead); it becomes a cut where the re-encoder's state can be placed (seam_encoder) -- the
//     byte form of the arithmetic's low L = V - codIOffset, V the payload's first bitpos bits;
//   - each piece has its own re-coded stream (Block.cabac holds them one after the other) and starts
//     with a fresh model whose upper row of model bytes is zero;
//   - Block field 16 ("seams", zlib) carries, per cut, what the piece after it needs: its first
//     macroblock, its first output byte q, the re-encoder state, the CABAC contexts, last_dqp_nz
//     and the upper row's edges (the parse's neighbour fields).
// Compress takes the long slices through the split kernels twice (avr_k_split.hip): the cut scan --
// the CABAC parse of each whole slice alone (a trace walk without output: no model, one wave),
// recording the candidates, on its own stream beside the rest of the batch -- then the pieces (a
// slice without a cut: one piece).  Decompress runs the pieces side by side and splices them: piece
// i's bytes up to cut i's q.
constexpr size_t kSplitBytesDefault = 98304;

bool split_candidate(const avr_slice_desc& d, size_t split_bytes) {
  return split_bytes && split_bytes < ((size_t)1 << 28) && d.structure == AVR_STRUCT_FRAME &&
         d.mb_width <= avr::kMringCols && 2 * (uint64_t)d.payload_size >= 3 * (uint64_t)split_bytes;
}

struct SeamCe {
  uint32_t q, low, outstanding, cache, range;
  int32_t queue;
};
// The re-encoder where the decoder stands after bitpos bits with codIOffset `offset` (the oracle's
// avr_seam_encoder): m = (bitpos - 10) / 8 whole bytes have left the window; the last byte of L
// below m that is not 0xFF (q) is the cache, the 0xFF bytes after it outstanding, the rest in low.
bool seam_encoder(const uint8_t* pay, size_t n, uint64_t bitpos, uint32_t offset, uint32_t range, SeamCe* s) {
  if (bitpos < 26) return false;
  const uint64_t m = (bitpos - 10) / 8, sb = m > 12 ? m - 12 : 0, e = (bitpos + 7) / 8;
  unsigned __int128 x = 0;
  for (uint64_t j = sb; j < e; j++) x = x << 8 | (j < n ? pay[j] : 0);
  x >>= 8 * e - bitpos;
  if (x < offset) return false;
  const unsigned __int128 y = x - offset;
  for (uint64_t j = m; j-- > sb;) {
    const uint32_t b = (uint32_t)(y >> (bitpos - 8 * j - 8)) & 0xff;
    if (b == 0xff) continue;
    const unsigned lowbits = (unsigned)(bitpos - 8 * m);
    s->q = (uint32_t)j;
    s->cache = b;
    s->outstanding = (uint32_t)(m - 1 - j);
    s->low = (uint32_t)(y & (((unsigned __int128)1 << lowbits) - 1));
    s->queue = (int32_t)lowbits - 18;
    s->range = range;
    return true;
  }
  return false;
}

void put_le32(std::vector<uint8_t>* o, uint32_t v) {
  for (int k = 0; k < 4; k++) o->push_back((uint8_t)(v >> (8 * k)));
}
uint32_t get_le32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// The slice's initial context states (9.3.1.1), as init_slice_state sets them on the device.
void cabac_init_states(const avr_slice_desc& d, uint8_t out[1024]) {
  const int qp = d.slice_qp < 0 ? 0 : d.slice_qp > 51 ? 51 : d.slice_qp;
  for (int c = 0; c < 1024; c++) {
    int m, n;
    avr::mn_for_ctx(d.slice_type == 2 ? -1 : d.cabac_init_idc, c, &m, &n);
    int pre = ((m * qp) >> 4) + n;
    pre = pre < 1 ? 1 : pre > 126 ? 126 : pre;
    out[c] = pre <= 63 ? (uint8_t)((63 - pre) << 1) : (uint8_t)(((pre - 64) << 1) | 1);
  }
}
// an upper-row edge byte as the seams field keeps it: what the parse of the row below reads of it --
// nnz only as nonzero (coded_block_flag's context), |mvd| only up to 33 (absMvdComp's sum against
// 3 and 32)
uint8_t edge_norm(int j, uint8_t b) {
  if (j >= 4 && j < 16) return b != 0;
  if (j >= 16 && j < 32) return b > 33 ? 33 : b;
  return b;
}

// Block field 16: u32 raw length, then zlib (level 9) of { u32 2, u32 cuts, u32 mb_width,
// u32 piece_len[cuts + 1], per cut { u32 first_mb, q, last_dqp_nz, ce_low, ce_queue,
// ce_outstanding, ce_cache, ce_range, u8 state[1024] XOR the slice's initial states, u8 edges
// byte-major (byte j of every column, j = 0..39; edge_norm) } } (little-endian)
bool seams_encode(const std::vector<const avr::SeamRec*>& recs, const std::vector<SeamCe>& ce, const avr_slice_desc& d,
                  const std::vector<uint32_t>& piece_len, std::vector<uint8_t>* out) {
  const int mb_width = d.mb_width;
  uint8_t init[1024];
  cabac_init_states(d, init);
  std::vector<uint8_t> raw;
  put_le32(&raw, 2);
  put_le32(&raw, (uint32_t)recs.size());
  put_le32(&raw, (uint32_t)mb_width);
  for (uint32_t l : piece_len) put_le32(&raw, l);
  for (size_t i = 0; i < recs.size(); i++) {
    put_le32(&raw, recs[i]->first_mb);
    put_le32(&raw, ce[i].q);
    put_le32(&raw, recs[i]->last_dqp_nz);
    put_le32(&raw, ce[i].low);
    put_le32(&raw, (uint32_t)ce[i].queue);
    put_le32(&raw, ce[i].outstanding);
    put_le32(&raw, ce[i].cache);
    put_le32(&raw, ce[i].range);
    for (int c = 0; c < 1024; c++) raw.push_back((uint8_t)(recs[i]->state[c] ^ init[c]));
    const uint8_t* e = (const uint8_t*)(recs[i] + 1);
    for (int j = 0; j < avr::kEdgeBytes; j++)
      for (int c = 0; c < mb_width; c++) raw.push_back(edge_norm(j, e[(size_t)avr::kEdgeBytes * c + j]));
  }
  uLongf zl = compressBound(raw.size());
  out->assign(4 + zl, 0);
  if (compress2(out->data() + 4, &zl, raw.data(), raw.size(), 9) != Z_OK) return false;
  out->resize(4 + zl);
  for (int k = 0; k < 4; k++) (*out)[k] = (uint8_t)(raw.size() >> (8 * k));
  return true;
}

// the pieces of a split block: per cut a device record (decompress fields), the pieces' streams
struct SeamsDecoded {
  int cuts = 0;
  std::vector<uint32_t> piece_len, first_mb, q;
  std::vector<uint8_t> recs;   // cuts records of rec_stride bytes
};
bool seams_decode(const uint8_t* p, size_t n, const avr_slice_desc& d, size_t rec_stride, SeamsDecoded* sd) {
  const int mb_width = d.mb_width;
  uint8_t init[1024];
  cabac_init_states(d, init);
  if (n < 4) return false;
  const uint32_t rl = get_le32(p);
  if (rl < 12 || rl > (1u << 30)) return false;
  std::vector<uint8_t> raw(rl);
  uLongf got = rl;
  if (uncompress(raw.data(), &got, p + 4, n - 4) != Z_OK || got != rl || get_le32(raw.data()) != 2) return false;
  const uint32_t k = get_le32(raw.data() + 4), w = get_le32(raw.data() + 8);
  const size_t per = 32 + 1024 + (size_t)avr::kEdgeBytes * w;
  if ((int)w != mb_width || k == 0 || k > 65536 || 12 + 4 * ((size_t)k + 1) + per * k != rl) return false;
  sd->cuts = (int)k;
  const uint8_t* q = raw.data() + 12;
  sd->piece_len.resize(k + 1);
  for (uint32_t i = 0; i <= k; i++, q += 4) sd->piece_len[i] = get_le32(q);
  sd->recs.assign((size_t)k * rec_stride, 0);
  sd->first_mb.resize(k);
  sd->q.resize(k);
  for (uint32_t i = 0; i < k; i++, q += per) {
    avr::SeamRec* r = (avr::SeamRec*)(sd->recs.data() + (size_t)i * rec_stride);
    r->first_mb = sd->first_mb[i] = get_le32(q);
    sd->q[i] = get_le32(q + 4);
    r->last_dqp_nz = get_le32(q + 8);
    r->ce_low = get_le32(q + 12);
    r->ce_queue = (int32_t)get_le32(q + 16);
    r->ce_outstanding = get_le32(q + 20);
    r->ce_cache = get_le32(q + 24);
    r->ce_range = get_le32(q + 28);
    // a cut's state is what seam_encoder can produce: the window 12 bytes deep at most
    if (r->ce_queue < -8 || r->ce_queue > -1 || r->ce_cache > 0xff || r->ce_range < 256 || r->ce_range > 510 ||
        r->ce_low >= (1u << (r->ce_queue + 18)) || r->ce_outstanding > 12 || (i && sd->q[i] <= sd->q[i - 1]) ||
        (i && sd->first_mb[i] <= sd->first_mb[i - 1]) || sd->first_mb[i] % w ||
        sd->first_mb[i] >= (uint32_t)w * (uint32_t)std::max(1, d.mb_height))
      return false;
    for (int c = 0; c < 1024; c++) r->state[c] = (uint8_t)(q[32 + c] ^ init[c]);
    uint8_t* e = (uint8_t*)(r + 1);
    for (int j = 0; j < avr::kEdgeBytes; j++)
      for (uint32_t c = 0; c < w; c++) e[(size_t)avr::kEdgeBytes * c + j] = q[32 + 1024 + (size_t)j * w + c];
  }
  return true;
}

// Compress of the long slices, in two calls around the rest of the batch: begin uploads them and
// launches the split compress on the split stream (each slice cut as it is walked: the records,
// the pieces' streams one after the other, their ends); finish checks every cut against the host's
// restatement of the re-encoder state, and (verify) decompresses the pieces and compares.
struct SplitOut {
  int32_t status = 0;
  std::vector<uint8_t> recoded, seams;   // seams empty: no cut
  avr_slice_result bill{};
};
struct SplitJob {
  std::vector<const avr::SliceInfo*> sl;
  std::vector<avr_slice_desc> d;
  std::vector<avr::PieceCtl> ctl;
  Bytes arena;
  uint64_t out_total = 0;
  uint32_t nrec = 0, split_bits = 0;
  size_t stride = 0;
  int max_w = 1;
  uint32_t flags = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
};

int split_begin(avr_ctx* c, SplitJob* j, size_t split_bytes, uint32_t flags) {
  const int n = (int)j->sl.size();
  if (!n) return AVR_OK;
  j->flags = flags & avr::kFlagBill;
  j->split_bits = (uint32_t)(8 * split_bytes);
  j->d.resize(n);
  j->ctl.resize(n);
  for (int k = 0; k < n; k++) {
    const avr::SliceInfo& s = *j->sl[k];
    avr_slice_desc& d = j->d[k];
    d = desc_from_header(s);
    append_aligned(&j->arena, s.payload(), s.read_limit, 16, &d.payload_offset);
    d.payload_size = (uint32_t)s.size;
    d.read_limit = (uint32_t)s.read_limit;
    const uint32_t cap = (uint32_t)(8ull * s.size / j->split_bits) + 1;
    d.out_capacity = (uint32_t)(s.size * 2 + 256 + 64 * (size_t)cap);
    d.out_offset = j->out_total;
    j->out_total += ((uint64_t)d.out_capacity + 15) & ~15ull;
    j->max_w = std::max(j->max_w, d.mb_width);
    j->ctl[k] = avr::PieceCtl{-1, 0, (int32_t)j->nrec, cap};
    j->nrec += cap;
  }
  j->stride = avr::seam_rec_bytes(j->max_w);
  const int grid = avr::split_grid(n, j->max_w);
  HIP_TRY(c, c->sp_in.reserve(j->arena.size() + 4096));
  HIP_TRY(c, c->sp_out.reserve(j->out_total + 4096));
  HIP_TRY(c, c->sp_descs.reserve(sizeof(avr_slice_desc) * n));
  HIP_TRY(c, c->sp_res.reserve(sizeof(avr_slice_result) * n));
  HIP_TRY(c, c->sp_ctl.reserve(sizeof(avr::PieceCtl) * n));
  HIP_TRY(c, c->sp_recs.reserve(j->stride * j->nrec + 64));
  HIP_TRY(c, c->sp_snapn.reserve(sizeof(uint32_t) * ((size_t)n + j->nrec)));
  HIP_TRY(c, c->sp_est.reserve(sizeof(uint16_t) * (size_t)avr::kEstGlobal * std::max(1, grid), true));
  HIP_TRY(c, hipEventCreate(&j->e0));
  HIP_TRY(c, hipEventCreate(&j->e1));
  hipStream_t st = c->split_stream;
  HIP_TRY(c, hipMemcpyAsync(c->sp_in.p, j->arena.data(), j->arena.size(), hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(c->sp_descs.p, j->d.data(), sizeof(avr_slice_desc) * n, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(c->sp_ctl.p, j->ctl.data(), sizeof(avr::PieceCtl) * n, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemsetAsync(c->sp_snapn.p, 0, sizeof(uint32_t) * ((size_t)n + j->nrec), st));
  avr::SplitArgs sa;
  sa.ctl = c->sp_ctl.as<avr::PieceCtl>();
  sa.recs = c->sp_recs.as<uint8_t>();
  sa.rec_stride = (uint32_t)j->stride;
  sa.split_bits = j->split_bits;
  sa.snap_n = c->sp_snapn.as<uint32_t>();
  sa.piece_end = sa.snap_n + n;
  HIP_TRY(c, hipEventRecord(j->e0, st));
  HIP_TRY(c, avr::launch_split(0, c->tables.as<avr::EngineTables>(), c->sp_descs.as<avr_slice_desc>(), n, j->max_w,
                               c->sp_in.as<uint8_t>(), c->sp_out.as<uint8_t>(), c->sp_res.as<avr_slice_result>(),
                               c->sp_est.as<uint16_t>(), sa, j->flags, st));
  HIP_TRY(c, hipEventRecord(j->e1, st));
  return AVR_OK;
}

// One launch of pieces on the split stream: descs / ctl uploaded, records already in sp_recs,
// results and outputs downloaded -- waited for, or (pending != nullptr) left in flight for
// split_wait, so the rest of a batch runs beside it.
// (The downloads wait for split_wait: a copy into pageable host memory would block the host until
// the kernel before it is done, and with it the launches meant to run beside it.)
struct SplitPending {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  void* res = nullptr;
  void* out = nullptr;
  const void* res_dev = nullptr;
  const void* out_dev = nullptr;
  size_t res_bytes = 0, out_bytes = 0;
};
bool split_timing() { return getenv("AVR_SPLIT_TIMING") != nullptr; }
int split_wait(avr_ctx* c, SplitPending* pend) {
  if (!pend->e0) return AVR_OK;
  HIP_TRY(c, hipStreamSynchronize(c->split_stream));
  HIP_TRY(c, hipMemcpy(pend->res, pend->res_dev, pend->res_bytes, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(pend->out, pend->out_dev, pend->out_bytes, hipMemcpyDeviceToHost));
  float ms = 0;
  HIP_TRY(c, hipEventElapsedTime(&ms, pend->e0, pend->e1));
  if (split_timing()) fprintf(stderr, "split: pieces kernel %.3f s\n", 1e-3 * ms);
  c->phase.kernel_s += 1e-3 * ms;
  (void)hipEventDestroy(pend->e0);
  (void)hipEventDestroy(pend->e1);
  pend->e0 = pend->e1 = nullptr;
  return AVR_OK;
}
int split_launch(avr_ctx* c, int mode, std::vector<avr_slice_desc>& d, const std::vector<avr::PieceCtl>& ctl,
                 const uint8_t* in_dev, int max_w, size_t stride, uint32_t flags, std::vector<avr_slice_result>* res,
                 Bytes* out, DevBuf* out_dev, SplitPending* pending = nullptr) {
  const int n = (int)d.size();
  uint64_t total = 0;
  for (auto& x : d) {
    x.out_offset = total;
    total += ((uint64_t)x.out_capacity + 15) & ~15ull;
  }
  res->assign(n, avr_slice_result{});
  out->resize(total);
  if (!n) return AVR_OK;
  hipStream_t st = c->split_stream;
  HIP_TRY(c, out_dev->reserve(total + 4096));
  HIP_TRY(c, c->sp_descs.reserve(sizeof(avr_slice_desc) * n));
  HIP_TRY(c, c->sp_res.reserve(sizeof(avr_slice_result) * n));
  HIP_TRY(c, c->sp_ctl.reserve(sizeof(avr::PieceCtl) * n));
  HIP_TRY(c, c->sp_est.reserve(sizeof(uint16_t) * (size_t)avr::kEstGlobal * std::max(1, avr::split_grid(n, max_w)), true));
  HIP_TRY(c, hipMemcpyAsync(c->sp_descs.p, d.data(), sizeof(avr_slice_desc) * n, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(c->sp_ctl.p, ctl.data(), sizeof(avr::PieceCtl) * n, hipMemcpyHostToDevice, st));
  avr::SplitArgs sa;
  sa.ctl = c->sp_ctl.as<avr::PieceCtl>();
  sa.recs = c->sp_recs.as<uint8_t>();
  sa.rec_stride = (uint32_t)stride;
  SplitPending local;
  SplitPending* pend = pending ? pending : &local;
  HIP_TRY(c, hipEventCreate(&pend->e0));
  HIP_TRY(c, hipEventCreate(&pend->e1));
  HIP_TRY(c, hipEventRecord(pend->e0, st));
  HIP_TRY(c, avr::launch_split(mode, c->tables.as<avr::EngineTables>(), c->sp_descs.as<avr_slice_desc>(), n, max_w,
                               in_dev, out_dev->as<uint8_t>(), c->sp_res.as<avr_slice_result>(), c->sp_est.as<uint16_t>(),
                               sa, flags, st));
  HIP_TRY(c, hipEventRecord(pend->e1, st));
  pend->res = res->data();
  pend->res_dev = c->sp_res.p;
  pend->res_bytes = sizeof(avr_slice_result) * n;
  pend->out = out->data();
  pend->out_dev = out_dev->p;
  pend->out_bytes = total;
  return pending ? AVR_OK : split_wait(c, pend);
}

// the regenerated bytes of a split slice: piece i's bytes up to cut i's q (the cut's first byte),
// the last piece whole; false if a piece failed or came out short
bool splice_pieces(const std::vector<const uint8_t*>& p, const std::vector<uint32_t>& len,
                   const std::vector<int32_t>& status, const std::vector<uint32_t>& q, std::vector<uint8_t>* o) {
  o->clear();
  for (size_t i = 0; i < p.size(); i++) {
    if (status[i]) return false;
    const size_t start = i ? q[i - 1] : 0;
    if (o->size() != start) return false;
    size_t keep = len[i];
    if (i < q.size()) {
      if (q[i] < start || q[i] - start > len[i]) return false;
      keep = q[i] - start;
    }
    o->insert(o->end(), p[i], p[i] + keep);
  }
  return true;
}
// recode.cpp:1345-1356 on a regenerated slice (before it: the trailing 0x80 already dropped)
void last_byte_patch(std::vector<uint8_t>* o, const uint8_t* payload, size_t size) {
  if (size <= 1) return;
  if ((int)(size & 1) != (int)(o->size() & 1)) o->push_back(payload[size - 1]);
  else if (!o->empty()) o->back() = payload[size - 1];
}

int split_finish(avr_ctx* c, SplitJob* j, bool verify, std::vector<SplitOut>* out) {
  const int n = (int)j->sl.size();
  out->assign(n, SplitOut());
  if (!n) return AVR_OK;
  hipStream_t st = c->split_stream;
  // 1) the split compress: statuses, streams, cut records, piece ends
  std::vector<avr_slice_result> r1(n);
  std::vector<uint32_t> cnt((size_t)n + j->nrec);
  Bytes out1(j->out_total), recs((size_t)j->stride * j->nrec);
  HIP_TRY(c, hipMemcpyAsync(r1.data(), c->sp_res.p, sizeof(avr_slice_result) * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(cnt.data(), c->sp_snapn.p, sizeof(uint32_t) * cnt.size(), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(out1.data(), c->sp_out.p, j->out_total, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(recs.data(), c->sp_recs.p, recs.size(), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  float ms = 0;
  HIP_TRY(c, hipEventElapsedTime(&ms, j->e0, j->e1));
  if (split_timing()) fprintf(stderr, "split: compress kernel %.3f s (%d slices)\n", 1e-3 * ms, n);
  c->phase.kernel_s += 1e-3 * ms;
  (void)hipEventDestroy(j->e0);
  (void)hipEventDestroy(j->e1);
  j->e0 = j->e1 = nullptr;
  const uint32_t* piece_end = cnt.data() + n;
  // 2) every cut checked against the host's restatement (seam_encoder), the pieces' lengths
  std::vector<std::vector<const avr::SeamRec*>> cuts(n);
  std::vector<std::vector<SeamCe>> ces(n);
  std::vector<std::vector<uint32_t>> plen(n);
  for (int k = 0; k < n; k++) {
    SplitOut& so = (*out)[k];
    so.status = r1[k].status;
    so.bill = r1[k];
    if (so.status) continue;
    const avr::SliceInfo& s = *j->sl[k];
    const uint32_t nc = cnt[k], base = (uint32_t)j->ctl[k].snap;
    if (nc >= j->ctl[k].snap_cap || piece_end[base + nc] != r1[k].out_len) {
      so.status = AVR_SLICE_CODER;
      continue;
    }
    for (uint32_t i = 0; i < nc && !so.status; i++) {
      const avr::SeamRec* r = (const avr::SeamRec*)(recs.data() + (size_t)(base + i) * j->stride);
      SeamCe ce;
      const uint64_t bitpos = 8ull * r->cd_next - r->cd_k;
      if (!seam_encoder(s.payload(), s.size, bitpos, r->cd_low >> r->cd_k, r->cd_range, &ce) || ce.q != r->q ||
          ce.low != r->ce_low || ce.range != r->ce_range || ce.outstanding != r->ce_outstanding ||
          ce.cache != r->ce_cache || ce.queue != r->ce_queue)
        so.status = AVR_SLICE_CODER;
      cuts[k].push_back(r);
      ces[k].push_back(ce);
    }
    for (uint32_t i = 0; i <= nc; i++) plen[k].push_back(piece_end[base + i] - (i ? piece_end[base + i - 1] : 0u));
    if (!so.status)
      so.recoded.assign(out1.begin() + j->d[k].out_offset, out1.begin() + j->d[k].out_offset + r1[k].out_len);
  }
  // 3) verify: the pieces decompressed from the records as a container gives them, spliced, compared
  if (verify) {
    std::vector<avr_slice_desc> dd;
    std::vector<avr::PieceCtl> pc;
    std::vector<int> first(n, -1);
    Bytes arena;
    for (int k = 0; k < n; k++) {
      if ((*out)[k].status) continue;
      first[k] = (int)dd.size();
      uint64_t off = 0;
      const size_t np = cuts[k].size() + 1;
      for (size_t i = 0; i < np; i++) {
        avr_slice_desc d = j->d[k];
        if (i) d.first_mb = (int32_t)cuts[k][i - 1]->first_mb;
        append_aligned(&arena, (*out)[k].recoded.data() + off, plen[k][i], 16, &d.payload_offset);
        off += plen[k][i];
        d.payload_size = d.read_limit = plen[k][i];
        d.out_capacity = (uint32_t)j->sl[k]->size + 4096;
        const uint32_t next = i + 1 < np ? cuts[k][i]->first_mb : 0u;
        pc.push_back(avr::PieceCtl{i ? j->ctl[k].snap + (int32_t)i - 1 : -1, next ? next - (uint32_t)d.first_mb : 0u,
                                   -1, 0});
        dd.push_back(d);
      }
    }
    if (!dd.empty()) {
      HIP_TRY(c, c->sp_in2.reserve(arena.size() + 4096));
      HIP_TRY(c, hipMemcpyAsync(c->sp_in2.p, arena.data(), arena.size(), hipMemcpyHostToDevice, st));
      std::vector<avr_slice_result> r3;
      Bytes out3;
      if (int e = split_launch(c, 1, dd, pc, c->sp_in2.as<uint8_t>(), j->max_w, j->stride, 0, &r3, &out3, &c->sp_out2))
        return e;
      for (int k = 0; k < n; k++) {
        if (first[k] < 0) continue;
        const avr::SliceInfo& s = *j->sl[k];
        const size_t np = cuts[k].size() + 1;
        std::vector<const uint8_t*> p(np);
        std::vector<uint32_t> len(np), q(np - 1);
        std::vector<int32_t> stt(np);
        for (size_t i = 0; i < np; i++) {
          const int x = first[k] + (int)i;
          p[i] = out3.data() + dd[x].out_offset;
          len[i] = r3[x].out_len;
          stt[i] = r3[x].status;
          if (i + 1 < np) q[i] = ces[k][i].q;
        }
        std::vector<uint8_t> regen;
        bool ok = splice_pieces(p, len, stt, q, &regen);
        if (ok) {
          last_byte_patch(&regen, s.payload(), s.size);
          ok = regen.size() == s.size && memcmp(regen.data(), s.payload(), s.size) == 0;
        }
        if (!ok) (*out)[k].status = AVR_SLICE_NO_ROUNDTRIP;
      }
    }
  }
  // 4) the seams fields
  for (int k = 0; k < n; k++) {
    SplitOut& so = (*out)[k];
    if (so.status || cuts[k].empty()) continue;
    if (!seams_encode(cuts[k], ces[k], j->d[k], plen[k], &so.seams)) return fail(c, AVR_ERR_DEVICE, "zlib failed");
  }
  return AVR_OK;
}

struct ParsedFile {
  std::vector<avr::SliceInfo> slices;
};

// views: slices without emulation-prevention bytes point into `in` instead of holding a copy (the
// caller keeps `in` alive while it uses pf)
int parse_file(avr_ctx* c, const uint8_t* in, size_t n, ParsedFile* pf, bool views = false,
               const avr::SkipRanges* skips = nullptr) {
  std::vector<avr::NalRef> nals;
  if (!avr::demux(in, n, &nals, skips)) return fail(c, AVR_ERR_FORMAT, "not an MP4/avcC or Annex-B H.264 stream");
  avr::StreamParser sp;
  sp.set_skips(in, skips);
  for (auto& nr : nals) {
    avr::SliceInfo s;
    if (sp.next(in + nr.offset, nr.size, &s, views)) {
      s.nal_offset = nr.offset;
      s.nal_size = nr.size;
      pf->slices.push_back(std::move(s));
    }
  }
  return AVR_OK;
}

// A slice the device can take: supported syntax, at least a surrogate marker long, and an LDS ring
// (ring_cols: 3 W + 7 records for an MBAFF slice) that fits a workgroup's LDS -- a very wide MBAFF
// picture is stored skip_coded instead of failing the whole file's launch.
bool recodable_candidate(const avr::SliceInfo& s) {
  const int cols = s.h.mbaff && !s.h.field_pic ? 3 * s.h.mb_width + 7 : s.h.mb_width;
  return s.h.supported && s.size >= (size_t)avr::kSurrogateMarkerBytes && avr::shared_bytes(cols) <= kLdsBudget;
}

// A slice as the container writer sees it: its payload (init_decoder's buf, size) and whether the
// device may re-code it (recodable_candidate).
struct SliceView {
  const uint8_t* payload;
  size_t size;
  bool candidate;
  uint64_t file_pos;   // where the payload stands verbatim in the file (the parse knows), or ~0
};
std::vector<SliceView> views_of(const ParsedFile& pf) {
  std::vector<SliceView> v(pf.slices.size());
  for (size_t i = 0; i < v.size(); i++)
    v[i] = {pf.slices[i].payload(), pf.slices[i].size, recodable_candidate(pf.slices[i]),
            pf.slices[i].file_payload_offset()};
  return v;
}

// Host threads for one file's bulk steps (trigram index, container copies): up to 16, or 1 inside a
// parallel_files worker, which already spreads the files over the thread budget (a corpus of large
// files would otherwise start ~16 x 16 threads at once).
thread_local bool tl_in_file_pool = false;
unsigned bulk_threads() {
  return tl_in_file_pool ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Every 00 00 0y trigram (y <= 3) of a file, keyed by y and the four bytes after it, then by
// position.  In an escaped H.264 stream these occur only at start codes, emulation-prevention bytes
// (00 00 03) and container bytes (MP4 lengths and boxes), so the index is small.
struct TrigramIndex {
  bool built = false;
  struct Entry {
    uint64_t key;   // y << 32 | the next four bytes (big-endian, zeros past the end)
    uint64_t pos;
    bool operator<(const Entry& o) const { return key != o.key ? key < o.key : pos < o.pos; }
  };
  std::vector<Entry> e;
  // per y, every trigram position in ascending order: the lookups whose payload holds no four bytes
  // after its trigram (built at the first such lookup)
  bool pos_built = false;
  std::vector<uint64_t> pos[4];
  void build_pos() {
    pos_built = true;
    for (const Entry& x : e) pos[x.key >> 32].push_back(x.pos);
    for (auto& v : pos) std::sort(v.begin(), v.end());
  }
  static uint64_t key_at(const uint8_t* f, size_t n, size_t p) {   // trigram at p (p + 2 < n)
    uint32_t nx = 0;
    for (int k = 0; k < 4; k++) nx = nx << 8 | (p + 3 + k < n ? f[p + 3 + k] : 0u);
    return (uint64_t)f[p + 2] << 32 | nx;
  }
  // the trigrams starting in [lo, hi)
  static void scan(const uint8_t* f, size_t n, size_t lo, size_t hi, std::vector<Entry>* out) {
    const uint8_t* end = f + std::min(hi, n >= 2 ? n - 2 : 0);
    for (const uint8_t* p = f + lo; p < end;) {
      p = (const uint8_t*)memchr(p, 0, (size_t)(end - p));
      if (!p) break;
      if (p[1] == 0 && p[2] <= 3) out->push_back({key_at(f, n, (size_t)(p - f)), (uint64_t)(p - f)});
      p++;
    }
  }
  void build(const uint8_t* f, size_t n) {
    built = true;
    // a multi-GB file is scanned in chunks on host threads
    const unsigned T = n < ((size_t)256 << 20) ? 1u : bulk_threads();
    std::vector<std::vector<Entry>> part(T);
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; t++) th.emplace_back(scan, f, n, n * t / T, n * (t + 1) / T, &part[t]);
    scan(f, n, 0, n / T, &part[0]);
    for (auto& x : th) x.join();
    for (auto& v : part) e.insert(e.end(), v.begin(), v.end());
    std::sort(e.begin(), e.end());
  }
};

// memmem(in + from, n - from, P, m) (the reference's search, recode.cpp:1285) without its cost on a
// miss.  A payload P holding a 00 00 0y trigram (y <= 3) at offset j -- an unescaped payload whose
// NAL had emulation-prevention bytes -- can only occur at q with a trigram of the file at q + j
// followed by the same four bytes as in P (when P has them), so the index's entries with that key
// from position from + j on, in ascending order, are the only candidates and the first that matches
// is memmem's answer.  Such payloads are exactly the ones that usually occur nowhere, where memmem
// would scan to the end of the file for each of them (O(misses x file): minutes for a 10-minute 4K
// stream); with the key a miss costs a binary search.  A payload without one is found in its own
// NAL (its bytes are verbatim there), so memmem stops at most one NAL past `from`.
const uint8_t* find_payload(const uint8_t* in, size_t n, size_t from, const uint8_t* P, size_t m, TrigramIndex* ix) {
  size_t j = 0;
  bool anchor = false;
  for (const uint8_t* q = P; m >= 3 && q + 2 < P + m;) {
    q = (const uint8_t*)memchr(q, 0, (size_t)(P + m - 2 - q));
    if (!q) break;
    if (q[1] == 0 && q[2] <= 3) {
      j = (size_t)(q - P);
      anchor = true;
      break;
    }
    q++;
  }
  if (!anchor) return (const uint8_t*)memmem(in + from, n - from, P, m);
  if (!ix->built) {
    const double tb = now_s();
    ix->build(in, n);
    if (getenv("AVR_ASM_TIMING")) fprintf(stderr, "index build %.3f s, %zu entries\n", now_s() - tb, ix->e.size());
  }
  using E = TrigramIndex::Entry;
  if (j + 7 > m) {
    // the trigram lies in P's last six bytes: no key beyond y; y's positions from from + j on, in
    // ascending order -- the first that matches is memmem's answer
    if (!ix->pos_built) ix->build_pos();
    const std::vector<uint64_t>& ps = ix->pos[P[j + 2]];
    for (auto it = std::lower_bound(ps.begin(), ps.end(), (uint64_t)(from + j)); it != ps.end(); ++it) {
      const size_t q = (size_t)*it - j;
      if (q + m > n) break;
      if (memcmp(in + q, P, m) == 0) return in + q;
    }
    return nullptr;
  }
  const uint64_t key = TrigramIndex::key_at(P, m, j);   // P holds the four bytes after its trigram
  for (auto it = std::lower_bound(ix->e.begin(), ix->e.end(), E{key, (uint64_t)(from + j)}); it != ix->e.end(); ++it) {
    if (it->key != key) break;
    const size_t q = (size_t)it->pos - j;
    if (q + m > n) break;
    if (memcmp(in + q, P, m) == 0) return in + q;
  }
  return nullptr;
}

// memmem(in + from, n - from, P, m) for a payload that stands verbatim at `own` >= from (segment
// checks it): memmem's
// answer is the first occurrence at or after `from` and `own` is one, so only [from, own) -- the
// literal gap before the slice: start code or length, NAL and slice header, skipped NAL units --
// needs a search.  Candidates are the gap's bytes equal to P[0] (memchr), each checked on its first
// 64 bytes and, if those agree, in full; a gap with more than a few such deep candidates (only a
// degenerate payload has them) goes to memmem over [from, own + m - 1).  O(gap) per slice instead
// of memmem's O(m) needle preparation plus its scan: the segmentation of a 4 GB stream no longer
// reads the stream once more.
const uint8_t* find_before(const uint8_t* in, size_t from, size_t own, const uint8_t* P, size_t m) {
  const size_t head = std::min<size_t>(m, 64);
  int deep = 0;
  for (size_t q = from; q < own;) {
    const uint8_t* h = (const uint8_t*)memchr(in + q, P[0], own - q);
    if (!h) break;
    if (memcmp(h, P, head) == 0) {
      if (++deep > 4) {
        const uint8_t* r = (const uint8_t*)memmem(in + from, own - from + m - 1, P, m);
        return r ? r : in + own;
      }
      if (memcmp(h + head, P + head, m - head) == 0) return h;
    }
    q = (size_t)(h - in) + 1;
  }
  return in + own;
}

// find_next_coded_block_and_emit_literal (recode.cpp:1275-1297): slice i becomes a cabac block when
// it is recodable (ok[i]), at least a surrogate marker long, and its payload occurs verbatim after
// the previous coded block.  Returns the payload's position in the file per slice (null = skip).
std::vector<const uint8_t*> segment(const uint8_t* in, size_t n, const std::vector<SliceView>& sv,
                                    const std::vector<char>& ok) {
  std::vector<const uint8_t*> found(sv.size(), nullptr);
  TrigramIndex ix;
  // a recorded position is trusted only where the payload's bytes stand there (a payload that is a
  // view of the file at that position trivially; a copy -- rank 0's parse arena, another revision
  // of the file -- compared in full, on host threads); else the plain search
  std::vector<char> own_ok(sv.size(), 0);
  {
    std::vector<size_t> chk;
    for (size_t i = 0; i < sv.size(); i++) {
      const uint64_t own = sv[i].file_pos;
      if (!ok[i] || sv[i].size < (size_t)avr::kSurrogateMarkerBytes || own == ~(uint64_t)0 || own + sv[i].size > n) continue;
      if (sv[i].payload == in + own) own_ok[i] = 1;
      else chk.push_back(i);
    }
    uint64_t bytes = 0;
    for (size_t i : chk) bytes += sv[i].size;
    const unsigned T = bytes < ((uint64_t)64 << 20) ? 1u : bulk_threads();
    auto work = [&](unsigned t) {
      for (size_t k = t; k < chk.size(); k += T) {
        const size_t i = chk[k];
        own_ok[i] = memcmp(in + sv[i].file_pos, sv[i].payload, sv[i].size) == 0;
      }
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
  }
  size_t prev_end = 0;
  for (size_t i = 0; i < sv.size(); i++) {
    if (!ok[i] || sv[i].size < (size_t)avr::kSurrogateMarkerBytes) continue;
    const uint64_t own = sv[i].file_pos;
    const uint8_t* f = own_ok[i] && own >= prev_end
                           ? find_before(in, prev_end, (size_t)own, sv[i].payload, sv[i].size)
                           : find_payload(in, n, prev_end, sv[i].payload, sv[i].size, &ix);
    if (f) {
      found[i] = f;
      prev_end = (size_t)(f - in) + sv[i].size;
    }
  }
  return found;
}
std::vector<const uint8_t*> segment(const uint8_t* in, size_t n, const ParsedFile& pf, const std::vector<char>& ok) {
  return segment(in, n, views_of(pf), ok);
}

// A large host output buffer handed to the caller (freed by avr_free = free): 2 MiB aligned and
// advised to transparent huge pages, so its first touch costs one fault per 2 MiB instead of per
// 4 KiB page (a 4.4 GB container or payload arena: ~1 s of page faults otherwise).
uint8_t* host_alloc(size_t n) {
  constexpr size_t kHuge = (size_t)2 << 20;
  if (n < 16 * kHuge) return (uint8_t*)malloc(n ? n : 1);
  void* p = nullptr;
  if (posix_memalign(&p, kHuge, n)) return nullptr;
  (void)madvise(p, n & ~(kHuge - 1), MADV_HUGEPAGE);
  return (uint8_t*)p;
}

// Byte copies of a container's literals and re-coded blocks, spread over host threads when they are
// large (a 10-minute 4K stream's container is 4.4 GB).  A job without a source fills its bytes
// with `fill` (the decompressor's surrogate blocks).
void copy_part(uint8_t* dst, const uint8_t* src, size_t len, uint8_t fill) {
  if (src) memcpy(dst, src, len);
  else memset(dst, fill, len);
}
void parallel_copies(const std::vector<avr::PbCopy>& jobs, uint8_t* base, uint8_t fill = 0) {
  uint64_t total = 0;
  for (const auto& j : jobs) total += j.len;
  const unsigned T = total < ((uint64_t)64 << 20) ? 1u : bulk_threads();
  if (T == 1) {
    for (const auto& j : jobs) copy_part(base + j.dst, j.src, j.len, fill);
    return;
  }
  // thread t copies the bytes [t total / T, (t + 1) total / T) of the concatenated jobs
  auto work = [&](unsigned t) {
    const uint64_t lo = total * t / T, hi = total * (t + 1) / T;
    uint64_t at = 0;
    for (const auto& j : jobs) {
      const uint64_t a = std::max(at, lo), b = std::min(at + j.len, hi);
      if (a < b) copy_part(base + j.dst + (a - at), j.src ? j.src + (a - at) : nullptr, (size_t)(b - a), fill);
      at += j.len;
      if (at >= hi) break;
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < T; t++) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
}

// fn(f) for f in [0, nf) on up to 16 host threads (independent files: segmentation, containers).
// An exception in a worker (allocation failure) is rethrown here, on the caller's thread, so that
// guarded() still turns it into a status.
template <class F>
void parallel_files(int nf, F&& fn) {
  const unsigned T = (unsigned)std::min<int>(nf, (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  if (T <= 1) {
    for (int f = 0; f < nf; f++) fn(f);
    return;
  }
  std::atomic<int> next{0};
  std::exception_ptr err;
  std::mutex mu;
  auto work = [&]() {
    const bool was = tl_in_file_pool;
    tl_in_file_pool = true;   // each file's own bulk steps stay on this thread
    try {
      for (int f; (f = next.fetch_add(1)) < nf;) fn(f);
    } catch (...) {
      std::lock_guard<std::mutex> g(mu);
      if (!err) err = std::current_exception();
      next = nf;
    }
    tl_in_file_pool = was;
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < T; t++) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
}

// compressor::run's block stream (recode.cpp:1115-1125, 1275-1297) as a Recoded protobuf, written
// once: the blocks' headers in order, their bytes by parallel_copies, into the caller's buffer dst
// (cap bytes; too small: AVR_ERR_INVALID_ARGUMENT with *out_len = the size needed) or, without one,
// into one exactly sized buffer allocated here (*out).
int emit_container(const uint8_t* in, size_t n, const std::vector<SliceView>& sv, const std::vector<const uint8_t*>& found,
                   const std::vector<std::pair<const uint8_t*, size_t>>& recoded, int model, uint8_t** out,
                   size_t* out_len, uint8_t* dst = nullptr, size_t cap = 0,
                   const std::vector<std::pair<const uint8_t*, size_t>>* seams = nullptr) {
  std::vector<avr::PbBlock> blocks;
  blocks.reserve(2 * sv.size() + 1);
  size_t prev_end = 0;
  for (size_t i = 0; i < sv.size(); i++) {
    const SliceView& s = sv[i];
    avr::PbBlock b;
    if (found[i]) {
      avr::PbBlock lit;
      lit.has_literal = true;
      lit.literal = in + prev_end;
      lit.literal_len = (size_t)(found[i] - (in + prev_end));
      blocks.push_back(lit);
      prev_end = (size_t)(found[i] - in) + s.size;
      b.has_size = true;
      b.size = (int64_t)s.size;
      b.has_parity = true;
      b.length_parity = s.size & 1;
      if (s.size > 1) b.has_last_byte = true, b.last_byte.assign(1, (char)s.payload[s.size - 1]);
      b.has_cabac = true;
      b.cabac = recoded[i].first;
      b.cabac_len = recoded[i].second;
      if (seams && (*seams)[i].second) b.has_seams = true, b.seams = (*seams)[i].first, b.seams_len = (*seams)[i].second;
    } else {
      b.has_skip = true;
      b.skip_coded = true;
      b.has_size = true;
      b.size = (int64_t)s.size;
    }
    blocks.push_back(std::move(b));
  }
  avr::PbBlock lit;
  lit.has_literal = true;
  lit.literal = in + prev_end;
  lit.literal_len = n - prev_end;
  blocks.push_back(lit);
  std::vector<uint8_t> md;
  if (const char* tag = avr::version_of_model(model)) avr::pb_put_metadata_version(&md, tag);
  size_t total = md.size();
  for (const auto& b : blocks) total += avr::pb_block_size(b);
  if (dst && total > cap) {
    *out_len = total;
    return AVR_ERR_INVALID_ARGUMENT;
  }
  uint8_t* o = dst ? dst : host_alloc(total);
  if (!o) return AVR_ERR_OUT_OF_MEMORY;
  if (!md.empty()) memcpy(o, md.data(), md.size());
  size_t at = md.size();
  std::vector<avr::PbCopy> copies;
  copies.reserve(2 * blocks.size());
  for (const auto& b : blocks) at = avr::pb_write_block(o, at, b, &copies);
  if (at != total) {
    if (!dst) free(o);
    return fail(nullptr, AVR_ERR_DEVICE, "internal error: container size");
  }
  parallel_copies(copies, o);
  if (out) *out = dst ? nullptr : o;
  *out_len = total;
  return AVR_OK;
}

// compressor::run (recode.cpp:1102-1132) for several files at once.  The device work of every
// file is batched: one parallel launch checks every candidate slice of every file (parse, restore,
// device roundtrip), and the reference model runs all files in one pass (the parallel R-mode
// pipeline over all their slices with per-file estimators, or one workgroup per file).  out[f] is
// malloc'd; status[f] (optional) is file f's result; the return value is the first failure.
// Host side of avr_phase_times for one whole-file call: the time before the first device pass is
// demux, the wall time inside run_plan is the device passes (split by their HIP events, the rest
// of it overhead), everything else container work.
struct PhaseClock {
  avr_ctx* c;
  double t0, t_demux = -1;
  explicit PhaseClock(avr_ctx* ctx) : c(ctx), t0(now_s()) {
    c->phase = avr_phase_times{};
    c->plan_wall = 0;
  }
  void mark_demux() {
    if (t_demux < 0) t_demux = now_s() - t0;
  }
  void finish() {
    mark_demux();
    avr_phase_times& p = c->phase;
    const double wall = now_s() - t0, dev = p.upload_s + p.kernel_s + p.download_s;
    p.demux_s = t_demux;
    p.container_s = std::max(0.0, wall - t_demux - c->plan_wall);
    p.other_s = std::max(0.0, c->plan_wall - dev);
  }
};

typedef std::array<uint64_t, 6> Bill;   // h264_model::bill / cabac_bill by avr_pip_coding_type
void add_bill(Bill* b, const avr_slice_result& r) {
  for (int i = 0; i < 6; i++) (*b)[i] += r.bill[i];
}

// verify (parallel model): decompress every candidate slice on the device and code only those that
// regenerate their payload.  avr_roundtrip_file skips it on a first attempt -- its own whole-file
// decompress and compare check the same thing, as the reference's roundtrip() does with a
// compressor that never verifies (recode.cpp:1594-1624) -- and repeats with it on a mismatch.
int compress_files(avr_ctx* c, int nf, const uint8_t* const* in, const size_t* in_len, int model, uint8_t** out,
                   size_t* out_len, int32_t* status, std::vector<Bill>* bills = nullptr, bool verify = true) {
  if (bills) bills->assign(nf, Bill{});
  HIP_TRY(c, hipSetDevice(c->device));
  PhaseClock pc(c);
  std::vector<int32_t> st(nf, AVR_OK);
  std::vector<ParsedFile> pf(nf);
  for (int f = 0; f < nf; f++) {
    out[f] = nullptr;
    out_len[f] = 0;
    st[f] = parse_file(c, in[f], in_len[f], &pf[f], /*views=*/true);
  }
  // 1) parallel model: every candidate slice of every file through the parallel kernel -- per-slice
  //    parse, restore check, device roundtrip and the model's output.  Reference model: nothing
  //    here; the reference-model pass below parses and checks every candidate itself (its statuses
  //    carry the same parse / restore verdict) and demotes the failures, so a well-formed file
  //    costs one reference-model pass, not a parallel-model pass before it.
  Plan plan;
  // the parallel model's long slices (split_candidate): the split job, its first pass on the split
  // stream beside the batch (cand_of = -2 - index there)
  SplitJob sj;
  const size_t split_bytes = model == AVR_MODEL_PARALLEL ? c->split_bytes : 0;
  std::vector<std::vector<int>> cand_of(nf);
  for (int f = 0; f < nf; f++) {
    cand_of[f].assign(pf[f].slices.size(), -1);
    if (st[f] || reference_model(model)) continue;
    for (size_t i = 0; i < pf[f].slices.size(); i++) {
      const avr::SliceInfo& s = pf[f].slices[i];
      if (!recodable_candidate(s)) continue;
      avr_slice_desc d = desc_from_header(s);
      d.payload_size = (uint32_t)s.size;
      if (split_candidate(d, split_bytes)) {
        cand_of[f][i] = -2 - (int)sj.sl.size();
        sj.sl.push_back(&s);
        continue;
      }
      append_aligned(&plan.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
      d.payload_size = (uint32_t)s.size;
      d.read_limit = (uint32_t)s.read_limit;
      d.out_capacity = (uint32_t)(s.size * 2 + 256);
      plan.max_w = std::max(plan.max_w, ring_cols(d));
      cand_of[f][i] = (int)plan.descs.size();
      plan.descs.push_back(d);
    }
  }
  std::vector<avr_slice_result> res;
  Bytes outb;
  pc.mark_demux();
  if (int r = split_begin(c, &sj, split_bytes, bills ? avr::kFlagBill : 0u)) return r;
  if (int r = run_plan(c, 0, false, plan, &res, &outb, verify,
                       (bills ? avr::kFlagBill : 0u) | coder_flag(model))) {
    (void)hipStreamSynchronize(c->split_stream);   // its first pass still reads sj's buffers
    return r;
  }
  std::vector<SplitOut> so;
  {
    const double t = now_s();
    if (int r = split_finish(c, &sj, verify, &so)) return r;
    c->plan_wall += now_s() - t;
  }
  // 2) segmentation (find_next_coded_block_and_emit_literal, recode.cpp:1275-1297)
  std::vector<std::vector<char>> ok(nf);
  std::vector<std::vector<const uint8_t*>> found(nf);
  for (int f = 0; f < nf; f++) {
    ok[f].assign(pf[f].slices.size(), 0);
    for (size_t i = 0; i < pf[f].slices.size(); i++)
      ok[f][i] = reference_model(model) ? st[f] == AVR_OK && recodable_candidate(pf[f].slices[i])
                 : cand_of[f][i] >= 0    ? res[cand_of[f][i]].status == 0
                 : cand_of[f][i] <= -2   ? so[-2 - cand_of[f][i]].status == 0
                                         : false;
  }
  parallel_files(nf, [&](int f) { found[f] = segment(in[f], in_len[f], pf[f], ok[f]); });
  // 3) reference model: the coded slices of every file in file order, estimators per file; a
  //    slice that fails there is demoted to skip_coded and its file's pass repeated
  std::vector<std::vector<std::vector<uint8_t>>> recoded(nf);
  for (int f = 0; f < nf; f++) recoded[f].resize(pf[f].slices.size());
  std::vector<std::vector<std::pair<const uint8_t*, size_t>>> seams_of(nf);
  for (int f = 0; f < nf; f++) seams_of[f].assign(pf[f].slices.size(), {nullptr, 0});
  if (reference_model(model)) {
    std::vector<char> todo(nf, 0);
    for (int f = 0; f < nf; f++) todo[f] = st[f] == AVR_OK;
    for (int attempt = 0;; attempt++) {
      Plan rp;
      std::vector<std::pair<int, int>> idx;   // (file, slice) per desc
      for (int f = 0; f < nf; f++) {
        if (!todo[f]) continue;
        if (bills) (*bills)[f] = Bill{};   // this pass re-codes the whole file
        rp.file_first.push_back((int)rp.descs.size());
        int coded_n = 0;
        for (size_t i = 0; i < pf[f].slices.size(); i++) {
          const avr::SliceInfo& s = pf[f].slices[i];
          avr_slice_desc d = desc_from_header(s);
          d.coded = found[f][i] != nullptr;
          // chained model: a fresh model (a new "file" of the pass: estimators, frames) before every
          // AVR_CHAIN_SLICES-th coded slice; uncoded slices before it still flip the old chain's frames
          if (d.coded && model == AVR_MODEL_CHAINED && coded_n > 0 && coded_n % AVR_CHAIN_SLICES == 0)
            rp.file_first.push_back((int)rp.descs.size());
          coded_n += d.coded;
          if (d.coded) {
            append_aligned(&rp.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
            d.payload_size = (uint32_t)s.size;
            d.read_limit = (uint32_t)s.read_limit;
            d.out_capacity = (uint32_t)(s.size * 4 + 4096);
            rp.max_w = std::max(rp.max_w, ring_cols(d));   // uncoded slices only flip frames
          }
          idx.push_back({f, (int)i});
          rp.descs.push_back(d);
        }
      }
      if (rp.file_first.empty()) break;
      rp.file_first.push_back((int)rp.descs.size());
      std::vector<avr_slice_result> rr;
      Bytes ro;
      if (int r = run_plan(c, 0, true, rp, &rr, &ro, false, bills ? avr::kFlagBill : 0)) return r;
      std::fill(todo.begin(), todo.end(), 0);
      for (size_t k = 0; k < idx.size(); k++) {
        const int f = idx[k].first, i = idx[k].second;
        if (!found[f][i]) continue;
        if (rr[k].status != 0) {
          found[f][i] = nullptr;
          todo[f] = 1;
          continue;
        }
        recoded[f][i].assign(ro.begin() + rp.descs[k].out_offset,
                             ro.begin() + rp.descs[k].out_offset + rr[k].out_len);
        if (bills) add_bill(&(*bills)[f], rr[k]);
      }
      bool again = false;
      for (int f = 0; f < nf; f++) {
        if (!todo[f]) continue;
        again = true;
        // a demoted slice changes the literal gaps of later ones: redo the segmentation
        for (size_t i = 0; i < pf[f].slices.size(); i++) ok[f][i] = ok[f][i] && found[f][i] != nullptr;
        found[f] = segment(in[f], in_len[f], pf[f], ok[f]);
        if (attempt == 7) {
          st[f] = fail(c, AVR_ERR_DEVICE, "reference-model pass did not converge");
          todo[f] = 0;
        }
      }
      if (!again) break;
    }
  } else {
    for (int f = 0; f < nf; f++)
      for (size_t i = 0; i < pf[f].slices.size(); i++)
        if (found[f][i]) {
          const int k = cand_of[f][i];
          if (k <= -2) {   // a split slice: its pieces' streams and seams
            SplitOut& x = so[-2 - k];
            recoded[f][i].swap(x.recoded);
            seams_of[f][i] = {x.seams.data(), x.seams.size()};
            if (bills) add_bill(&(*bills)[f], x.bill);
            continue;
          }
          recoded[f][i].assign(outb.begin() + plan.descs[k].out_offset,
                               outb.begin() + plan.descs[k].out_offset + res[k].out_len);
          if (bills) add_bill(&(*bills)[f], res[k]);
        }
  }
  // 4) containers (compressor::run, recode.cpp:1115-1125)
  int first_err = AVR_OK;
  parallel_files(nf, [&](int f) {
    if (st[f] != AVR_OK) return;
    std::vector<std::pair<const uint8_t*, size_t>> blobs(pf[f].slices.size(), {nullptr, 0});
    for (size_t i = 0; i < pf[f].slices.size(); i++) blobs[i] = {recoded[f][i].data(), recoded[f][i].size()};
    st[f] = emit_container(in[f], in_len[f], views_of(pf[f]), found[f], blobs, model, &out[f], &out_len[f], nullptr, 0,
                           &seams_of[f]);
  });
  for (int f = 0; f < nf; f++) {
    if (status) status[f] = st[f];
    if (st[f] && !first_err) first_err = st[f];
  }
  pc.finish();
  return status ? AVR_OK : first_err;
}

// decompressor::run (recode.cpp:1312-1357) for several files at once: the slices of every
// parallel-model file go to one parallel launch, every reference-model file to one workgroup of a
// sequential launch.
// A split block (the parallel model's long-slice split): its pieces in the split plan, the cuts' q
// (piece i's bytes end at q[i]), the spliced regenerated bytes after the run
struct SplitBlock {
  int block = -1, first = 0, pieces = 0;
  std::vector<uint32_t> q;
  std::vector<uint8_t> regen;
  int32_t status = 0;
  avr_slice_result bill{};
};
struct SplitPlan {
  Plan plan;                        // the pieces (descs, their re-coded streams in the arena)
  std::vector<avr::PieceCtl> ctl;
  Bytes recs;                       // the cut records, rec_stride apart
  size_t stride = avr::seam_rec_bytes(kMringCols);
  static constexpr int kMringCols = avr::kMringCols;   // widest picture a record holds
};
struct DecJob {
  std::vector<avr::PbBlock> blocks;
  Bytes stream;                      // read_packet's stream: literals + surrogate blocks
  bool parallel = false;
  int model = AVR_MODEL_REFERENCE;   // from Recoded.Metadata.version
  std::vector<int> desc_of_block;    // plan index per coded block (-1: none; <= -2: split block -2 - k)
  std::vector<SplitBlock> splits;
};

// sp: where the pieces of split blocks go (nullptr: such a container is refused -- the sharded and
// hooks paths decompress slices, not pieces)
int decompress_setup(avr_ctx* c, const uint8_t* in, size_t n, DecJob* j, Plan* plan, SplitPlan* sp = nullptr) {
  const bool tm = getenv("AVR_ASM_TIMING") != nullptr;
  double t0 = now_s();
  std::string version;
  if (!avr::pb_parse(in, n, &j->blocks, &version)) return fail(c, AVR_ERR_FORMAT, "not a Recoded protobuf");
  j->model = avr::model_of_version(version);
  // another avrecode-amd container format (the round-2 "avrecode-amd:P", ...) would be read as a
  // reference-model container and fail late: refuse it here
  if (j->model < 0)
    return fail(c, AVR_ERR_FORMAT, "unsupported container version " + version + " (expected " + avr::kParallelModelTag +
                                       " or " + avr::kParallel32ModelTag + ")");
  j->parallel = parallel_model(j->model);
  // read_packet (recode.cpp:1359-1409): literals and surrogate blocks form the stream -- its layout
  // first, then one allocation, the markers, and the literal copies and 'X' fills on host threads
  uint64_t seq = 1;
  size_t total = 0;
  for (auto& b : j->blocks) {
    if ((int)b.has_literal + (int)b.has_cabac + (int)b.has_skip != 1)
      return fail(c, AVR_ERR_FORMAT, "Invalid input block: must have exactly one type");
    if (b.has_literal) {
      total += b.literal_len;
    } else if (b.has_cabac) {
      if (!b.has_size) return fail(c, AVR_ERR_FORMAT, "CABAC block requires size field.");
      if (b.size < avr::kSurrogateMarkerBytes || b.size > ((int64_t)1 << 31))
        return fail(c, AVR_ERR_FORMAT, "Invalid coded block size for surrogate: " + std::to_string(b.size));
      total += (size_t)b.size;
    } else if (!b.skip_coded) {
      return fail(c, AVR_ERR_FORMAT, "Unknown input block type");
    }
  }
  j->stream.resize(total);
  // the surrogate fills: no 0x00 / 0x03 byte in them ('X'), so the parse steps over them
  avr::SkipRanges skips;
  {
    std::vector<avr::PbCopy> fills;
    fills.reserve(j->blocks.size());
    size_t at = 0;
    for (auto& b : j->blocks) {
      if (b.has_literal) {
        if (b.literal_len) fills.push_back({at, b.literal, b.literal_len});
        at += b.literal_len;
      } else if (b.has_cabac) {
        avr::surrogate_marker(seq++, j->stream.data() + at);
        fills.push_back({at + 8, nullptr, (size_t)b.size - 8});
        if (b.size > 8) skips.push_back({at + 8, at + (size_t)b.size});
        at += (size_t)b.size;
      }
    }
    parallel_copies(fills, j->stream.data(), (uint8_t)'X');
  }
  static_assert('X' != 0 && 'X' != 3, "surrogate fill: no start-code or emulation-prevention byte");
  if (tm) fprintf(stderr, "setup: pb+stream %.3f s\n", now_s() - t0), t0 = now_s();
  ParsedFile pf;
  if (int r = parse_file(c, j->stream.data(), j->stream.size(), &pf, /*views=*/true, &skips)) return r;
  if (tm) fprintf(stderr, "setup: parse %.3f s\n", now_s() - t0), t0 = now_s();
  // recognize_coded_block (recode.cpp:1546-1573): slices claim coded blocks in order
  j->desc_of_block.assign(j->blocks.size(), -1);
  size_t next_coded = 0;
  uint64_t seq_check = 1;
  std::vector<avr_slice_desc> descs;
  std::vector<int> block_of;
  Plan local;
  for (auto& s : pf.slices) {
    while (next_coded < j->blocks.size() && !j->blocks[next_coded].has_cabac && !j->blocks[next_coded].has_skip)
      next_coded++;
    if (next_coded >= j->blocks.size())
      return fail(c, AVR_ERR_FORMAT, "Coded block expected, but not recorded in the compressed data.");
    const avr::PbBlock& b = j->blocks[next_coded];
    if ((size_t)b.size != s.size) return fail(c, AVR_ERR_FORMAT, "Invalid surrogate block size.");
    avr_slice_desc d = desc_from_header(s);
    if (b.has_cabac) {
      uint8_t mk[8];
      avr::surrogate_marker(seq_check++, mk);
      if (memcmp(s.payload(), mk, 8) != 0) return fail(c, AVR_ERR_FORMAT, "Invalid surrogate marker in coded block.");
      d.payload_size = (uint32_t)b.cabac_len;
      d.read_limit = (uint32_t)b.cabac_len;
      d.out_capacity = (uint32_t)(b.size + 64);
    } else {
      d.coded = 0;
    }
    if (b.has_cabac && b.has_seams) {   // a split block: its pieces go to the split plan
      if (!sp) return fail(c, AVR_ERR_UNSUPPORTED, "split slices (block field 16) decompress through the whole-file calls only");
      if (j->model != AVR_MODEL_PARALLEL || d.structure != AVR_STRUCT_FRAME || d.mb_width > SplitPlan::kMringCols)
        return fail(c, AVR_ERR_FORMAT, "seams on a block that cannot be split");
      SeamsDecoded sd;
      if (!seams_decode(b.seams, b.seams_len, d, sp->stride, &sd))
        return fail(c, AVR_ERR_FORMAT, "Invalid seams field in coded block.");
      uint64_t tot = 0;
      for (uint32_t l : sd.piece_len) tot += l;
      if (tot != b.cabac_len || sd.q.back() >= (uint64_t)b.size || sd.first_mb[0] <= (uint32_t)d.first_mb)
        return fail(c, AVR_ERR_FORMAT, "Invalid seams field in coded block.");
      SplitBlock x;
      x.block = (int)next_coded;
      x.first = (int)sp->plan.descs.size();
      x.pieces = sd.cuts + 1;
      x.q = sd.q;
      const uint32_t rec0 = (uint32_t)(sp->recs.size() / sp->stride);
      sp->recs.insert(sp->recs.end(), sd.recs.begin(), sd.recs.end());
      uint64_t off = 0;
      for (int i = 0; i <= sd.cuts; i++) {
        avr_slice_desc pd = d;
        if (i) pd.first_mb = (int32_t)sd.first_mb[i - 1];
        append_aligned(&sp->plan.arena, b.cabac + off, sd.piece_len[i], 16, &pd.payload_offset);
        off += sd.piece_len[i];
        pd.payload_size = pd.read_limit = sd.piece_len[i];
        pd.out_capacity = (uint32_t)((i < sd.cuts ? sd.q[i] : (uint32_t)b.size) - (i ? sd.q[i - 1] : 0u) + 4096);
        sp->plan.max_w = std::max(sp->plan.max_w, pd.mb_width);
        sp->plan.descs.push_back(pd);
        sp->ctl.push_back(avr::PieceCtl{i ? (int32_t)(rec0 + i - 1) : -1,
                                        i < sd.cuts ? sd.first_mb[i] - (uint32_t)pd.first_mb : 0u, -1, 0});
      }
      j->desc_of_block[next_coded] = -2 - (int)j->splits.size();
      j->splits.push_back(std::move(x));
      next_coded++;
      continue;
    }
    if (j->parallel && !d.coded) {   // the parallel model has no cross-slice state: skip it
      next_coded++;
      continue;
    }
    block_of.push_back((int)next_coded);
    descs.push_back(d);
    next_coded++;
  }
  // all checks passed: append to the shared plan (append_aligned's layout: 16-byte aligned streams,
  // each followed by >= 16 zero bytes), the re-coded streams copied on host threads
  if (!plan) {
    for (size_t k = 0; k < descs.size(); k++) j->desc_of_block[block_of[k]] = (int)k;
    return AVR_OK;
  }
  std::vector<avr::PbCopy> copies;
  copies.reserve(descs.size());
  uint64_t at = plan->layout_only ? plan->arena_end : plan->arena.size();
  for (size_t k = 0; k < descs.size(); k++) {
    avr_slice_desc& d = descs[k];
    const avr::PbBlock& b = j->blocks[block_of[k]];
    if (d.coded) {
      d.payload_offset = (at + 15) & ~(uint64_t)15;
      copies.push_back({(size_t)d.payload_offset, b.cabac, b.cabac_len});
      at = d.payload_offset + b.cabac_len + 16;
      plan->max_w = std::max(plan->max_w, ring_cols(d));
    }
  }
  if (plan->layout_only) {
    plan->arena_copies.insert(plan->arena_copies.end(), copies.begin(), copies.end());
    plan->arena_end = at;
    for (size_t k = 0; k < descs.size(); k++) {
      j->desc_of_block[block_of[k]] = (int)plan->descs.size();
      plan->descs.push_back(descs[k]);
    }
    return AVR_OK;
  }
  const size_t a0 = plan->arena.size();
  plan->arena.resize(at);
  {
    uint64_t z = a0;   // the zero bytes between the streams
    for (const auto& cp : copies) {
      memset(plan->arena.data() + z, 0, cp.dst - z);
      z = cp.dst + cp.len;
    }
    memset(plan->arena.data() + z, 0, at - z);
  }
  parallel_copies(copies, plan->arena.data());
  for (size_t k = 0; k < descs.size(); k++) {
    j->desc_of_block[block_of[k]] = (int)plan->descs.size();
    plan->descs.push_back(descs[k]);
  }
  if (tm) fprintf(stderr, "setup: match+arena %.3f s\n", now_s() - t0);
  return AVR_OK;
}

// decompressor::run's output (recode.cpp:1338-1357): the literals and the regenerated slices in
// block order, each slice patched by the last-byte rule (x264 padding correction, 1345-1356).
// slice(k, &p, &len) gives plan slice k's regenerated bytes and returns its status.
template <class Slice>
int splice_job(avr_ctx* c, const DecJob& j, Slice&& slice, std::vector<uint8_t>* o) {
  o->reserve(j.stream.size());
  for (size_t i = 0; i < j.blocks.size(); i++) {
    const avr::PbBlock& b = j.blocks[i];
    if (b.has_literal) {
      o->insert(o->end(), b.literal, b.literal + b.literal_len);
      continue;
    }
    if (!b.has_cabac) continue;
    const int k = j.desc_of_block[i];
    if (k == -1) return fail(c, AVR_ERR_FORMAT, "Not all blocks were decoded.");
    const uint8_t* p = nullptr;
    size_t len = 0;
    if (int stt = slice(k, &p, &len))
      return fail(c, AVR_ERR_FORMAT, "slice " + std::to_string(k) + " failed to decode (" + std::to_string(stt) + ")");
    const size_t o0 = o->size();
    o->insert(o->end(), p, p + len);
    if (b.has_parity && b.has_last_byte && !b.last_byte.empty()) {
      const size_t n = o->size() - o0;
      if ((int)b.length_parity != (int)(n & 1)) o->push_back((uint8_t)b.last_byte[0]);
      else if (n) o->back() = (uint8_t)b.last_byte[0];
    }
  }
  return AVR_OK;
}

int decompress_files(avr_ctx* c, int nf, const uint8_t* const* in, const size_t* in_len, uint8_t** out,
                     size_t* out_len, int32_t* status, std::vector<Bill>* bills = nullptr) {
  HIP_TRY(c, hipSetDevice(c->device));
  PhaseClock pc(c);
  if (bills) bills->assign(nf, Bill{});
  const uint32_t flags = bills ? avr::kFlagBill : 0;
  std::vector<int32_t> st(nf, AVR_OK);
  std::vector<DecJob> jobs(nf);
  // plans[AVR_MODEL_*]: reference-model files (one workgroup each); parallel-model slices on the
  // u64 coder; on the P32 coder
  Plan plans[3];   // indexed by plan_of(model): the chained model's chains go to the reference plan
  Plan& rp = plans[AVR_MODEL_REFERENCE];
  SplitPlan sp;    // the pieces of split blocks
  auto plan_of = [](int m) { return parallel_model(m) ? m : (int)AVR_MODEL_REFERENCE; };
  for (int f = 0; f < nf; f++) {
    out[f] = nullptr;
    out_len[f] = 0;
    std::string version;
    std::vector<avr::PbBlock> probe;
    const int m = avr::pb_parse(in[f], in_len[f], &probe, &version) ? std::max(0, avr::model_of_version(version)) : 0;
    const bool parallel = parallel_model(m);
    Plan* plan = &plans[plan_of(m)];
    const size_t n0 = plan->descs.size();
    if (!parallel) rp.file_first.push_back((int)n0);
    const size_t s_descs = sp.plan.descs.size(), s_recs = sp.recs.size(), s_arena = sp.plan.arena.size();
    st[f] = decompress_setup(c, in[f], in_len[f], &jobs[f], plan, &sp);
    if (st[f]) {   // drop whatever the failed file left
      plan->descs.resize(n0);
      sp.plan.descs.resize(s_descs);
      sp.ctl.resize(s_descs);
      sp.recs.resize(s_recs);
      sp.plan.arena.resize(s_arena);
      if (!parallel) rp.file_first.pop_back();
    } else if (jobs[f].model == AVR_MODEL_CHAINED) {
      // one workgroup per chain: a new "file" of the sequential launch before every
      // AVR_CHAIN_SLICES-th coded slice (the compress side's boundaries)
      int coded_n = 0;
      for (size_t k = n0; k < plan->descs.size(); k++) {
        if (!plan->descs[k].coded) continue;
        if (coded_n > 0 && coded_n % AVR_CHAIN_SLICES == 0) rp.file_first.push_back((int)k);
        coded_n++;
      }
    }
  }
  std::vector<avr_slice_result> res_of[3];
  std::vector<uint8_t> out_of[3];
  pc.mark_demux();
  // the pieces of split blocks on the split stream, beside the other plans
  std::vector<avr_slice_result> pr;
  Bytes po;
  SplitPending pend;
  double t_split = 0;
  if (!sp.plan.descs.empty()) {
    const double t = now_s();
    hipStream_t ss = c->split_stream;
    HIP_TRY(c, c->sp_in.reserve(sp.plan.arena.size() + 4096));
    HIP_TRY(c, c->sp_recs.reserve(sp.recs.size() + 64));
    HIP_TRY(c, hipMemcpyAsync(c->sp_in.p, sp.plan.arena.data(), sp.plan.arena.size(), hipMemcpyHostToDevice, ss));
    HIP_TRY(c, hipMemcpyAsync(c->sp_recs.p, sp.recs.data(), sp.recs.size(), hipMemcpyHostToDevice, ss));
    if (int r = split_launch(c, 1, sp.plan.descs, sp.ctl, c->sp_in.as<uint8_t>(), sp.plan.max_w, sp.stride, flags, &pr,
                             &po, &c->sp_out, &pend)) {
      (void)hipStreamSynchronize(ss);
      return r;
    }
    t_split += now_s() - t;
  }
  auto drain = [&]() { (void)hipStreamSynchronize(c->split_stream); };
  for (int m = AVR_MODEL_PARALLEL; m <= AVR_MODEL_PARALLEL32; m++)
    if (!plans[m].descs.empty())
      if (int r = run_plan(c, 1, false, plans[m], &res_of[m], &out_of[m], false, flags | coder_flag(m))) {
        drain();
        return r;
      }
  if (!rp.file_first.empty()) {
    rp.file_first.push_back((int)rp.descs.size());
    if (int r = run_plan(c, 1, true, rp, &res_of[0], &out_of[0], false, flags)) {
      drain();
      return r;
    }
  }
  if (!sp.plan.descs.empty()) {   // the pieces of split blocks, then each block spliced
    const double t = now_s();
    if (int r = split_wait(c, &pend)) return r;
    for (int f = 0; f < nf; f++) {
      if (st[f]) continue;
      for (SplitBlock& x : jobs[f].splits) {
        std::vector<const uint8_t*> pp(x.pieces);
        std::vector<uint32_t> len(x.pieces);
        std::vector<int32_t> stt(x.pieces);
        for (int i = 0; i < x.pieces; i++) {
          const int k = x.first + i;
          pp[i] = po.data() + sp.plan.descs[k].out_offset;
          len[i] = pr[k].out_len;
          stt[i] = pr[k].status;
          if (pr[k].status == 0)
            for (int b = 0; b < 6; b++) x.bill.bill[b] += pr[k].bill[b];
        }
        x.status = splice_pieces(pp, len, stt, x.q, &x.regen) ? 0 : AVR_SLICE_NO_END;
        for (int i = 0; i < x.pieces && !x.status; i++) x.status = stt[i];
      }
    }
    c->plan_wall += t_split + (now_s() - t);
  }
  int first_err = AVR_OK;
  for (int f = 0; f < nf; f++) {
    DecJob& j = jobs[f];
    const Plan& plan = plans[plan_of(j.model)];
    const std::vector<avr_slice_result>& res = res_of[plan_of(j.model)];
    const std::vector<uint8_t>& outb = out_of[plan_of(j.model)];
    std::vector<uint8_t> o;
    if (st[f] == AVR_OK)
      st[f] = splice_job(c, j, [&](int k, const uint8_t** p, size_t* len) {
        if (k <= -2) {   // a split block, spliced from its pieces
          const SplitBlock& x = j.splits[-2 - k];
          *p = x.regen.data();
          *len = x.regen.size();
          if (bills && x.status == 0) add_bill(&(*bills)[f], x.bill);
          return (int)x.status;
        }
        *p = outb.data() + plan.descs[k].out_offset;
        *len = res[k].out_len;
        if (bills && res[k].status == 0) add_bill(&(*bills)[f], res[k]);
        return res[k].status;
      }, &o);
    if (st[f] == AVR_OK) {
      out[f] = (uint8_t*)malloc(o.size() ? o.size() : 1);
      if (!out[f]) {
        st[f] = AVR_ERR_OUT_OF_MEMORY;
      } else {
        if (!o.empty()) memcpy(out[f], o.data(), o.size());
        out_len[f] = o.size();
      }
    }
    if (status) status[f] = st[f];
    if (st[f] && !first_err) first_err = st[f];
  }
  pc.finish();
  return status ? AVR_OK : first_err;
}

// ------------------------------------------------------------ the chained model across GPUs
// The chained model's chains are independent by construction (a fresh model -- estimators, frames --
// before every AVR_CHAIN_SLICES-th coded slice of a file), so one file's chains can run on several
// GPUs: each rank takes a contiguous range of chains, balanced by payload bytes, and the re-coded
// (or regenerated) slices are gathered to rank 0, which assembles (splices) them as for the
// parallel model.  Chain c of a file starts at slice first[c]: the slice holding the
// (AVR_CHAIN_SLICES c)-th coded slice (uncoded slices before it stay in chain c - 1, where they
// only turn the old chain's frames over); first.back() = the slice count.
std::vector<int> chain_starts(const std::vector<char>& coded) {
  std::vector<int> first{0};
  int coded_n = 0;
  for (size_t i = 0; i < coded.size(); i++) {
    if (!coded[i]) continue;
    if (coded_n > 0 && coded_n % AVR_CHAIN_SLICES == 0) first.push_back((int)i);
    coded_n++;
  }
  first.push_back((int)coded.size());
  return first;
}

// [lo, hi) of rank's contiguous range of units weighted w: shard.partition's rule (the owner of a
// unit is the rank its byte-prefix midpoint falls in), so both sides cut identically.
std::pair<int, int> partition_range(const std::vector<double>& w, int world, int rank) {
  const int n = (int)w.size();
  if (world <= 1) return rank == 0 ? std::make_pair(0, n) : std::make_pair(n, n);
  double total = 0;
  for (double x : w) total += x;
  std::vector<int> cuts(world + 1, n);
  if (total <= 0) {
    for (int r = 0; r < world; r++) cuts[r] = (int)std::nearbyint((double)r * n / world);
  } else {
    std::vector<int> owner(n);
    double acc = 0;
    for (int i = 0; i < n; i++) {
      acc += w[i];
      const double mid = acc - w[i] / 2;
      owner[i] = std::min((int)(mid * world / total), world - 1);
    }
    for (int r = 0; r < world; r++) cuts[r] = (int)(std::lower_bound(owner.begin(), owner.end(), r) - owner.begin());
  }
  return {cuts[rank], cuts[rank + 1]};
}

// One rank's outputs over its slice range [lo, hi) of the file (compress) or of the container's
// plan (decompress): per slice a status and its bytes (blob + offsets[k], lens[k]).
struct ChainRangeOut {
  int lo = 0, hi = 0;
  std::vector<int32_t> status;
  std::vector<uint64_t> offsets;
  std::vector<uint32_t> lens;
  std::vector<uint8_t> blob;
};

// compressor::run (recode.cpp:1102-1132) of the chained model, this rank's chains only: the parse
// and the segmentation of the whole file (the coded slices, hence the chains, depend on every block
// before them), then the reference-model pass over the chains [clo, chi) (run_plan: one workgroup
// per chain, or the parallel reference-model compress when it pays).  status: 0 coded (bytes),
// -1 not coded, -2 a coded slice the pass failed (the whole-file call would demote it and
// re-segment, moving every later chain: the caller compresses the file whole instead).
int compress_chain_range(avr_ctx* c, const uint8_t* in, size_t n, int world, int rank, ChainRangeOut* o) {
  HIP_TRY(c, hipSetDevice(c->device));
  ParsedFile pf;
  if (int r = parse_file(c, in, n, &pf, /*views=*/true)) return r;
  const size_t ns = pf.slices.size();
  std::vector<char> ok(ns), coded(ns);
  for (size_t i = 0; i < ns; i++) ok[i] = recodable_candidate(pf.slices[i]);
  const std::vector<const uint8_t*> found = segment(in, n, pf, ok);
  for (size_t i = 0; i < ns; i++) coded[i] = found[i] != nullptr;
  const std::vector<int> first = chain_starts(coded);
  const int nc = (int)first.size() - 1;
  std::vector<double> w(nc, 0.0);
  for (int ch = 0; ch < nc; ch++)
    for (int i = first[ch]; i < first[ch + 1]; i++)
      if (coded[i]) w[ch] += (double)pf.slices[i].size;
  const auto [clo, chi] = partition_range(w, world, rank);
  o->lo = first[clo];
  o->hi = first[chi];
  const int nr = o->hi - o->lo;
  o->status.assign(nr, -1);
  o->offsets.assign(nr, 0);
  o->lens.assign(nr, 0);
  o->blob.clear();
  if (chi <= clo) return AVR_OK;
  Plan rp;
  for (int ch = clo; ch < chi; ch++) {
    rp.file_first.push_back((int)rp.descs.size());
    for (int i = first[ch]; i < first[ch + 1]; i++) {   // as compress_files builds a chain
      const avr::SliceInfo& s = pf.slices[i];
      avr_slice_desc d = desc_from_header(s);
      d.coded = coded[i];
      if (d.coded) {
        append_aligned(&rp.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
        d.payload_size = (uint32_t)s.size;
        d.read_limit = (uint32_t)s.read_limit;
        d.out_capacity = (uint32_t)(s.size * 4 + 4096);
        rp.max_w = std::max(rp.max_w, ring_cols(d));
      }
      rp.descs.push_back(d);
    }
  }
  rp.file_first.push_back((int)rp.descs.size());
  std::vector<avr_slice_result> rr;
  Bytes ro;
  if (int r = run_plan(c, 0, true, rp, &rr, &ro, false, 0)) return r;
  uint64_t total = 0;
  for (int k = 0; k < nr; k++)
    if (rp.descs[k].coded && rr[k].status == 0) total += rr[k].out_len;
  o->blob.resize(total);
  uint64_t at = 0;
  for (int k = 0; k < nr; k++) {
    if (!rp.descs[k].coded) continue;
    if (rr[k].status != 0) {
      o->status[k] = -2;
      continue;
    }
    o->status[k] = 0;
    o->offsets[k] = at;
    o->lens[k] = rr[k].out_len;
    if (rr[k].out_len) memcpy(o->blob.data() + at, ro.data() + rp.descs[k].out_offset, rr[k].out_len);
    at += rr[k].out_len;
  }
  return AVR_OK;
}

// decompressor::run (recode.cpp:1312-1357) of a chained-model container, this rank's chains only:
// the container planned as the whole-file call plans it (every slice, coded or not: the reference
// model turns frames over on uncoded ones), the chains cut by the same rule, and the plan's slices
// [lo, hi) of this rank's chains regenerated on the device (one workgroup per chain).  status per
// plan slice: 0 regenerated (bytes), 1 not coded, < 0 failed.  The caller splices the gathered
// slices with avr_dec_plan_splice (rank 0's plan of the same container).
int decompress_chain_range(avr_ctx* c, const uint8_t* avrc, size_t n, int world, int rank, ChainRangeOut* o) {
  HIP_TRY(c, hipSetDevice(c->device));
  DecJob j;
  Plan full;
  full.layout_only = true;
  if (int r = decompress_setup(c, avrc, n, &j, &full)) return r;
  if (!reference_model(j.model)) return fail(c, AVR_ERR_UNSUPPORTED, "not a reference- or chained-model container");
  const int ns = (int)full.descs.size();
  std::vector<char> coded(ns);
  for (int k = 0; k < ns; k++) coded[k] = full.descs[k].coded != 0;
  // the reference model (one chain per file) is a single unit; the chained model's chains
  const std::vector<int> first = j.model == AVR_MODEL_CHAINED ? chain_starts(coded) : std::vector<int>{0, ns};
  const int nc = (int)first.size() - 1;
  std::vector<double> w(nc, 0.0);
  for (int ch = 0; ch < nc; ch++)
    for (int k = first[ch]; k < first[ch + 1]; k++)
      if (coded[k]) w[ch] += (double)full.descs[k].payload_size;
  const auto [clo, chi] = partition_range(w, world, rank);
  o->lo = first[clo];
  o->hi = first[chi];
  const int nr = o->hi - o->lo;
  o->status.assign(nr, 1);
  o->offsets.assign(nr, 0);
  o->lens.assign(nr, 0);
  o->blob.clear();
  if (chi <= clo) return AVR_OK;
  // the range's re-coded streams: decompress_setup listed every coded slice's copy in plan order
  Plan sub;
  size_t ci = 0;
  for (int k = 0; k < ns && k < o->hi; k++) {
    avr_slice_desc d = full.descs[k];
    const avr::PbCopy* cp = d.coded ? &full.arena_copies[ci++] : nullptr;
    if (k < o->lo) continue;
    if (cp) {
      append_aligned(&sub.arena, cp->src, cp->len, 16, &d.payload_offset);
      sub.max_w = std::max(sub.max_w, ring_cols(d));
    }
    sub.descs.push_back(d);
  }
  for (int ch = clo; ch <= chi; ch++) sub.file_first.push_back(first[ch] - o->lo);
  std::vector<avr_slice_result> rr;
  Bytes ro;
  if (int r = run_plan(c, 1, true, sub, &rr, &ro, false, 0)) return r;
  uint64_t total = 0;
  for (int k = 0; k < nr; k++)
    if (sub.descs[k].coded && rr[k].status == 0) total += rr[k].out_len;
  o->blob.resize(total);
  uint64_t at = 0;
  for (int k = 0; k < nr; k++) {
    if (!sub.descs[k].coded) continue;
    o->status[k] = rr[k].status == 0 ? 0 : std::min(-1, (int)rr[k].status);
    if (rr[k].status != 0) continue;
    o->offsets[k] = at;
    o->lens[k] = rr[k].out_len;
    if (rr[k].out_len) memcpy(o->blob.data() + at, ro.data() + sub.descs[k].out_offset, rr[k].out_len);
    at += rr[k].out_len;
  }
  return AVR_OK;
}

// a ChainRangeOut to the caller's malloc'd buffers (avr_free)
int export_range(const ChainRangeOut& o, int* lo, int* hi, int32_t** status, uint8_t** blob, size_t* blob_len,
                 uint64_t** offsets, uint32_t** lens) {
  const size_t nr = (size_t)(o.hi - o.lo);
  *status = (int32_t*)malloc(sizeof(int32_t) * std::max<size_t>(1, nr));
  *offsets = (uint64_t*)malloc(sizeof(uint64_t) * std::max<size_t>(1, nr));
  *lens = (uint32_t*)malloc(sizeof(uint32_t) * std::max<size_t>(1, nr));
  *blob = host_alloc(std::max<size_t>(1, o.blob.size()));
  if (!*status || !*offsets || !*lens || !*blob) {
    free(*status), free(*offsets), free(*lens), free(*blob);
    *status = nullptr, *offsets = nullptr, *lens = nullptr, *blob = nullptr;
    return AVR_ERR_OUT_OF_MEMORY;
  }
  if (nr) {
    memcpy(*status, o.status.data(), sizeof(int32_t) * nr);
    memcpy(*offsets, o.offsets.data(), sizeof(uint64_t) * nr);
    memcpy(*lens, o.lens.data(), sizeof(uint32_t) * nr);
  }
  if (!o.blob.empty()) memcpy(*blob, o.blob.data(), o.blob.size());
  *blob_len = o.blob.size();
  *lo = o.lo;
  *hi = o.hi;
  return AVR_OK;
}

}  // namespace

// ================================================================================ C ABI
extern "C" {

int avr_create(int device, avr_ctx** out) {
  if (!out) return AVR_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return AVR_ERR_DEVICE;
  std::unique_ptr<avr_ctx> c(new avr_ctx());
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) return AVR_ERR_DEVICE;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return AVR_ERR_DEVICE;
  if (hipStreamCreateWithFlags(&c->split_stream, hipStreamNonBlocking) != hipSuccess) return AVR_ERR_DEVICE;
  {
    const char* e = getenv("AVR_SPLIT_BYTES");
    c->split_bytes = e ? (size_t)strtoull(e, nullptr, 10) : kSplitBytesDefault;
  }
  if (const char* e = getenv("AVR_FIELD_LANE"); !e || strcmp(e, "0") != 0) {
    if (hipStreamCreateWithFlags(&c->fld_stream, hipStreamNonBlocking) != hipSuccess) return AVR_ERR_DEVICE;
    for (auto& ev : c->fld_ev)
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return AVR_ERR_DEVICE;
  }
  avr::EngineTables t;
  build_tables(&t);
  if (!check_reciprocals(t)) return AVR_ERR_DEVICE;
  if (c->tables.reserve(sizeof(t)) != hipSuccess) return AVR_ERR_OUT_OF_MEMORY;
  if (hipMemcpy(c->tables.p, &t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess) return AVR_ERR_DEVICE;
  // CU grouping of the slice kernels only where the dispatcher deals workgroups round-robin
  if (avr::probe_round_robin(avr::shared_bytes(120), &c->round_robin) != hipSuccess) return AVR_ERR_DEVICE;
  if (getenv("AVR_NO_SCHEDULE")) c->round_robin = false;
  *out = c.release();
  return AVR_OK;
}

void avr_destroy(avr_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;   // every DevBuf frees itself
}

const char* avr_last_error(const avr_ctx* c) { return c ? c->err.c_str() : "no context"; }

int avr_set_split_bytes(avr_ctx* c, size_t bytes) {
  if (!c || bytes >= ((size_t)1 << 28)) return AVR_ERR_INVALID_ARGUMENT;
  c->split_bytes = bytes;
  return AVR_OK;
}
size_t avr_get_split_bytes(const avr_ctx* c) { return c ? c->split_bytes : 0; }

void avr_free(void* p) { free(p); }

// ------------------------------------------------------------------ sharded decompress plans
// decompressor::run (recode.cpp:1338-1409) cut in two around the device work: load = read_packet's
// surrogate stream parsed and matched to the container's coded blocks (decompress_setup in layout
// mode: descs and the arena layout, no bytes copied), then the arena written where the caller wants
// it, and the splice of the regenerated slices with the literals and the last-byte patch
// (recode.cpp:1345-1356).  A handle keeps its scratch (the surrogate stream) for the next load.
}  // extern "C"
struct avr_dec_plan {
  DecJob job;
  Plan plan;
  uint64_t work = 0;
  int max_h = 1;
  const uint8_t* avrc = nullptr;   // the caller's container (the blocks point into it)
  size_t n = 0;
};
extern "C" {

int avr_dec_plan_new(avr_dec_plan** out) {
  if (!out) return AVR_ERR_INVALID_ARGUMENT;
  return guarded(nullptr, [&]() -> int {
    *out = new avr_dec_plan();
    return AVR_OK;
  });
}

void avr_dec_plan_free(avr_dec_plan* h) { delete h; }

int avr_dec_plan_load(avr_dec_plan* h, const uint8_t* avrc, size_t n, int* n_slices, size_t* arena_len,
                      size_t* work_len, int* max_mb_width, int* max_mb_height) {
  if (!h || !avrc || !n_slices || !arena_len || !work_len || !max_mb_width || !max_mb_height)
    return AVR_ERR_INVALID_ARGUMENT;
  return guarded(nullptr, [&]() -> int {
    h->avrc = nullptr;
    h->job.blocks.clear();
    h->job.desc_of_block.clear();
    h->job.stream.clear();   // keeps its capacity: the next stream is written over mapped pages
    h->plan.descs.clear();
    h->plan.arena_copies.clear();
    h->plan.arena_end = 0;
    h->plan.max_w = 1;
    h->plan.layout_only = true;
    if (int r = decompress_setup(nullptr, avrc, n, &h->job, &h->plan)) return r;
    uint64_t w = 0;
    int mh = 1;
    for (auto& d : h->plan.descs) {
      d.out_offset = w;
      w += ((uint64_t)d.out_capacity + 15) & ~15ull;
      mh = std::max(mh, d.mb_height);
    }
    h->avrc = avrc;
    h->n = n;
    h->work = w;
    h->max_h = mh;
    *n_slices = (int)h->plan.descs.size();
    *arena_len = h->plan.arena_end + 16;
    *work_len = w;
    *max_mb_width = h->plan.max_w;
    *max_mb_height = mh;
    return AVR_OK;
  });
}

int avr_dec_plan_descs(const avr_dec_plan* h, avr_slice_desc* out) {
  if (!h || !h->avrc || (!out && !h->plan.descs.empty())) return AVR_ERR_INVALID_ARGUMENT;
  if (!h->plan.descs.empty()) memcpy(out, h->plan.descs.data(), sizeof(avr_slice_desc) * h->plan.descs.size());
  return AVR_OK;
}

int avr_dec_plan_arena(const avr_dec_plan* h, uint8_t* out, size_t cap) {
  if (!h || !h->avrc || !out || cap < h->plan.arena_end + 16) return AVR_ERR_INVALID_ARGUMENT;
  return guarded(nullptr, [&]() -> int {
    const auto& cp = h->plan.arena_copies;
    const uint64_t end = h->plan.arena_end + 16;
    uint64_t z = 0;   // the zero bytes between and after the streams
    for (const auto& c : cp) {
      memset(out + z, 0, c.dst - z);
      z = c.dst + c.len;
    }
    memset(out + z, 0, end - z);
    parallel_copies(cp, out);
    return AVR_OK;
  });
}

}  // extern "C"
namespace {
// splice_job's output laid out: the literal and regenerated-slice copies, the last-byte patches
// (position, byte) and the total length.
int splice_layout(const avr_dec_plan* h, const int32_t* status, const uint8_t* regen, size_t regen_len,
                  const uint64_t* offsets, const uint32_t* lens, std::vector<avr::PbCopy>* copies,
                  std::vector<std::pair<size_t, uint8_t>>* patches, size_t* total) {
  const DecJob& j = h->job;
  const int ns = (int)h->plan.descs.size();
  // every slice's regenerated bytes inside regen and within its own output capacity
  for (int k = 0; k < ns; k++)
    if (status[k] == 0 && (offsets[k] > regen_len || lens[k] > regen_len - offsets[k] ||
                           lens[k] > h->plan.descs[k].out_capacity))
      return AVR_ERR_INVALID_ARGUMENT;
  copies->reserve(j.blocks.size());
  size_t at = 0;
  for (size_t i = 0; i < j.blocks.size(); i++) {
    const avr::PbBlock& b = j.blocks[i];
    if (b.has_literal) {
      if (b.literal_len) copies->push_back({at, b.literal, b.literal_len});
      at += b.literal_len;
      continue;
    }
    if (!b.has_cabac) continue;
    const int k = j.desc_of_block[i];
    if (k < 0) return AVR_ERR_FORMAT;          // "Not all blocks were decoded." (recode.cpp:1354)
    if (status[k]) return AVR_ERR_FORMAT;      // the slice failed to decode
    const size_t len = lens[k];
    if (len) copies->push_back({at, regen + offsets[k], len});
    size_t m = len;
    if (b.has_parity && b.has_last_byte && !b.last_byte.empty()) {   // recode.cpp:1345-1356
      if ((int)b.length_parity != (int)(m & 1)) patches->push_back({at + m, (uint8_t)b.last_byte[0]}), m++;
      else if (m) patches->push_back({at + m - 1, (uint8_t)b.last_byte[0]});
    }
    at += m;
  }
  *total = at;
  return AVR_OK;
}
}  // namespace
extern "C" {

int avr_dec_plan_splice(const avr_dec_plan* h, const int32_t* status, const uint8_t* regen, size_t regen_len,
                        const uint64_t* offsets, const uint32_t* lens, uint8_t* out, size_t out_cap, size_t* out_len) {
  const int ns = h ? (int)h->plan.descs.size() : 0;
  if (!h || !h->avrc || !out_len || (ns && (!status || !regen || !offsets || !lens))) return AVR_ERR_INVALID_ARGUMENT;
  *out_len = 0;
  return guarded(nullptr, [&]() -> int {
    std::vector<avr::PbCopy> copies;
    std::vector<std::pair<size_t, uint8_t>> patches;
    size_t total = 0;
    if (int r = splice_layout(h, status, regen, regen_len, offsets, lens, &copies, &patches, &total)) return r;
    *out_len = total;
    if (total > out_cap || (total && !out)) return AVR_ERR_INVALID_ARGUMENT;
    parallel_copies(copies, out);
    for (const auto& pt : patches) out[pt.first] = pt.second;
    return AVR_OK;
  });
}

int avr_plan_decompress(const uint8_t* avrc, size_t n, avr_slice_desc** descs, int* n_slices, uint8_t** arena,
                        size_t* arena_len, size_t* work_len, int* max_mb_width, int* max_mb_height) {
  if (!avrc || !descs || !n_slices || !arena || !arena_len || !work_len || !max_mb_width || !max_mb_height)
    return AVR_ERR_INVALID_ARGUMENT;
  *descs = nullptr;
  *arena = nullptr;
  return guarded(nullptr, [&]() -> int {
    avr_dec_plan h;
    int ns = 0;
    size_t al = 0;
    if (int r = avr_dec_plan_load(&h, avrc, n, &ns, &al, work_len, max_mb_width, max_mb_height)) return r;
    // a slice batch for slice-range sharding: the parallel models only (the reference model's
    // slices chain; the chained model shards by chains, avr_decompress_chain_range)
    if (!h.job.parallel) return AVR_ERR_UNSUPPORTED;
    *descs = (avr_slice_desc*)malloc(sizeof(avr_slice_desc) * std::max(1, ns));
    *arena = host_alloc(al);
    if (!*descs || !*arena) {
      free(*descs);
      free(*arena);
      *descs = nullptr;
      *arena = nullptr;
      return AVR_ERR_OUT_OF_MEMORY;
    }
    avr_dec_plan_descs(&h, *descs);
    if (int r = avr_dec_plan_arena(&h, *arena, al)) return r;
    *n_slices = ns;
    *arena_len = al;
    return AVR_OK;
  });
}

int avr_splice_container(const uint8_t* avrc, size_t n, int n_slices, const int32_t* status, const uint8_t* regen,
                         size_t regen_len, const uint64_t* offsets, const uint32_t* lens, uint8_t** out,
                         size_t* out_len) {
  if (!avrc || n_slices < 0 || (n_slices && (!status || !regen || !offsets || !lens)) || !out || !out_len)
    return AVR_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  return guarded(nullptr, [&]() -> int {
    avr_dec_plan h;
    int ns = 0, mw = 0, mh = 0;
    size_t al = 0, wl = 0;
    if (int r = avr_dec_plan_load(&h, avrc, n, &ns, &al, &wl, &mw, &mh)) return r;
    if (ns != n_slices) return AVR_ERR_INVALID_ARGUMENT;
    std::vector<avr::PbCopy> copies;
    std::vector<std::pair<size_t, uint8_t>> patches;
    size_t total = 0;
    if (int r = splice_layout(&h, status, regen, regen_len, offsets, lens, &copies, &patches, &total)) return r;
    uint8_t* o = host_alloc(total);
    if (!o) return AVR_ERR_OUT_OF_MEMORY;
    parallel_copies(copies, o);
    for (const auto& pt : patches) o[pt.first] = pt.second;
    *out = o;
    *out_len = total;
    return AVR_OK;
  });
}

int avr_last_phase_times(const avr_ctx* c, avr_phase_times* out) {
  if (!c || !out) return AVR_ERR_INVALID_ARGUMENT;
  *out = c->phase;
  return AVR_OK;
}

int avr_neighbor_tables(avr_ctx* c, uint8_t out[96]) {
  if (!out) return AVR_ERR_INVALID_ARGUMENT;
  static_assert(offsetof(avr::HotTables, nb_up) == offsetof(avr::HotTables, nb_left) + 48, "nb_left, nb_up adjacent");
  if (!c) {
    std::unique_ptr<avr::EngineTables> t(new avr::EngineTables());
    build_tables(t.get());
    memcpy(out, t->hot.nb_left, 96);
    return AVR_OK;
  }
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t off = offsetof(avr::EngineTables, hot) + offsetof(avr::HotTables, nb_left);
  HIP_TRY(c, hipMemcpy(out, c->tables.as<uint8_t>() + off, 96, hipMemcpyDeviceToHost));
  return AVR_OK;
}

int avr_compress_file(avr_ctx* c, const uint8_t* in, size_t n, int model, uint8_t** out, size_t* out_len) {
  if (!c || !in || !out || !out_len || !valid_model(model)) return AVR_ERR_INVALID_ARGUMENT;
  int32_t st = 0;
  const int r = guarded(c, [&] { return compress_files(c, 1, &in, &n, model, out, out_len, &st); });
  return r ? r : st;
}

int avr_compress_files(avr_ctx* c, int n_files, const uint8_t* const* in, const size_t* in_len, int model,
                       uint8_t** out, size_t* out_len, int32_t* status) {
  if (!c || n_files < 0 || (n_files && (!in || !in_len || !out || !out_len)) || !valid_model(model))
    return AVR_ERR_INVALID_ARGUMENT;
  for (int f = 0; f < n_files; f++)
    if (!in[f]) return AVR_ERR_INVALID_ARGUMENT;
  return guarded(c, [&] { return compress_files(c, n_files, in, in_len, model, out, out_len, status); });
}

namespace {
// Rank 0's container from gathered per-slice outputs (both avr_assemble_container entry points).
int assemble(const uint8_t* file, size_t n, int model, const std::vector<SliceView>& sv, const int32_t* status,
             const uint8_t* recoded, size_t recoded_len, const uint64_t* offsets, const uint32_t* lens, uint8_t** out,
             size_t* out_len, uint8_t* dst = nullptr, size_t cap = 0) {
  std::vector<char> ok(sv.size(), 0);
  std::vector<std::pair<const uint8_t*, size_t>> blobs(sv.size(), {nullptr, 0});
  for (size_t i = 0; i < sv.size(); i++) {
    ok[i] = sv[i].candidate && status[i] == 0;
    if (ok[i]) {
      if (!recoded || offsets[i] > recoded_len || lens[i] > recoded_len - offsets[i]) return AVR_ERR_INVALID_ARGUMENT;
      blobs[i] = {recoded + offsets[i], lens[i]};
    }
  }
  const double t0 = now_s();
  const std::vector<const uint8_t*> found = segment(file, n, sv, ok);
  const double t1 = now_s();
  const int r = emit_container(file, n, sv, found, blobs, model, out, out_len, dst, cap);
  if (getenv("AVR_ASM_TIMING")) fprintf(stderr, "assemble: segment %.3f s, emit %.3f s\n", t1 - t0, now_s() - t1);
  return r;
}
}  // namespace

int avr_assemble_container(const uint8_t* file, size_t n, int model, int n_slices, const int32_t* status,
                           const uint8_t* recoded, size_t recoded_len, const uint64_t* offsets, const uint32_t* lens,
                           uint8_t** out, size_t* out_len) {
  if (!file || !out || !out_len || n_slices < 0 || (n_slices && (!status || !offsets || !lens)) || !assemblable(model))
    return AVR_ERR_INVALID_ARGUMENT;
  return guarded(nullptr, [&]() -> int {
    ParsedFile pf;
    if (int r = parse_file(nullptr, file, n, &pf, /*views=*/true)) return r;
    if ((size_t)n_slices != pf.slices.size()) return AVR_ERR_INVALID_ARGUMENT;
    return assemble(file, n, model, views_of(pf), status, recoded, recoded_len, offsets, lens, out, out_len);
  });
}

namespace {
int assemble_parsed(const uint8_t* file, size_t n, int model, const avr_slice_desc* descs, int n_slices,
                    const uint8_t* arena, size_t arena_len, const int32_t* status, const uint8_t* recoded,
                    size_t recoded_len, const uint64_t* offsets, const uint32_t* lens, uint8_t** out, size_t* out_len,
                    uint8_t* dst, size_t cap) {
  if (!file || !out_len || n_slices < 0 || (n_slices && (!descs || !arena || !status || !offsets || !lens)) ||
      !assemblable(model))
    return AVR_ERR_INVALID_ARGUMENT;
  return guarded(nullptr, [&]() -> int {
    std::vector<SliceView> sv((size_t)n_slices);
    for (int i = 0; i < n_slices; i++) {
      const avr_slice_desc& d = descs[i];
      if (d.payload_offset > arena_len || d.payload_size > arena_len - d.payload_offset) return AVR_ERR_INVALID_ARGUMENT;
      // only avr_parse_stream's own descriptors of this file: a coded slice is one recodable_candidate
      // accepted (a surrogate marker long, its LDS ring within a workgroup), and a payload the parse
      // found verbatim stands at file_offset (its first and last bytes checked: O(1) per slice)
      if (d.coded && (d.payload_size < (uint32_t)avr::kSurrogateMarkerBytes ||
                      avr::shared_bytes(ring_cols(d)) > kLdsBudget))
        return AVR_ERR_INVALID_ARGUMENT;
      const uint8_t* P = arena + d.payload_offset;
      const size_t m = d.payload_size;
      if (d.file_offset != ~(uint64_t)0) {
        const size_t k = std::min<size_t>(m, 16);
        if (d.file_offset > n || m > n - d.file_offset || memcmp(file + d.file_offset, P, k) != 0 ||
            memcmp(file + d.file_offset + m - k, P + m - k, k) != 0)
          return AVR_ERR_INVALID_ARGUMENT;
      }
      sv[i] = {P, m, d.coded != 0, d.file_offset};
    }
    return assemble(file, n, model, sv, status, recoded, recoded_len, offsets, lens, out, out_len, dst, cap);
  });
}
}  // namespace

int avr_assemble_container_parsed(const uint8_t* file, size_t n, int model, const avr_slice_desc* descs, int n_slices,
                                  const uint8_t* arena, size_t arena_len, const int32_t* status,
                                  const uint8_t* recoded, size_t recoded_len, const uint64_t* offsets,
                                  const uint32_t* lens, uint8_t** out, size_t* out_len) {
  if (!out) return AVR_ERR_INVALID_ARGUMENT;
  return assemble_parsed(file, n, model, descs, n_slices, arena, arena_len, status, recoded, recoded_len, offsets, lens,
                         out, out_len, nullptr, 0);
}

int avr_assemble_container_into(const uint8_t* file, size_t n, int model, const avr_slice_desc* descs, int n_slices,
                                const uint8_t* arena, size_t arena_len, const int32_t* status, const uint8_t* recoded,
                                size_t recoded_len, const uint64_t* offsets, const uint32_t* lens, uint8_t* out,
                                size_t out_cap, size_t* out_len) {
  if (!out) return AVR_ERR_INVALID_ARGUMENT;
  return assemble_parsed(file, n, model, descs, n_slices, arena, arena_len, status, recoded, recoded_len, offsets, lens,
                         nullptr, out_len, out, out_cap);
}

int avr_container_model(const uint8_t* avrc, size_t n, int* model) {
  if (!avrc || !model) return AVR_ERR_INVALID_ARGUMENT;
  return guarded(nullptr, [&]() -> int {
    std::vector<avr::PbBlock> blocks;
    std::string version;
    if (!avr::pb_parse(avrc, n, &blocks, &version)) return AVR_ERR_FORMAT;
    const int m = avr::model_of_version(version);
    if (m < 0) return AVR_ERR_FORMAT;
    *model = m;
    return AVR_OK;
  });
}

int avr_decompress_file(avr_ctx* c, const uint8_t* in, size_t n, uint8_t** out, size_t* out_len) {
  if (!c || !in || !out || !out_len) return AVR_ERR_INVALID_ARGUMENT;
  int32_t st = 0;
  const int r = guarded(c, [&] { return decompress_files(c, 1, &in, &n, out, out_len, &st); });
  return r ? r : st;
}

int avr_decompress_files(avr_ctx* c, int n_files, const uint8_t* const* in, const size_t* in_len, uint8_t** out,
                         size_t* out_len, int32_t* status) {
  if (!c || n_files < 0 || (n_files && (!in || !in_len || !out || !out_len))) return AVR_ERR_INVALID_ARGUMENT;
  for (int f = 0; f < n_files; f++)
    if (!in[f]) return AVR_ERR_INVALID_ARGUMENT;
  return guarded(c, [&] { return decompress_files(c, n_files, in, in_len, out, out_len, status); });
}

static int roundtrip_file(avr_ctx* c, const uint8_t* in, size_t n, int model, uint8_t** compressed,
                          size_t* compressed_len, avr_file_stats* stats);
int avr_roundtrip_file(avr_ctx* c, const uint8_t* in, size_t n, int model, uint8_t** compressed,
                       size_t* compressed_len, avr_file_stats* stats) {
  return guarded(c, [&] { return roundtrip_file(c, in, n, model, compressed, compressed_len, stats); });
}
static int roundtrip_file(avr_ctx* c, const uint8_t* in, size_t n, int model, uint8_t** compressed,
                          size_t* compressed_len, avr_file_stats* stats) {
  if (!c || !in) return AVR_ERR_INVALID_ARGUMENT;
  if (!valid_model(model)) return AVR_ERR_INVALID_ARGUMENT;
  uint8_t *comp = nullptr, *dec = nullptr;
  size_t cn = 0, dn = 0;
  std::vector<Bill> cbill, dbill;
  int32_t st = 0;
  double tc = 0, td = 0;
  avr_phase_times pcomp{}, pdec{};
  uint32_t attempts = 0;
  auto add_phases = [](avr_phase_times* a, const avr_phase_times& b) {
    a->demux_s += b.demux_s, a->upload_s += b.upload_s, a->kernel_s += b.kernel_s;
    a->download_s += b.download_s, a->container_s += b.container_s, a->other_s += b.other_s;
  };
  bool same = false;
  // the parallel model's per-slice device check is left to the whole-file compare below; a file
  // that does not come back is compressed again with it (every slice that fails it stored as is)
  for (int attempt = parallel_model(model) ? 0 : 1; attempt < 2; attempt++) {
    free(comp);
    comp = nullptr;
    cn = 0;
    attempts++;
    const double t0 = now_s();
    if (int r = compress_files(c, 1, &in, &n, model, &comp, &cn, &st, &cbill, /*verify=*/attempt > 0)) {
      free(comp);
      return r;
    }
    if (st) {
      free(comp);
      return st;
    }
    const double t1 = now_s();
    add_phases(&pcomp, c->phase);
    const uint8_t* cp = comp;
    int r = decompress_files(c, 1, &cp, &cn, &dec, &dn, &st, &dbill);
    if (!r) r = st;
    const double t2 = now_s();
    add_phases(&pdec, c->phase);
    tc += t1 - t0;
    td += t2 - t1;
    same = !r && dn == n && memcmp(dec, in, n) == 0;
    free(dec);
    dec = nullptr;
    if (attempt == 0 && getenv("AVR_ROUNDTRIP_FORCE_VERIFY")) continue;   // tests: the second path
    if (same) break;
    if (attempt == 1 && r) {
      free(comp);
      return r;
    }
  }
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->file_bytes = n;
    stats->compress_s = tc;
    stats->decompress_s = td;
    stats->attempts = attempts;
    stats->compress_phases = pcomp;
    stats->decompress_phases = pdec;
    for (int i = 0; i < 6; i++) {
      stats->bill[i] = cbill[0][i];
      stats->cabac_bill[i] = dbill[0][i];
    }
    std::vector<avr::PbBlock> blocks;
    std::string v;
    if (avr::pb_parse(comp, cn, &blocks, &v)) {
      for (auto& b : blocks) {
        if (b.has_cabac) stats->coded_slices++, stats->payload_bytes += (uint64_t)b.size, stats->recoded_bytes += b.cabac_len;
        if (b.has_skip) stats->skipped_slices++;
      }
      stats->slices = stats->coded_slices + stats->skipped_slices;
    }
  }
  if (compressed && compressed_len) {
    *compressed = comp;
    *compressed_len = cn;
  } else {
    free(comp);
  }
  if (!same) return fail(c, AVR_ERR_ROUNDTRIP, "Compress-decompress roundtrip failed.");
  return AVR_OK;
}

// roundtrip_file's two attempts over a corpus: each attempt is one batched compress_files and one
// batched decompress_files over the files still open.
static int roundtrip_files(avr_ctx* c, int nf, const uint8_t* const* in, const size_t* in_len, int model,
                           uint8_t** out, size_t* out_len, int32_t* status, double* times) {
  for (int f = 0; f < nf; f++) out[f] = nullptr, out_len[f] = 0, status[f] = AVR_ERR_ROUNDTRIP;
  double tc = 0, td = 0;
  std::vector<int> open(nf);
  for (int f = 0; f < nf; f++) open[f] = f;
  const bool force_verify = getenv("AVR_ROUNDTRIP_FORCE_VERIFY") != nullptr;   // tests: the second path
  for (int attempt = parallel_model(model) ? 0 : 1; attempt < 2 && !open.empty(); attempt++) {
    const int k = (int)open.size();
    std::vector<const uint8_t*> ins(k);
    std::vector<size_t> lens(k), clen(k, 0), dlen(k, 0);
    std::vector<uint8_t*> comp(k, nullptr), dec(k, nullptr);
    std::vector<int32_t> cst(k, AVR_OK), dst(k, AVR_OK);
    for (int j = 0; j < k; j++) ins[j] = in[open[j]], lens[j] = in_len[open[j]];
    auto free_all = [&] {
      for (int j = 0; j < k; j++) free(comp[j]), free(dec[j]);
    };
    const double t0 = now_s();
    if (int r = compress_files(c, k, ins.data(), lens.data(), model, comp.data(), clen.data(), cst.data(), nullptr,
                               /*verify=*/attempt > 0)) {
      free_all();
      return r;
    }
    const double t1 = now_s();
    // decompress the containers that came out (a file whose compress failed keeps its status)
    std::vector<int> idx;
    std::vector<const uint8_t*> cin;
    std::vector<size_t> cn;
    for (int j = 0; j < k; j++)
      if (cst[j] == AVR_OK) idx.push_back(j), cin.push_back(comp[j]), cn.push_back(clen[j]);
    std::vector<uint8_t*> dout(idx.size(), nullptr);
    std::vector<size_t> dn(idx.size(), 0);
    std::vector<int32_t> ds(idx.size(), AVR_OK);
    if (!idx.empty()) {
      if (int r = decompress_files(c, (int)idx.size(), cin.data(), cn.data(), dout.data(), dn.data(), ds.data())) {
        for (uint8_t* p : dout) free(p);
        free_all();
        return r;
      }
    }
    for (size_t q = 0; q < idx.size(); q++) dec[idx[q]] = dout[q], dlen[idx[q]] = dn[q], dst[idx[q]] = ds[q];
    const double t2 = now_s();
    tc += t1 - t0;
    td += t2 - t1;
    std::vector<int> again;
    for (int j = 0; j < k; j++) {
      const int f = open[j];
      const bool same = cst[j] == AVR_OK && dst[j] == AVR_OK && dlen[j] == in_len[f] &&
                        (in_len[f] == 0 || memcmp(dec[j], in[f], in_len[f]) == 0);
      free(out[f]);
      out[f] = nullptr, out_len[f] = 0;
      if (same && !(attempt == 0 && force_verify)) {
        out[f] = comp[j], out_len[f] = clen[j], comp[j] = nullptr;
        status[f] = AVR_OK;
      } else if (attempt == 0) {
        again.push_back(f);
      } else {
        status[f] = cst[j] != AVR_OK ? cst[j] : AVR_ERR_ROUNDTRIP;
      }
    }
    free_all();
    open.swap(again);
  }
  if (times) times[0] = tc, times[1] = td;
  for (int f = 0; f < nf; f++)
    if (status[f] != AVR_OK) fail(c, status[f], "file " + std::to_string(f) + ": compress-decompress roundtrip failed");
  return AVR_OK;
}
int avr_roundtrip_files(avr_ctx* c, int n_files, const uint8_t* const* in, const size_t* in_len, int model,
                        uint8_t** out, size_t* out_len, int32_t* status, double* times) {
  if (!c || n_files < 0 || (n_files && (!in || !in_len || !out || !out_len || !status)) || !valid_model(model))
    return AVR_ERR_INVALID_ARGUMENT;
  for (int f = 0; f < n_files; f++)
    if (!in[f]) return AVR_ERR_INVALID_ARGUMENT;
  const int r = guarded(c, [&] { return roundtrip_files(c, n_files, in, in_len, model, out, out_len, status, times); });
  if (r != AVR_OK) {
    // a batch that failed as a whole leaves no partial outputs: every file gets the error
    for (int f = 0; f < n_files; f++) {
      free(out[f]);
      out[f] = nullptr;
      out_len[f] = 0;
      status[f] = r;
    }
  }
  return r;
}

static int batch(avr_ctx* c, int mode, const avr_slice_desc* d_desc, int n, int max_w, int max_h,
                 const uint8_t* d_in, uint8_t* d_out, avr_slice_result* d_res, int model, void* stream) {
  if (!c || n < 0 || (n && (!d_desc || !d_in || !d_out || !d_res)) || max_w <= 0 || max_h <= 0 || !valid_model(model) ||
      model == AVR_MODEL_CHAINED)   // a slice batch has no file to chain over: whole-file calls only
    return AVR_ERR_INVALID_ARGUMENT;
  if (avr::shared_bytes(max_w) > 160 * 1024) return fail(c, AVR_ERR_UNSUPPORTED, "picture too wide for the LDS ring");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  if (model == AVR_MODEL_REFERENCE) {
    HIP_TRY(c, c->est.reserve(sizeof(uint16_t) * avr::kEstGlobal, true));
    HIP_TRY(c, c->frames.reserve((size_t)2 * max_w * max_h * 52 + 64));
    HIP_TRY(c, c->frame_meta.reserve(64));
    HIP_TRY(c, avr::launch_slices(mode, true, c->tables.as<avr::EngineTables>(), d_desc, n, max_w, d_in, d_out, d_res,
                                  c->est.as<uint16_t>(), c->frames.as<uint8_t>(), c->frame_meta.as<int>(), nullptr, s,
                                  avr::SeqFiles(), avr::kFlagFields));
    return AVR_OK;
  }
  HIP_TRY(c, reserve_parallel(c, n, max_w));
  HIP_TRY(c, avr::launch_slices(mode, false, c->tables.as<avr::EngineTables>(), d_desc, n, max_w, d_in, d_out, d_res,
                                c->est.as<uint16_t>(), nullptr, nullptr, c->order_or_null(), s, avr::SeqFiles(),
                                avr::kFlagFields | coder_flag(model), c->queue.p));
  return AVR_OK;
}

int avr_compress_slices(avr_ctx* c, const avr_slice_desc* d_desc, int n, int max_mb_width, int max_mb_height,
                        const uint8_t* d_in, uint8_t* d_out, avr_slice_result* d_res, int model, void* stream) {
  return batch(c, 0, d_desc, n, max_mb_width, max_mb_height, d_in, d_out, d_res, model, stream);
}

int avr_decompress_slices(avr_ctx* c, const avr_slice_desc* d_desc, int n, int max_mb_width, int max_mb_height,
                          const uint8_t* d_in, uint8_t* d_out, avr_slice_result* d_res, int model, void* stream) {
  return batch(c, 1, d_desc, n, max_mb_width, max_mb_height, d_in, d_out, d_res, model, stream);
}

int avr_roundtrip_slices(avr_ctx* c, const avr_slice_desc* d_desc, int n, int max_w, int max_h, const uint8_t* d_in,
                         uint8_t* d_work, uint8_t* d_regen, avr_slice_desc* d_dec_desc, avr_slice_result* d_res_c,
                         avr_slice_result* d_res_d, int32_t* d_verdict, int model, void* stream) {
  if (!c || n < 0 || (n && (!d_regen || !d_dec_desc || !d_res_d || !d_verdict))) return AVR_ERR_INVALID_ARGUMENT;
  if (int r = batch(c, 0, d_desc, n, max_w, max_h, d_in, d_work, d_res_c, model, stream)) return r;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(c, avr::launch_derive_decompress(d_desc, d_res_c, n, d_dec_desc, s));
  if (int r = batch(c, 1, d_dec_desc, n, max_w, max_h, d_work, d_regen, d_res_d, model, stream)) return r;
  HIP_TRY(c, avr::launch_verify(d_desc, d_res_c, d_res_d, n, d_in, d_regen, d_verdict, s));
  return AVR_OK;
}

int avr_derive_decompress_descs(avr_ctx* c, const avr_slice_desc* d_desc, const avr_slice_result* d_res_c, int n,
                                avr_slice_desc* d_dec_desc, void* stream) {
  if (!c || n < 0 || (n && (!d_desc || !d_res_c || !d_dec_desc))) return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, avr::launch_derive_decompress(d_desc, d_res_c, n, d_dec_desc, (hipStream_t)stream));
  return AVR_OK;
}

int avr_verify_slices(avr_ctx* c, const avr_slice_desc* d_desc, const avr_slice_result* d_res_c,
                      const avr_slice_result* d_res_d, int n, const uint8_t* d_in, const uint8_t* d_regen,
                      int32_t* d_verdict, void* stream) {
  if (!c || n < 0 || (n && (!d_desc || !d_res_c || !d_res_d || !d_in || !d_regen || !d_verdict)))
    return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, avr::launch_verify(d_desc, d_res_c, d_res_d, n, d_in, d_regen, d_verdict, (hipStream_t)stream));
  return AVR_OK;
}

int avr_compress_chain_range(avr_ctx* c, const uint8_t* file, size_t n, int world, int rank, int* lo, int* hi,
                             int32_t** status, uint8_t** recoded, size_t* recoded_len, uint64_t** offsets,
                             uint32_t** lens) {
  if (!c || !file || world < 1 || rank < 0 || rank >= world || !lo || !hi || !status || !recoded || !recoded_len ||
      !offsets || !lens)
    return AVR_ERR_INVALID_ARGUMENT;
  *status = nullptr, *recoded = nullptr, *offsets = nullptr, *lens = nullptr;
  return guarded(c, [&]() -> int {
    ChainRangeOut o;
    if (int r = compress_chain_range(c, file, n, world, rank, &o)) return r;
    return export_range(o, lo, hi, status, recoded, recoded_len, offsets, lens);
  });
}

int avr_decompress_chain_range(avr_ctx* c, const uint8_t* avrc, size_t n, int world, int rank, int* lo, int* hi,
                               int32_t** status, uint8_t** regen, size_t* regen_len, uint64_t** offsets,
                               uint32_t** lens) {
  if (!c || !avrc || world < 1 || rank < 0 || rank >= world || !lo || !hi || !status || !regen || !regen_len ||
      !offsets || !lens)
    return AVR_ERR_INVALID_ARGUMENT;
  *status = nullptr, *regen = nullptr, *offsets = nullptr, *lens = nullptr;
  return guarded(c, [&]() -> int {
    ChainRangeOut o;
    if (int r = decompress_chain_range(c, avrc, n, world, rank, &o)) return r;
    return export_range(o, lo, hi, status, regen, regen_len, offsets, lens);
  });
}

int avr_slice_kernel(avr_ctx* c, int decompress, int n, int max_mb_width, int* kind) {
  if (!c || !kind || n < 0 || max_mb_width <= 0) return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  *kind = avr::parallel_kernel_kind(decompress ? 1 : 0, n, max_mb_width);
  return AVR_OK;
}

int avr_parse_stream_range(const uint8_t* file, size_t n, int lo, int hi, avr_slice_desc** descs, int* n_slices,
                           uint8_t** arena, size_t* arena_len, size_t* work_len, int* max_w, int* max_h) {
  if (!file || !descs || !n_slices || !arena || !arena_len || !work_len || !max_w || !max_h || lo < 0)
    return AVR_ERR_INVALID_ARGUMENT;
  *descs = nullptr;
  *arena = nullptr;
  return guarded(nullptr, [&]() -> int {
    ParsedFile pf;
    if (int r = parse_file(nullptr, file, n, &pf, /*views=*/true)) return r;
    const int total = (int)pf.slices.size();
    const int b = std::min(lo, total), e = hi < 0 ? total : std::max(b, std::min(hi, total));
    // the arena's layout first (append_aligned's: 16-byte aligned payloads, each followed by >= 16
    // zero bytes), then one allocation and the payload copies on host threads
    const size_t ns = (size_t)(e - b);
    std::vector<avr_slice_desc> dv(ns);
    std::vector<avr::PbCopy> copies(ns);
    uint64_t work = 0, at = 0;
    int mw = 1, mh = 1;
    for (size_t i = 0; i < ns; i++) {
      const avr::SliceInfo& s = pf.slices[b + i];
      avr_slice_desc& d = dv[i];
      d = desc_from_header(s);
      d.payload_offset = (at + 15) & ~(uint64_t)15;
      at = d.payload_offset + s.read_limit + 16;
      copies[i] = {(size_t)d.payload_offset, s.payload(), s.read_limit};
      d.payload_size = (uint32_t)s.size;
      d.read_limit = (uint32_t)s.read_limit;
      d.coded = recodable_candidate(s);
      d.file_offset = s.file_payload_offset();
      d.out_offset = work;
      d.out_capacity = (uint32_t)(s.size * 2 + 256);
      work += ((uint64_t)d.out_capacity + 15) & ~15ull;
      if (d.coded) mw = std::max(mw, ring_cols(d));   // uncoded slices are never walked
      mh = std::max(mh, d.mb_height);
    }
    const size_t alen = at + 16;
    const size_t dn = sizeof(avr_slice_desc) * ns;
    *descs = (avr_slice_desc*)malloc(dn ? dn : 1);
    *arena = host_alloc(alen);
    if (!*descs || !*arena) {
      free(*descs);
      free(*arena);
      *descs = nullptr;
      *arena = nullptr;
      return AVR_ERR_OUT_OF_MEMORY;
    }
    if (dn) memcpy(*descs, dv.data(), dn);
    parallel_copies(copies, *arena);
    // the zero bytes between and after the payloads
    uint64_t z = 0;
    for (const auto& cp : copies) {
      memset(*arena + z, 0, cp.dst - z);
      z = cp.dst + cp.len;
    }
    memset(*arena + z, 0, alen - z);
    *n_slices = (int)ns;
    *arena_len = alen;
    *work_len = work;
    *max_w = mw;
    *max_h = mh;
    return AVR_OK;
  });
}

int avr_parse_stream(const uint8_t* file, size_t n, avr_slice_desc** descs, int* n_slices, uint8_t** arena,
                     size_t* arena_len, size_t* work_len, int* max_w, int* max_h) {
  return avr_parse_stream_range(file, n, 0, -1, descs, n_slices, arena, arena_len, work_len, max_w, max_h);
}

int avr_slice_payload_sizes(const uint8_t* file, size_t n, uint32_t** sizes, int* n_slices) {
  if (!file || !sizes || !n_slices) return AVR_ERR_INVALID_ARGUMENT;
  *sizes = nullptr;
  return guarded(nullptr, [&]() -> int {
    ParsedFile pf;
    if (int r = parse_file(nullptr, file, n, &pf, /*views=*/true)) return r;
    *sizes = (uint32_t*)malloc(sizeof(uint32_t) * std::max<size_t>(1, pf.slices.size()));
    if (!*sizes) return AVR_ERR_OUT_OF_MEMORY;
    for (size_t i = 0; i < pf.slices.size(); i++) (*sizes)[i] = (uint32_t)pf.slices[i].size;
    *n_slices = (int)pf.slices.size();
    return AVR_OK;
  });
}

int avr_pack_outputs(avr_ctx* c, const avr_slice_desc* d_desc, const avr_slice_result* d_res, int n,
                     const uint8_t* d_out, uint8_t* d_packed, uint64_t* d_offsets, void* stream) {
  if (!c || n < 0 || (n && (!d_desc || !d_res || !d_out || !d_packed || !d_offsets))) return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, avr::launch_pack(d_desc, d_res, n, d_out, d_packed, d_offsets, (hipStream_t)stream));
  return AVR_OK;
}

int avr_container_describe(const uint8_t* in, size_t n, char** json, uint8_t** reserialized, size_t* len) {
  if (!in || !json || !reserialized || !len) return AVR_ERR_INVALID_ARGUMENT;
  *json = nullptr;
  *reserialized = nullptr;
  std::vector<avr::PbBlock> blocks;
  std::string version;
  bool has_md = false;
  if (!avr::pb_parse(in, n, &blocks, &version, &has_md)) return AVR_ERR_FORMAT;
  static const char* hexd = "0123456789abcdef";
  auto hex = [&](const uint8_t* p, size_t k) {
    std::string h;
    h.reserve(2 * k);
    for (size_t i = 0; i < k; i++) h += hexd[p[i] >> 4], h += hexd[p[i] & 15];
    return h;
  };
  std::string j = "{\"version\": ";
  j += has_md ? "\"" + hex((const uint8_t*)version.data(), version.size()) + "\"" : std::string("null");
  j += ", \"blocks\": [";
  std::vector<uint8_t> o;
  if (has_md) avr::pb_put_metadata_version(&o, version);
  for (size_t i = 0; i < blocks.size(); i++) {
    const avr::PbBlock& b = blocks[i];
    std::string e;
    auto add = [&](const std::string& kv) { e += (e.empty() ? "" : ", ") + kv; };
    if (b.has_size) add("\"size\": " + std::to_string(b.size));
    if (b.has_literal) add("\"literal\": \"" + hex(b.literal, b.literal_len) + "\"");
    if (b.has_skip) add(std::string("\"skip_coded\": ") + (b.skip_coded ? "true" : "false"));
    if (b.has_cabac) add("\"cabac\": \"" + hex(b.cabac, b.cabac_len) + "\"");
    if (b.has_parity) add(std::string("\"length_parity\": ") + (b.length_parity ? "true" : "false"));
    if (b.has_last_byte) add("\"last_byte\": \"" + hex((const uint8_t*)b.last_byte.data(), b.last_byte.size()) + "\"");
    if (b.has_seams) add("\"seams\": \"" + hex(b.seams, b.seams_len) + "\"");
    j += (i ? ", {" : "{") + e + "}";
    avr::pb_put_block(&o, b);
  }
  j += "]}";
  *json = (char*)malloc(j.size() + 1);
  *reserialized = (uint8_t*)malloc(o.size() ? o.size() : 1);
  if (!*json || !*reserialized) {
    free(*json);
    free(*reserialized);
    *json = nullptr;
    *reserialized = nullptr;
    return AVR_ERR_OUT_OF_MEMORY;
  }
  memcpy(*json, j.c_str(), j.size() + 1);
  if (!o.empty()) memcpy(*reserialized, o.data(), o.size());
  *len = o.size();
  return AVR_OK;
}

static int synthesize_stream(avr_ctx* c, const avr_synth_params* p, int n, uint8_t** out, size_t* out_len);
int avr_synthesize_stream(avr_ctx* c, const avr_synth_params* p, int n, uint8_t** out, size_t* out_len) {
  return guarded(c, [&] { return synthesize_stream(c, p, n, out, out_len); });
}
static int synthesize_stream(avr_ctx* c, const avr_synth_params* p, int n, uint8_t** out, size_t* out_len) {
  if (!c || !p || n <= 0 || !out || !out_len || p->mb_width <= 0 || p->mb_height <= 0 || p->slice_type < 0 ||
      p->slice_type > 2 || p->chroma_format_idc < 1 || p->chroma_format_idc > 3 || p->gop_length < 0 ||
      p->repeat < 0 || p->structure < 0 || p->structure > 3 || (p->structure && (p->mb_height & 1)))
    return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  Plan plan;
  // a coded picture: the frame, or (field pictures) each of its two fields in turn, the top
  // field first (structure 1) or the bottom field first (3)
  const bool paff = p->structure == 1 || p->structure == 3;
  const int fields = paff ? 2 : 1;
  const int mbs = p->mb_width * p->mb_height / fields;
  // MBAFF slices start on a macroblock pair
  const int unit = p->structure == 2 ? 2 : 1;
  const int spp = std::max(1, std::min(p->slices_per_picture, mbs / unit));
  std::vector<int> pic_of, first_of;
  for (int i = 0; i < n * fields * spp; i++) {
    const int pic = i / (spp * fields), fi = (i / spp) % fields, j = i % spp;
    const int first = unit * (int)((int64_t)j * (mbs / unit) / spp);
    const int next = unit * (int)((int64_t)(j + 1) * (mbs / unit) / spp);
    pic_of.push_back(pic);
    first_of.push_back(first);
    avr_slice_desc d;
    memset(&d, 0, sizeof(d));
    // GOP: an IDR I picture every gop_length pictures; with slice_type B the pictures between
    // follow B B P B B P ... (decode order), with P every picture between
    const int g = p->gop_length > 0 ? pic % p->gop_length : -1;
    const int st = g == 0 ? 2 : (g > 0 && p->slice_type == 1 && g % 3 == 0) ? 0 : p->slice_type;
    d.slice_type = st;
    d.slice_qp = p->slice_qp;
    d.cabac_init_idc = st == 2 ? -1 : 0;
    d.mb_width = p->mb_width;
    d.mb_height = p->mb_height;
    d.num_ref_idx_l0 = st == 2 ? 0 : std::max(1, p->num_ref_idx_l0);
    d.num_ref_idx_l1 = st == 1 ? std::max(1, p->num_ref_idx_l1) : 0;
    d.chroma_array_type = p->chroma_format_idc;
    d.transform_8x8_mode = p->transform_8x8_mode;
    d.direct_8x8_inference = 1;
    d.x264_build = -1;
    d.picture_id = pic;
    d.first_mb = first;
    d.coded = 1;
    d.structure = paff ? ((fi ^ (p->structure == 3)) ? AVR_STRUCT_BOTTOM_FIELD : AVR_STRUCT_TOP_FIELD)
                : p->structure == 2 ? AVR_STRUCT_MBAFF : AVR_STRUCT_FRAME;
    d.payload_offset = p->seed * 0x100000001B3ull + (uint64_t)i;  // generator seed
    d.payload_size = (uint32_t)(next - first);                    // generator: macroblocks to emit
    d.out_capacity = (uint32_t)std::min<uint64_t>((uint64_t)mbs * 384 + 4096, 0x7fffffffu);
    plan.descs.push_back(d);
  }
  plan.max_w = p->structure == 2 ? 3 * p->mb_width + 7 : p->mb_width;
  plan.arena.assign(16, 0);
  std::vector<avr_slice_result> res;
  std::vector<uint8_t> outb;
  if (int r = run_plan(c, 2, false, plan, &res, &outb)) return r;
  std::vector<uint8_t> stream;
  avr::synth_write_parameter_sets(&stream, *p);
  for (int i = 0; i < (int)plan.descs.size(); i++)
    if (res[i].status != 0) return fail(c, AVR_ERR_DEVICE, "generator failed on slice " + std::to_string(i));
  const int reps = std::max(1, p->repeat);
  // the tiled stream goes straight into the caller's buffer (one copy of it in host memory): each
  // NAL unit is written to a scratch vector and appended; 64 B per slice bound its header and
  // start code (checked at every append)
  size_t bytes = 0;
  for (int i = 0; i < (int)plan.descs.size(); i++) bytes += res[i].out_len + 64;
  if ((uint64_t)bytes * reps > kMaxSynthBytes) return fail(c, AVR_ERR_INVALID_ARGUMENT, "stream too large");
  const size_t cap = stream.size() + bytes * reps;
  uint8_t* o = (uint8_t*)malloc(cap);
  if (!o) return fail(c, AVR_ERR_OUT_OF_MEMORY, "synthetic stream: host allocation failed");
  memcpy(o, stream.data(), stream.size());
  size_t at = stream.size();
  std::vector<uint8_t> nal;
  for (int t = 0; t < reps; t++)
    for (int i = 0; i < (int)plan.descs.size(); i++) {
      nal.clear();
      avr::synth_write_slice(&nal, *p, plan.descs[i].slice_type, t * n + pic_of[i], plan.descs[i].structure,
                             paff && (i / spp) % 2 == 1, first_of[i], outb.data() + plan.descs[i].out_offset,
                             res[i].out_len);
      if (at + nal.size() > cap) {
        free(o);
        return fail(c, AVR_ERR_DEVICE, "synthetic stream: slice header larger than its bound");
      }
      memcpy(o + at, nal.data(), nal.size());
      at += nal.size();
    }
  *out = o;
  *out_len = at;
  return AVR_OK;
}

}  // extern "C"

// Debug only (not part of include/avrecode.h): section cycle counters (32 slots) of an AVR_PROFILE build of
// the slice kernels (mode 0 compress, 1 decompress, 2 generate, 3/4 sequential compress/decompress), read and cleared.
// Diagnostic (AVR_PROFILE builds): 8 u32 per slice of the last parallel compress (mode 0) or
// decompress (1) launch: HW_ID of waves 0-2, XCC_ID, walker start/end cycle counters.
extern "C" int avr_debug_placement(int mode, uint32_t* out8n, int n) {
  hipError_t e = mode == 0 ? avr::placement_parallel_compress(out8n, n) : avr::placement_parallel_decompress(out8n, n);
  return e == hipSuccess ? AVR_OK : AVR_ERR_DEVICE;
}

extern "C" int avr_debug_profile(int mode, unsigned long long* out16) {
  hipError_t e = mode == 0 ? avr::profile_parallel_compress(out16)
               : mode == 1 ? avr::profile_parallel_decompress(out16)
               : mode == 3 ? avr::profile_sequential_compress(out16)
               : mode == 4 ? avr::profile_sequential_decompress(out16)
                           : avr::profile_parallel_generate(out16);
  return e == hipSuccess ? AVR_OK : AVR_ERR_DEVICE;
}

// ==================================================================== libavcodec-hooks surface
// The reference's hook objects (compressor::cabac_decoder recode.cpp:1134-1268,
// decompressor::cabac_decoder 1411-1520) answer each bin request by running the model inline.
// Here the device has already done the whole file; the session replays the device's decode-order
// bin trace (MODE_TRACE kernel) to the caller and cross-checks the caller's parse against it.
struct avr_hooks_session;

// A significance map of the device's parse (MODE_TRACE event records): the bins [begin, end) it
// spans and the model state it starts under -- mb_xy and begin_sub_mb's arguments.
struct HookMap {
  uint32_t begin = 0, end = 0;
  int x = 0, y = 0;
  int sub[5] = {0, 0, 0, 0, 0};   // cat, scan8 index, max_coeff, is_dc, chroma422
};

struct avr_hooks_slice {
  avr_hooks_session* sess = nullptr;
  int index = 0;                 // slice index (decode order)
  const uint8_t* trace = nullptr;   // 2 bytes per bin: bin | kind << 1, state byte before it
  size_t nbins = 0, cur = 0;
  const HookMap* maps = nullptr;
  size_t nmaps = 0, map_cur = 0;
  bool sub_open = false;
  int sub_args[5] = {0, 0, 0, 0, 0};
  int coding_type = 0;
};

// Streaming compress session: incremental demux + parse of the bytes fed so far.  Only what is new
// is parsed: an Annex-B NAL unit once the next start code (00 00 00 / 00 00 01, demux_annexb's rule)
// has been fed -- the unit in progress provisionally when a decoder already asks for its slice (a
// later feed that extends it fails the session) -- and an MP4 sample once the moov box and the
// whole sample are in.  Slices come out in decode order exactly as parse_file gives them.
struct StreamIngest {
  avr::StreamParser sp;
  int kind = 0;                 // 0 undecided (< 8 bytes), 1 Annex-B, 2 MP4
  // Annex-B
  size_t scan = 0;              // where the search for the next boundary / start code resumes
  bool in_nal = false;          // a NAL unit started at nal_begin (after its start code)
  size_t nal_begin = 0;
  size_t prov_end = 0;          // the unit in progress was parsed provisionally through here (0: not)
  // MP4
  bool have_layout = false;
  avr::Mp4Layout layout;
  size_t next_sample = 0;
};

struct avr_hooks_session {
  avr_ctx* c = nullptr;
  bool decompress = false;
  std::vector<uint8_t> original;   // the H.264 file
  std::vector<uint8_t> result;     // compress: the container; decompress: the original file
  std::vector<uint8_t> stream;     // decompress: read_packet's stream
  ParsedFile pf;
  std::vector<char> coded;
  std::vector<std::vector<uint8_t>> bins;   // per slice: the device's bins (2 bytes each)
  std::vector<std::vector<HookMap>> maps;    // per slice: its significance maps
  std::vector<avr_hooks_slice> slices;
  size_t next_slice = 0;
  uint64_t next_marker = 1;
  avr_hooks_slice* live = nullptr;  // the slice model hooks refer to (one live CABAC context, recode.cpp:199)
  uint64_t mb_calls = 0;
  int mb_x = -1, mb_y = -1;         // the caller's last mb_xy (h264_model::mb_coord)
  // frame_spec (update_frame_spec, recode.cpp:824-843): the caller's last call and the slice it
  // belonged to; a call made between slices waits for the next init_decoder
  bool fs_have = false, fs_pending = false;
  int fs_num = 0, fs_w = 0, fs_h = 0, fs_slice = -1;
  int pend_num = 0, pend_w = 0, pend_h = 0;
  // streaming compress (avr_hooks_compress_stream_begin): `original` grows by avr_hooks_feed; pf holds
  // the slices parsed from it so far (ing: incremental), traced[i] = slice i's device work is done --
  // its bin trace and, for the parallel model, its final re-coded block (blocks / block_status: the
  // container is assembled from them at avr_hooks_end without another device pass)
  bool streaming = false;
  StreamIngest ing;
  std::vector<char> traced;
  std::vector<std::vector<uint8_t>> blocks;
  std::vector<int32_t> block_status;
  int model = 0;
  // decompress of a parallel-model container, on demand: the container's plan (every coded slice's
  // re-coded block) is made at begin, and a slice is regenerated on the device -- with the coded
  // slices after it that are not yet, up to kLazyBatch -- when init_decoder reaches it; its bins
  // are traced from the regenerated payload (recode.cpp:1435-1449 decodes each bin as FFmpeg asks)
  bool lazy = false;
  DecJob job;
  Plan dplan;
  std::vector<int> plan_of;          // per slice: its dplan index (-1: not coded)
  std::vector<int> block_of;         // per slice: its container block
  std::vector<char> regen_done;
  std::vector<std::vector<uint8_t>> regen;   // per slice: its regenerated payload (last-byte patched)
  std::string err;
  void fail_once(const std::string& m) {
    if (err.empty()) err = m;
  }
};

namespace {

// FFmpeg's state transition for one decoded bin (ff_h264_mlps_state, cabac_code.h:46-48)
uint8_t next_state(uint8_t s, int bin) {
  const int p = s >> 1, mps = s & 1;
  if (bin == mps) return (uint8_t)(2 * (p < 62 ? p + 1 : p) + mps);
  return (uint8_t)(p == 0 ? (s ^ 1) : 2 * avr::kTransIdxLPS[p] + mps);
}

// Device trace (MODE_TRACE kernel) of the slices `which` of hs->pf into hs->bins / hs->maps.
int trace_slices(avr_hooks_session* hs, const std::vector<int>& which) {
  avr_ctx* c = hs->c;
  Plan plan;
  std::vector<int> slice_of;
  for (const int i : which) {
    const avr::SliceInfo& s = hs->pf.slices[i];
    avr_slice_desc d = desc_from_header(s);
    append_aligned(&plan.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
    d.payload_size = (uint32_t)s.size;
    d.read_limit = (uint32_t)s.read_limit;
    // 2 bytes per bin (H.264 bounds a slice's bins by ~32/3 per payload byte plus a per-macroblock
    // allowance, 7.4.2.2) and 12 bytes of map events per residual block (<= 51 per macroblock)
    d.out_capacity = (uint32_t)std::min<uint64_t>(
        0xfffffff0ull, 32ull * s.size + 1280ull * d.mb_width * d.mb_height + 8192);
    plan.max_w = std::max(plan.max_w, ring_cols(d));
    slice_of.push_back(i);
    plan.descs.push_back(d);
  }
  if (plan.descs.empty()) return AVR_OK;
  std::vector<avr_slice_result> res;
  std::vector<uint8_t> traces;
  if (int r = run_plan(c, 3, false, plan, &res, &traces)) return r;
  for (size_t k = 0; k < plan.descs.size(); k++) {
    const int i = slice_of[k];
    if (res[k].status != 0)
      return fail(c, AVR_ERR_FORMAT, "hooks: device trace of slice " + std::to_string(i) + " failed (" +
                                         std::to_string(res[k].status) + ")");
    // split the records: bins (kinds 0-2) and map events (kind 3, avr_walker.h TRACE_EV_*)
    const uint8_t* t = traces.data() + plan.descs[k].out_offset;
    const size_t len = res[k].out_len;
    std::vector<uint8_t>& b = hs->bins[i];
    std::vector<HookMap>& m = hs->maps[i];
    b.clear();
    m.clear();
    b.reserve(len);
    bool open = false;
    for (size_t at = 0; at + 2 <= len;) {
      if (((t[at] >> 1) & 3) != 3) {
        b.push_back(t[at]);
        b.push_back(t[at + 1]);
        at += 2;
        continue;
      }
      const uint32_t bin_index = (uint32_t)(b.size() / 2);
      if (t[at + 1] == 1 && at + 10 <= len && !open) {
        HookMap h;
        h.begin = bin_index;
        h.x = t[at + 2] | t[at + 3] << 8;
        h.y = t[at + 4] | t[at + 5] << 8;
        h.sub[0] = t[at + 6], h.sub[1] = t[at + 7], h.sub[2] = t[at + 8];
        h.sub[3] = t[at + 9] & 1, h.sub[4] = t[at + 9] >> 1;
        m.push_back(h);
        open = true;
        at += 10;
      } else if (t[at + 1] == 2 && open) {
        m.back().end = bin_index;
        open = false;
        at += 2;
      } else {
        return fail(c, AVR_ERR_DEVICE, "hooks: malformed device trace of slice " + std::to_string(i));
      }
    }
    if (open) return fail(c, AVR_ERR_DEVICE, "hooks: device trace of slice " + std::to_string(i) + " ends in a map");
  }
  return AVR_OK;
}

// Device trace of every coded slice of hs->pf (decode order).
int run_traces(avr_hooks_session* hs) {
  std::vector<int> which;
  for (size_t i = 0; i < hs->pf.slices.size(); i++)
    if (hs->coded[i]) which.push_back((int)i);
  hs->bins.assign(hs->pf.slices.size(), {});
  hs->maps.assign(hs->pf.slices.size(), {});
  return trace_slices(hs, which);
}

// Streaming session: one NAL unit of the fed bytes through the stream parser (a slice joins pf).
void ingest_nal(avr_hooks_session* hs, size_t off, size_t size) {
  avr::SliceInfo si;
  if (!hs->ing.sp.next(hs->original.data() + off, size, &si)) return;
  si.nal_offset = off;
  si.nal_size = size;
  hs->pf.slices.push_back(std::move(si));
}

// Parse what the fed bytes newly complete.  final: the stream has ended (avr_hooks_end: the unit in
// progress ends with it).  want: the number of slices a decoder needs now -- when the complete units
// do not reach it, the Annex-B unit in progress is taken provisionally.
int ingest(avr_hooks_session* hs, bool final, size_t want) {
  StreamIngest& g = hs->ing;
  const uint8_t* f = hs->original.data();
  const size_t n = hs->original.size();
  if (!g.kind) {
    if (n < 8 && !final) return AVR_OK;
    g.kind = avr::is_mp4(f, n) ? 2 : 1;
  }
  if (g.kind == 2) {
    if (!g.have_layout) {
      const int r = avr::mp4_layout(f, n, &g.layout);
      if (r < 0 || (r == 0 && final)) return fail(hs->c, AVR_ERR_FORMAT, "hooks: not an MP4/avcC H.264 stream");
      if (r == 0) return AVR_OK;   // the moov box is not in yet (a moov-last file: not before the end)
      g.have_layout = true;
      for (const avr::NalRef& nr : g.layout.param_sets) ingest_nal(hs, nr.offset, nr.size);
    }
    std::vector<avr::NalRef> nals;
    for (; g.next_sample < g.layout.samples.size(); g.next_sample++) {
      const avr::NalRef& smp = g.layout.samples[g.next_sample];
      if (smp.offset > n || smp.size > n - smp.offset) {
        if (final) return fail(hs->c, AVR_ERR_FORMAT, "hooks: an MP4 sample lies past the end of the stream");
        break;   // not complete yet
      }
      nals.clear();
      avr::mp4_sample_nals(f, smp, g.layout.len_size, &nals);
      for (const avr::NalRef& nr : nals) ingest_nal(hs, nr.offset, nr.size);
    }
    return AVR_OK;
  }
  // Annex-B (demux_annexb's rules, resumed where the last call stopped)
  auto is_sc = [&](size_t j) { return j + 3 <= n && f[j] == 0 && f[j + 1] == 0 && f[j + 2] == 1; };
  auto unit_end = [&](size_t begin, size_t end) {   // trailing zero bytes belong to the next start code
    while (end > begin && f[end - 1] == 0) end--;
    return end;
  };
  for (;;) {
    if (!g.in_nal) {
      size_t i = g.scan;
      while (i + 3 <= n && !is_sc(i)) i++;
      if (i + 3 > n) {
        g.scan = i;
        break;
      }
      g.in_nal = true;
      g.nal_begin = g.scan = i + 3;
    }
    size_t j = g.scan;
    while (j + 3 <= n && !(f[j] == 0 && f[j + 1] == 0 && (f[j + 2] == 1 || f[j + 2] == 0))) j++;
    if (j + 3 > n) {
      g.scan = j;
      break;
    }
    // the unit in progress is complete: [nal_begin, j) without trailing zeros
    const size_t end = unit_end(g.nal_begin, j);
    if (g.prov_end) {
      if (end != g.prov_end)
        return fail(hs->c, AVR_ERR_FORMAT, "hooks: a slice was decoded before its NAL unit was complete");
      g.prov_end = 0;
    } else if (end > g.nal_begin) {
      ingest_nal(hs, g.nal_begin, end - g.nal_begin);
    }
    g.in_nal = false;
    g.scan = j;
  }
  // the unit in progress: at the end of the stream it is complete; before it, it is parsed
  // provisionally when the decoder needs a slice the complete units do not hold
  if (g.in_nal && (final || hs->pf.slices.size() < want)) {
    const size_t end = unit_end(g.nal_begin, n);
    if (g.prov_end && end != g.prov_end)
      return fail(hs->c, AVR_ERR_FORMAT, "hooks: a slice was decoded before its NAL unit was complete");
    if (!g.prov_end && end > g.nal_begin) {
      ingest_nal(hs, g.nal_begin, end - g.nal_begin);
      g.prov_end = end;
    }
    if (final) g.in_nal = false, g.prov_end = 0;
  }
  return AVR_OK;
}

// Per-slice state for the slices parsed so far.
void grow_session(avr_hooks_session* hs) {
  const size_t n = hs->pf.slices.size();
  hs->coded.resize(n, 0);
  hs->bins.resize(n);
  hs->maps.resize(n);
  hs->slices.resize(n);   // no slice object is live here (init_decoder closed it first)
  hs->traced.resize(n, 0);
  hs->blocks.resize(n);
  hs->block_status.resize(n, AVR_SLICE_NO_ROUNDTRIP);
}

// Streaming session: the device work of slice i and of every parsed slice after it not done yet
// (trace-ahead: the slices a feed completed go to the device together) -- their decode-order bin
// traces, and for the parallel model their final re-coded blocks (compress + the per-slice device
// roundtrip check, as avr_compress_file runs it).
int stream_device_work(avr_hooks_session* hs, size_t i) {
  std::vector<int> which;
  for (size_t k = i; k < hs->pf.slices.size(); k++)
    if (!hs->traced[k]) {
      hs->traced[k] = 1;
      if (recodable_candidate(hs->pf.slices[k])) which.push_back((int)k);
    }
  if (which.empty()) return AVR_OK;
  if (int r = trace_slices(hs, which)) return r;
  if (!parallel_model(hs->model)) return AVR_OK;
  Plan plan;
  for (const int k : which) {
    const avr::SliceInfo& s = hs->pf.slices[k];
    avr_slice_desc d = desc_from_header(s);
    append_aligned(&plan.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
    d.payload_size = (uint32_t)s.size;
    d.read_limit = (uint32_t)s.read_limit;
    d.out_capacity = (uint32_t)(s.size * 2 + 256);
    plan.max_w = std::max(plan.max_w, ring_cols(d));
    plan.descs.push_back(d);
  }
  std::vector<avr_slice_result> res;
  std::vector<uint8_t> outb;
  if (int r = run_plan(hs->c, 0, false, plan, &res, &outb, /*verify=*/true, coder_flag(hs->model))) return r;
  for (size_t q = 0; q < which.size(); q++) {
    const int k = which[q];
    hs->block_status[k] = res[q].status;
    if (res[q].status == 0)
      hs->blocks[k].assign(outb.begin() + plan.descs[q].out_offset, outb.begin() + plan.descs[q].out_offset + res[q].out_len);
  }
  return AVR_OK;
}

// Lazy decompress session: regenerate the coded slices from i on that are not yet (at most
// kLazyBatch, one device launch), patch each by the last-byte rule (recode.cpp:1345-1356) and put
// the regenerated payload in place of the surrogate one; trace = also trace them (init_decoder).
constexpr size_t kLazyBatch = 32;
int lazy_device_work(avr_hooks_session* hs, size_t i, bool trace, size_t batch = kLazyBatch) {
  std::vector<int> which;
  for (size_t k = i; k < hs->pf.slices.size() && which.size() < batch; k++)
    if (hs->coded[k] && !hs->regen_done[k]) which.push_back((int)k);
  if (which.empty()) return AVR_OK;
  Plan sub;
  for (const int k : which) {
    avr_slice_desc d = hs->dplan.descs[hs->plan_of[k]];
    append_aligned(&sub.arena, hs->dplan.arena.data() + d.payload_offset, d.payload_size, 16, &d.payload_offset);
    sub.max_w = std::max(sub.max_w, ring_cols(d));
    sub.descs.push_back(d);
  }
  std::vector<avr_slice_result> res;
  std::vector<uint8_t> outb;
  if (int r = run_plan(hs->c, 1, false, sub, &res, &outb, false, coder_flag(hs->model))) return r;
  for (size_t q = 0; q < which.size(); q++) {
    const int k = which[q];
    if (res[q].status != 0)
      return fail(hs->c, AVR_ERR_FORMAT, "slice " + std::to_string(k) + " failed to decode (" +
                                             std::to_string(res[q].status) + ")");
    std::vector<uint8_t>& g = hs->regen[k];
    g.assign(outb.begin() + sub.descs[q].out_offset, outb.begin() + sub.descs[q].out_offset + res[q].out_len);
    const avr::PbBlock& b = hs->job.blocks[hs->block_of[k]];
    if (b.has_parity && b.has_last_byte && !b.last_byte.empty()) {   // as splice_job
      if ((int)b.length_parity != (int)(g.size() & 1)) g.push_back((uint8_t)b.last_byte[0]);
      else if (!g.empty()) g.back() = (uint8_t)b.last_byte[0];
    }
    // the regenerated payload in place of the surrogate one; the NAL's bytes after the payload
    // (from the literal that follows the block) stay, as does the parse's read limit
    avr::SliceInfo& s = hs->pf.slices[k];
    s.own();
    if (g.size() != s.size || s.rbsp.size() < s.h.cabac_start + s.size)
      return fail(hs->c, AVR_ERR_FORMAT, "slice " + std::to_string(k) + " regenerated " + std::to_string(g.size()) +
                                             " bytes for a " + std::to_string(s.size) + "-byte payload");
    std::copy(g.begin(), g.end(), s.rbsp.begin() + s.h.cabac_start);
    hs->regen_done[k] = 1;
  }
  return trace ? trace_slices(hs, which) : AVR_OK;
}

// which slices of the file a container re-codes: the i-th non-literal block is slice i's
bool coded_from_container(const std::vector<avr::PbBlock>& blocks, size_t n_slices, std::vector<char>* coded) {
  coded->assign(n_slices, 0);
  size_t i = 0;
  for (auto& b : blocks) {
    if (b.has_literal) continue;
    if (i >= n_slices) return false;
    (*coded)[i++] = b.has_cabac ? 1 : 0;
  }
  return i == n_slices;
}

// the live slice is done (the next init_decoder or avr_hooks_end): every bin and every map consumed
void close_live(avr_hooks_session* hs) {
  avr_hooks_slice* h = hs->live;
  hs->live = nullptr;
  if (!h) return;
  if (h->cur != h->nbins)
    hs->fail_once("hooks: slice " + std::to_string(h->index) + " ended after " + std::to_string(h->cur) + " of " +
                  std::to_string(h->nbins) + " bins");
  else if (h->map_cur != h->nmaps)
    hs->fail_once("hooks: slice " + std::to_string(h->index) + " reported " + std::to_string(h->map_cur) + " of its " +
                  std::to_string(h->nmaps) + " significance maps");
  else if (!hs->fs_have || hs->pf.slices[hs->fs_slice].picture_id != hs->pf.slices[h->index].picture_id)
    hs->fail_once("hooks: slice " + std::to_string(h->index) + " was decoded without a frame_spec for its picture");
}

// frame_spec of slice i: the model's frames (update_frame_spec, recode.cpp:824-843) turn over where
// the device's pictures do (its decode-order picture counter, which the two fields of a frame
// share, as they share frame_num), and the size must be the picture's.  A caller that starts a new
// frame inside one of the device's pictures is refused.  A caller whose frame_num stays the same
// while the device starts a new picture is accepted only where the two pictures' slice headers
// carry the same frame_num: the fork passes that syntax element, and consecutive pictures share it
// after a non-reference picture (e.g. B(frame_num 4, nal_ref_idc 0) then P(4)) -- the model keeps
// its per-picture frames there (frame_spec takes a picture counter).  Any other
// repeat is a caller whose frames differ from the pictures it decodes.
void check_frame_spec(avr_hooks_session* hs, int i, int frame_num, int w, int h) {
  const avr::SliceInfo& s = hs->pf.slices[i];
  const std::string where = "hooks: slice " + std::to_string(i) + ": frame_spec(" + std::to_string(frame_num) + ", " +
                            std::to_string(w) + ", " + std::to_string(h) + ")";
  if (w != s.h.mb_width || h != s.h.mb_height) {
    hs->fail_once(where + " size differs from the picture's " + std::to_string(s.h.mb_width) + " x " +
                  std::to_string(s.h.mb_height));
    return;
  }
  if (hs->fs_have) {
    const avr::SliceInfo& p = hs->pf.slices[hs->fs_slice];
    const bool caller_new = frame_num != hs->fs_num || w != hs->fs_w || h != hs->fs_h;
    const bool device_new = s.picture_id != p.picture_id || w != hs->fs_w || h != hs->fs_h;
    const bool syntax_repeat = !caller_new && device_new && s.h.frame_num == p.h.frame_num;
    if (caller_new != device_new && !syntax_repeat)
      hs->fail_once(where + (device_new ? " keeps the frame of slice " : " starts a new frame after slice ") +
                    std::to_string(hs->fs_slice) + ", the device's parse " +
                    (device_new ? "starts a new picture" : "stays in the same picture"));
  }
  hs->fs_have = true;
  hs->fs_num = frame_num, hs->fs_w = w, hs->fs_h = h, hs->fs_slice = i;
}

int hooks_finish_setup(avr_hooks_session* hs, const std::vector<avr::PbBlock>& blocks) {
  if (int r = parse_file(hs->c, hs->original.data(), hs->original.size(), &hs->pf)) return r;
  if (!coded_from_container(blocks, hs->pf.slices.size(), &hs->coded))
    return fail(hs->c, AVR_ERR_FORMAT, "hooks: container blocks do not match the file's slices");
  if (int r = run_traces(hs)) return r;
  hs->slices.resize(hs->pf.slices.size());
  return AVR_OK;
}

}  // namespace

int avr_hooks_compress_begin(avr_ctx* c, const uint8_t* file, size_t n, int model, avr_hooks_session** out) {
  if (!c || !file || !out) return AVR_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  std::unique_ptr<avr_hooks_session> hs(new avr_hooks_session);
  hs->c = c;
  hs->original.assign(file, file + n);
  uint8_t* avrc = nullptr;
  size_t avrc_len = 0;
  if (int r = avr_compress_file(c, file, n, model, &avrc, &avrc_len)) return r;
  hs->result.assign(avrc, avrc + avrc_len);
  free(avrc);
  std::vector<avr::PbBlock> blocks;
  std::string version;
  if (!avr::pb_parse(hs->result.data(), hs->result.size(), &blocks, &version))
    return fail(c, AVR_ERR_FORMAT, "hooks: container does not parse");
  if (int r = hooks_finish_setup(hs.get(), blocks)) return r;
  *out = hs.release();
  return AVR_OK;
}

int avr_hooks_decompress_begin(avr_ctx* c, const uint8_t* avrc, size_t n, avr_hooks_session** out,
                               const uint8_t** stream, size_t* stream_len) {
  if (!c || !avrc || !out) return AVR_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  std::unique_ptr<avr_hooks_session> hs(new (std::nothrow) avr_hooks_session);
  if (!hs) return fail(c, AVR_ERR_OUT_OF_MEMORY, "host allocation failed");
  hs->c = c;
  hs->decompress = true;
  {
    // the container's model from its Metadata.version alone (no block list), inside guarded(): no
    // exception crosses the C ABI
    int m = 0;
    bool split = false;   // a long-slice split container: regenerated whole at begin (its pieces are
                          // a whole-file launch), as a reference-model one is
    if (int r = guarded(c, [&]() -> int {
          std::string version;
          m = avr::pb_read_version(avrc, n, &version) ? avr::model_of_version(version) : 0;
          if (m == AVR_MODEL_PARALLEL) {
            std::vector<avr::PbBlock> blocks;
            if (avr::pb_parse(avrc, n, &blocks, &version))
              for (const auto& b : blocks) split = split || b.has_seams;
          }
          return AVR_OK;
        }))
      return r;
    if (parallel_model(m) && !split && !getenv("AVR_HOOKS_EAGER")) {
      // the parallel model's slices are independent: plan the container now, regenerate on demand
      if (int r = guarded(c, [&]() -> int {
            hs->lazy = true;
            hs->model = m;
            hs->original.assign(avrc, avrc + n);   // the container (the job's blocks point into it)
            if (int e = decompress_setup(c, hs->original.data(), hs->original.size(), &hs->job, &hs->dplan)) return e;
            hs->stream.assign(hs->job.stream.begin(), hs->job.stream.end());
            if (int e = parse_file(c, hs->stream.data(), hs->stream.size(), &hs->pf)) return e;
            if (!coded_from_container(hs->job.blocks, hs->pf.slices.size(), &hs->coded))
              return fail(c, AVR_ERR_FORMAT, "hooks: container blocks do not match the file's slices");
            const size_t ns = hs->pf.slices.size();
            hs->plan_of.assign(ns, -1);
            hs->block_of.assign(ns, -1);
            size_t i = 0;
            for (size_t bi = 0; bi < hs->job.blocks.size(); bi++) {
              if (hs->job.blocks[bi].has_literal) continue;
              hs->block_of[i] = (int)bi;
              if (hs->job.blocks[bi].has_cabac) hs->plan_of[i] = hs->job.desc_of_block[bi];
              i++;
            }
            for (size_t k = 0; k < ns; k++)
              if (hs->coded[k] && hs->plan_of[k] < 0) return fail(c, AVR_ERR_FORMAT, "hooks: a coded block has no plan slice");
            hs->regen_done.assign(ns, 0);
            hs->regen.assign(ns, {});
            hs->bins.assign(ns, {});
            hs->maps.assign(ns, {});
            hs->slices.resize(ns);
            return AVR_OK;
          }))
        return r;
      if (stream) *stream = hs->stream.data();
      if (stream_len) *stream_len = hs->stream.size();
      *out = hs.release();
      return AVR_OK;
    }
  }
  uint8_t* orig = nullptr;
  size_t orig_len = 0;
  if (int r = avr_decompress_file(c, avrc, n, &orig, &orig_len)) return r;
  hs->original.assign(orig, orig + orig_len);
  hs->result = hs->original;
  free(orig);
  std::vector<avr::PbBlock> blocks;
  std::string version;
  if (!avr::pb_parse(avrc, n, &blocks, &version)) return fail(c, AVR_ERR_FORMAT, "hooks: container does not parse");
  // read_packet (recode.cpp:1359-1409)
  uint64_t seq = 1;
  for (auto& b : blocks) {
    if (b.has_literal) {
      hs->stream.insert(hs->stream.end(), b.literal, b.literal + b.literal_len);
    } else if (b.has_cabac) {
      uint8_t mk[8];
      avr::surrogate_marker(seq++, mk);
      hs->stream.insert(hs->stream.end(), mk, mk + 8);
      hs->stream.insert(hs->stream.end(), (size_t)b.size - 8, (uint8_t)'X');
    }
  }
  if (int r = hooks_finish_setup(hs.get(), blocks)) return r;
  if (stream) *stream = hs->stream.data();
  if (stream_len) *stream_len = hs->stream.size();
  *out = hs.release();
  return AVR_OK;
}

int avr_hooks_compress_stream_begin(avr_ctx* c, int model, avr_hooks_session** out) {
  if (!c || !out) return AVR_ERR_INVALID_ARGUMENT;
  if (!valid_model(model)) return AVR_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  avr_hooks_session* hs = new (std::nothrow) avr_hooks_session;
  if (!hs) return AVR_ERR_OUT_OF_MEMORY;
  hs->c = c;
  hs->streaming = true;
  hs->model = model;
  *out = hs;
  return AVR_OK;
}

int avr_hooks_feed(avr_hooks_session* hs, const uint8_t* bytes, size_t n) {
  if (!hs || (!bytes && n) || !hs->streaming) return AVR_ERR_INVALID_ARGUMENT;
  try {
    hs->original.insert(hs->original.end(), bytes, bytes + n);
  } catch (const std::bad_alloc&) {
    return AVR_ERR_OUT_OF_MEMORY;
  }
  return AVR_OK;
}

void* avr_hook_init_decoder(void* opaque, void* /*cabac_context*/, const uint8_t* buf, int size) {
  avr_hooks_session* hs = (avr_hooks_session*)opaque;
  if (!hs) return nullptr;
  close_live(hs);
  if (hs->streaming) {
    // the slice the decoder starts is in the bytes its demuxer has read (read_packet feeds them
    // before the packet is decoded): parse what is new
    int r = guarded(hs->c, [&] {
      const int e = ingest(hs, false, hs->next_slice + 1);
      grow_session(hs);
      return e;
    });
    if (r) {
      hs->fail_once("hooks: the bytes fed so far do not parse (" + std::to_string(r) + "): " + hs->c->err);
      hs->next_slice++;
      return nullptr;
    }
  }
  if (hs->next_slice >= hs->pf.slices.size()) {
    hs->fail_once(hs->streaming ? "hooks: init_decoder for a slice not yet fed" : "hooks: more slices than the file holds");
    return nullptr;
  }
  const size_t i = hs->next_slice++;
  if (hs->fs_pending) {   // the frame_spec made before this slice's decode
    hs->fs_pending = false;
    check_frame_spec(hs, (int)i, hs->pend_num, hs->pend_w, hs->pend_h);
  }
  const avr::SliceInfo& s = hs->pf.slices[i];
  if (!buf || size < 0 || (size_t)size != s.size) {
    hs->fail_once("hooks: slice " + std::to_string(i) + " size differs from the device's parse");
    return nullptr;
  }
  if (hs->streaming) {
    // find_next_coded_block (recode.cpp:1139-1145, 1275-1297) on the slice's own bytes: a slice the
    // device can re-code gets hooks; the container (avr_hooks_end) may still store it skip_coded
    hs->coded[i] = memcmp(buf, s.payload(), s.size) == 0 && recodable_candidate(s) ? 1 : 0;
    if (hs->coded[i] && guarded(hs->c, [&] { return stream_device_work(hs, i); }) != AVR_OK) {
      hs->fail_once("hooks: device trace of slice " + std::to_string(i) + " failed: " + hs->c->err);
      return nullptr;
    }
  }
  if (!hs->coded[i]) return nullptr;  // not re-coded: decode natively (recode.cpp:1139-1145)
  if (hs->lazy && !hs->regen_done[i] && guarded(hs->c, [&] { return lazy_device_work(hs, i, true); }) != AVR_OK) {
    hs->fail_once("hooks: device decode of slice " + std::to_string(i) + " failed: " + hs->c->err);
    return nullptr;
  }
  if (hs->decompress) {
    // recognize_coded_block (recode.cpp:1546-1573)
    uint8_t mk[8];
    avr::surrogate_marker(hs->next_marker++, mk);
    if (size < 8 || memcmp(buf, mk, 8) != 0) {
      hs->fail_once("hooks: invalid surrogate marker in slice " + std::to_string(i));
      return nullptr;
    }
  } else if (memcmp(buf, s.payload(), s.size) != 0) {
    hs->fail_once("hooks: slice " + std::to_string(i) + " payload differs from the file's");
    return nullptr;
  }
  avr_hooks_slice& h = hs->slices[i];
  h.sess = hs;
  h.index = (int)i;
  h.trace = hs->bins[i].data();
  h.nbins = hs->bins[i].size() / 2;
  h.cur = 0;
  h.maps = hs->maps[i].data();
  h.nmaps = hs->maps[i].size();
  h.map_cur = 0;
  hs->live = &h;
  return &h;
}

static int hook_bin(void* slice, int kind, uint8_t* state) {
  avr_hooks_slice* h = (avr_hooks_slice*)slice;
  if (!h || !h->sess) return 0;
  if (h->cur >= h->nbins) {
    h->sess->fail_once("hooks: slice " + std::to_string(h->index) + " asked for more bins than it holds");
    return 0;
  }
  const uint8_t t = h->trace[2 * h->cur], pre = h->trace[2 * h->cur + 1];
  h->cur++;
  const int bin = t & 1;
  if (((t >> 1) & 3) != kind) {
    h->sess->fail_once("hooks: slice " + std::to_string(h->index) + " bin " + std::to_string(h->cur - 1) +
                       ": bin kind differs from the device's parse");
    return bin;
  }
  if (state) {
    if (*state != pre)
      h->sess->fail_once("hooks: slice " + std::to_string(h->index) + " bin " + std::to_string(h->cur - 1) +
                         ": context state differs from the device's parse");
    *state = next_state(*state, bin);
  }
  return bin;
}

int avr_hook_get(void* slice, uint8_t* state) {
  if (!state) {
    if (slice && ((avr_hooks_slice*)slice)->sess) ((avr_hooks_slice*)slice)->sess->fail_once("hooks: get without a state");
    return 0;
  }
  return hook_bin(slice, 0, state);
}
int avr_hook_get_bypass(void* slice) { return hook_bin(slice, 1, nullptr); }
int avr_hook_get_terminate(void* slice) { return hook_bin(slice, 2, nullptr); }

const uint8_t* avr_hook_skip_bytes(void* slice, int /*n*/) {
  avr_hooks_slice* h = (avr_hooks_slice*)slice;
  if (h && h->sess) h->sess->fail_once("hooks: skip_bytes (I_PCM) is not supported");
  return nullptr;
}

void avr_hook_frame_spec(void* opaque, int frame_num, int mb_width, int mb_height) {
  avr_hooks_session* hs = (avr_hooks_session*)opaque;
  if (!hs) return;
  avr_hooks_slice* h = hs->live;
  if (h && h->cur < h->nbins) {   // inside a slice's decode: that slice's picture
    check_frame_spec(hs, h->index, frame_num, mb_width, mb_height);
    return;
  }
  if (hs->fs_pending && (hs->pend_num != frame_num || hs->pend_w != mb_width || hs->pend_h != mb_height))
    hs->fail_once("hooks: two different frame_spec calls before one slice");
  hs->fs_pending = true;
  hs->pend_num = frame_num, hs->pend_w = mb_width, hs->pend_h = mb_height;
}

void avr_hook_mb_xy(void* opaque, int x, int y) {
  avr_hooks_session* hs = (avr_hooks_session*)opaque;
  if (!hs) return;
  hs->mb_calls++;
  hs->mb_x = x;
  hs->mb_y = y;
}

void avr_hook_begin_sub_mb(void* opaque, int cat, int scan8index, int max_coeff, int is_dc, int chroma422) {
  avr_hooks_session* hs = (avr_hooks_session*)opaque;
  if (!hs || !hs->live) return;
  avr_hooks_slice* h = hs->live;
  if (h->sub_open) hs->fail_once("hooks: begin_sub_mb inside an open sub-macroblock");
  h->sub_open = true;
  const int a[5] = {cat, scan8index, max_coeff, is_dc, chroma422};
  memcpy(h->sub_args, a, sizeof(a));
}

void avr_hook_end_sub_mb(void* opaque, int cat, int scan8index, int max_coeff, int is_dc, int chroma422) {
  avr_hooks_session* hs = (avr_hooks_session*)opaque;
  if (!hs || !hs->live) return;
  avr_hooks_slice* h = hs->live;
  const int a[5] = {cat, scan8index, max_coeff, is_dc, chroma422};
  if (!h->sub_open || memcmp(h->sub_args, a, sizeof(a)) != 0)  // recode.cpp:185-189
    hs->fail_once("hooks: end_sub_mb does not match begin_sub_mb");
  h->sub_open = false;
}

// begin_coding_type(SIG_MAP) (recode.cpp:951-974) starts the model's significance-map keys: it
// must come exactly before the device's map's first bin, under the device's macroblock (mb_xy)
// and sub-macroblock (begin_sub_mb), with zigzag_index 0 (recode.cpp:961); end_coding_type right
// after its last bin (recode.cpp:931-950).  Other coding types carry no device event.
void avr_hook_begin_coding_type(void* opaque, int coding_type, int zigzag_index, int /*param0*/, int /*param1*/) {
  avr_hooks_session* hs = (avr_hooks_session*)opaque;
  if (!hs || !hs->live) return;
  avr_hooks_slice* h = hs->live;
  if (h->coding_type != AVR_PIP_UNKNOWN) hs->fail_once("hooks: nested begin_coding_type");
  h->coding_type = coding_type;
  if (coding_type != AVR_PIP_SIGNIFICANCE_MAP) return;
  const std::string where = "hooks: slice " + std::to_string(h->index) + " bin " + std::to_string(h->cur) + ": ";
  if (h->map_cur >= h->nmaps) {
    hs->fail_once(where + "begin_coding_type(SIG_MAP) where the device's parse has no significance map");
    return;
  }
  const HookMap& m = h->maps[h->map_cur];
  if (h->cur != m.begin)
    hs->fail_once(where + "begin_coding_type(SIG_MAP) where the device's map begins at bin " + std::to_string(m.begin));
  else if (zigzag_index != 0)
    hs->fail_once(where + "begin_coding_type(SIG_MAP) with zigzag_index != 0");
  else if (hs->mb_x != m.x || hs->mb_y != m.y)
    hs->fail_once(where + "significance map under mb_xy(" + std::to_string(hs->mb_x) + ", " + std::to_string(hs->mb_y) +
                  "), the device's is (" + std::to_string(m.x) + ", " + std::to_string(m.y) + ")");
  else if (!h->sub_open || memcmp(h->sub_args, m.sub, sizeof(m.sub)) != 0)
    hs->fail_once(where + "significance map outside the device's sub-macroblock (cat " + std::to_string(m.sub[0]) +
                  ", scan8 " + std::to_string(m.sub[1]) + ", max " + std::to_string(m.sub[2]) + ")");
}

void avr_hook_end_coding_type(void* opaque, int coding_type) {
  avr_hooks_session* hs = (avr_hooks_session*)opaque;
  if (!hs || !hs->live) return;
  avr_hooks_slice* h = hs->live;
  if (h->coding_type != coding_type) hs->fail_once("hooks: end_coding_type does not match begin_coding_type");
  h->coding_type = AVR_PIP_UNKNOWN;
  if (coding_type != AVR_PIP_SIGNIFICANCE_MAP || h->map_cur >= h->nmaps) return;
  const HookMap& m = h->maps[h->map_cur++];
  if (h->cur != m.end)
    hs->fail_once("hooks: slice " + std::to_string(h->index) + " bin " + std::to_string(h->cur) +
                  ": end_coding_type(SIG_MAP) where the device's map ends at bin " + std::to_string(m.end));
}

int avr_hooks_end(avr_hooks_session* hs, uint8_t** out, size_t* out_len) {
  if (!hs || !out || !out_len) return AVR_ERR_INVALID_ARGUMENT;
  close_live(hs);
  if (hs->streaming) {
    // the whole file is in: its last slices, and the container (recode.cpp:1102-1125).  The
    // parallel model's blocks are final as each slice was traced (slices independent): the container
    // is assembled from them.  The reference model's estimators chain across slices, so its
    // container comes from one compress of the whole file.
    if (int r = guarded(hs->c, [&] {
          const int e = ingest(hs, true, 0);
          grow_session(hs);
          if (!e && hs->err.empty() && parallel_model(hs->model)) return stream_device_work(hs, 0);
          return e;
        }))
      return r;
    if (hs->err.empty()) {
      uint8_t* avrc = nullptr;
      size_t avrc_len = 0;
      if (parallel_model(hs->model)) {
        if (int r = guarded(hs->c, [&] {
              std::vector<char> ok(hs->pf.slices.size(), 0);
              std::vector<std::pair<const uint8_t*, size_t>> blobs(hs->pf.slices.size(), {nullptr, 0});
              for (size_t i = 0; i < ok.size(); i++) {
                ok[i] = recodable_candidate(hs->pf.slices[i]) && hs->block_status[i] == 0;
                blobs[i] = {hs->blocks[i].data(), hs->blocks[i].size()};
              }
              const std::vector<SliceView> sv = views_of(hs->pf);
              return emit_container(hs->original.data(), hs->original.size(), sv,
                                    segment(hs->original.data(), hs->original.size(), sv, ok), blobs, hs->model,
                                    &avrc, &avrc_len);
            }))
          return r;
      } else if (int r = avr_compress_file(hs->c, hs->original.data(), hs->original.size(), hs->model, &avrc,
                                           &avrc_len)) {
        return r;
      }
      hs->result.assign(avrc, avrc + avrc_len);
      free(avrc);
    }
  }
  if (hs->lazy && hs->err.empty()) {
    // the original file: literals and regenerated slices in block order (decompressor::run's output,
    // recode.cpp:1338-1357), slices no init_decoder reached regenerated now
    if (int r = guarded(hs->c, [&]() -> int {
          if (int e = lazy_device_work(hs, 0, false, hs->pf.slices.size())) return e;
          std::vector<uint8_t> o;
          o.reserve(hs->stream.size());
          size_t i = 0;
          for (const avr::PbBlock& b : hs->job.blocks) {
            if (b.has_literal) {
              o.insert(o.end(), b.literal, b.literal + b.literal_len);
              continue;
            }
            if (b.has_cabac) o.insert(o.end(), hs->regen[i].begin(), hs->regen[i].end());
            i++;
          }
          hs->result.swap(o);
          return AVR_OK;
        }))
      return r;
  }
  if (hs->next_slice != hs->pf.slices.size())
    hs->fail_once("hooks: " + std::to_string(hs->next_slice) + " of " + std::to_string(hs->pf.slices.size()) +
                  " slices were decoded");
  if (!hs->err.empty()) return fail(hs->c, AVR_ERR_FORMAT, hs->err);
  *out = (uint8_t*)malloc(hs->result.size() ? hs->result.size() : 1);
  if (!*out) return AVR_ERR_OUT_OF_MEMORY;
  memcpy(*out, hs->result.data(), hs->result.size());
  *out_len = hs->result.size();
  return AVR_OK;
}

void avr_hooks_destroy(avr_hooks_session* hs) { delete hs; }

// Debug (tests, host only; not part of include/avrecode.h): how many slices a decompress session
// has regenerated on the device so far (a lazy parallel-model session: those init_decoder reached,
// in batches; -1: an eager session, which regenerated the whole file at begin).
extern "C" int avr_debug_hooks_regenerated(const avr_hooks_session* hs) {
  if (!hs || !hs->decompress) return AVR_ERR_INVALID_ARGUMENT;
  if (!hs->lazy) return -1;
  int k = 0;
  for (const char d : hs->regen_done) k += d ? 1 : 0;
  return k;
}

// Debug (tests, host only; not part of include/avrecode.h): the slices a streaming session's
// incremental parser finds when `file` is fed in pieces ending at cuts[0] < ... < cuts[ncuts - 1] = n
// (incremental = 1; after each piece the parser is asked for one slice more than it holds when
// provisional = 1, as a decoder's next init_decoder would), or that parse_file finds in the whole
// file (incremental = 0).  out: 4 u64 per slice (NAL offset, NAL size, payload size, picture id).
// Returns the slice count (at most cap written), or < 0.
extern "C" int avr_debug_stream_slices(const uint8_t* file, size_t n, const uint64_t* cuts, int ncuts, int incremental,
                                       int provisional, uint64_t* out, int cap) {
  if (!file || (incremental && (!cuts || ncuts <= 0)) || (!out && cap)) return AVR_ERR_INVALID_ARGUMENT;
  return guarded(nullptr, [&]() -> int {
    avr_hooks_session hs;
    hs.streaming = true;
    if (incremental) {
      size_t fed = 0;
      for (int k = 0; k < ncuts; k++) {
        const size_t end = std::min<size_t>(n, cuts[k]);
        if (end > fed) hs.original.insert(hs.original.end(), file + fed, file + end);
        fed = std::max(fed, end);
        if (int r = ingest(&hs, false, 0)) return r;
        if (provisional)
          if (int r = ingest(&hs, false, hs.pf.slices.size() + 1)) return r;
      }
      if (fed < n) hs.original.insert(hs.original.end(), file + fed, file + n);
      if (int r = ingest(&hs, true, 0)) return r;
    } else if (int r = parse_file(nullptr, file, n, &hs.pf)) {
      return r;
    }
    const int cnt = (int)hs.pf.slices.size();
    for (int i = 0; i < cnt && i < cap; i++) {
      const avr::SliceInfo& si = hs.pf.slices[i];
      out[4 * i] = si.nal_offset, out[4 * i + 1] = si.nal_size, out[4 * i + 2] = si.size;
      out[4 * i + 3] = (uint64_t)si.picture_id;
    }
    return cnt;
  });
}
