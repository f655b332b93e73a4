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

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

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
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
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
  DevBuf tables, est, frames, frame_meta, in, out, descs, res, packed, offsets;
};

namespace {

constexpr int kMaxSlicesPerLaunch = 4096;

int fail(avr_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
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

struct Plan {
  std::vector<avr_slice_desc> descs;
  std::vector<uint8_t> arena;   // payloads (compress) or recoded streams (decompress)
  int max_w = 1;
};

void append_aligned(std::vector<uint8_t>* arena, const uint8_t* p, size_t n, size_t extra, uint64_t* off) {
  size_t o = (arena->size() + 15) & ~(size_t)15;
  arena->resize(o + n + extra, 0);
  if (n) memcpy(arena->data() + o, p, n);
  *off = o;
}

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
  return d;
}

// Upload plan, run the slice kernel over it (in chunks), download results and outputs.
int run_plan(avr_ctx* c, int mode, bool sequential, Plan& plan, std::vector<avr_slice_result>* res,
             std::vector<uint8_t>* out_host) {
  const int n = (int)plan.descs.size();
  res->assign(n, avr_slice_result{0, 0, 0, 0});
  uint64_t out_total = 0;
  for (auto& d : plan.descs) {
    d.out_offset = out_total;
    out_total += ((uint64_t)d.out_capacity + 15) & ~15ull;
  }
  out_host->assign(out_total, 0);
  if (!n) return AVR_OK;
  HIP_TRY(c, c->in.reserve(plan.arena.size() + 4096));
  HIP_TRY(c, hipMemcpyAsync(c->in.p, plan.arena.data(), plan.arena.size(), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, c->out.reserve(out_total + 4096));
  HIP_TRY(c, c->descs.reserve(sizeof(avr_slice_desc) * n));
  HIP_TRY(c, c->res.reserve(sizeof(avr_slice_result) * n));
  HIP_TRY(c, hipMemcpyAsync(c->descs.p, plan.descs.data(), sizeof(avr_slice_desc) * n, hipMemcpyHostToDevice,
                            c->stream));
  if (sequential) {
    HIP_TRY(c, c->est.reserve(sizeof(uint16_t) * avr::kEstGlobal));
    size_t fbytes = 0;
    for (auto& d : plan.descs) fbytes = std::max(fbytes, (size_t)2 * d.mb_width * d.mb_height * 52);
    HIP_TRY(c, c->frames.reserve(fbytes + 64));
    HIP_TRY(c, c->frame_meta.reserve(64));
    HIP_TRY(c, avr::launch_slices(mode, true, c->tables.as<avr::EngineTables>(), c->descs.as<avr_slice_desc>(), n,
                                  plan.max_w, c->in.as<uint8_t>(), c->out.as<uint8_t>(), c->res.as<avr_slice_result>(),
                                  c->est.as<uint16_t>(), c->frames.as<uint8_t>(), c->frame_meta.as<int>(), c->stream));
  } else {
    const int chunk = std::min(n, kMaxSlicesPerLaunch);
    HIP_TRY(c, c->est.reserve(sizeof(uint16_t) * (size_t)avr::kEstGlobal * chunk));
    for (int s0 = 0; s0 < n; s0 += chunk) {
      const int m = std::min(chunk, n - s0);
      HIP_TRY(c, avr::launch_slices(mode, false, c->tables.as<avr::EngineTables>(), c->descs.as<avr_slice_desc>() + s0,
                                    m, plan.max_w, c->in.as<uint8_t>(), c->out.as<uint8_t>(),
                                    c->res.as<avr_slice_result>() + s0, c->est.as<uint16_t>(), nullptr, nullptr,
                                    c->stream));
    }
  }
  HIP_TRY(c, hipMemcpyAsync(res->data(), c->res.p, sizeof(avr_slice_result) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(out_host->data(), c->out.p, out_total, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return AVR_OK;
}

struct ParsedFile {
  std::vector<avr::SliceInfo> slices;
};

int parse_file(avr_ctx* c, const uint8_t* in, size_t n, ParsedFile* pf) {
  std::vector<avr::NalRef> nals;
  if (!avr::demux(in, n, &nals)) return fail(c, AVR_ERR_FORMAT, "not an MP4/avcC or Annex-B H.264 stream");
  avr::StreamParser sp;
  for (auto& nr : nals) {
    avr::SliceInfo s;
    if (sp.next(in + nr.offset, nr.size, &s)) {
      s.nal_offset = nr.offset;
      s.nal_size = nr.size;
      pf->slices.push_back(std::move(s));
    }
  }
  return AVR_OK;
}

bool recodable_candidate(const avr::SliceInfo& s) { return s.h.supported && s.size >= (size_t)avr::kSurrogateMarkerBytes; }

// find_next_coded_block_and_emit_literal (recode.cpp:1275-1297): slice i becomes a cabac block when
// it is recodable (ok[i]), at least a surrogate marker long, and its payload occurs verbatim after
// the previous coded block.  Returns the payload's position in the file per slice (null = skip).
std::vector<const uint8_t*> segment(const uint8_t* in, size_t n, const ParsedFile& pf, const std::vector<char>& ok) {
  std::vector<const uint8_t*> found(pf.slices.size(), nullptr);
  size_t prev_end = 0;
  for (size_t i = 0; i < pf.slices.size(); i++) {
    const avr::SliceInfo& s = pf.slices[i];
    if (!ok[i] || s.size < (size_t)avr::kSurrogateMarkerBytes) continue;
    const uint8_t* f = (const uint8_t*)memmem(in + prev_end, n - prev_end, s.payload(), s.size);
    if (f) {
      found[i] = f;
      prev_end = (size_t)(f - in) + s.size;
    }
  }
  return found;
}

// compressor::run's block stream (recode.cpp:1115-1125, 1275-1297) as a Recoded protobuf.
int emit_container(const uint8_t* in, size_t n, const ParsedFile& pf, const std::vector<const uint8_t*>& found,
                   const std::vector<std::pair<const uint8_t*, size_t>>& recoded, bool parallel, uint8_t** out,
                   size_t* out_len) {
  std::vector<uint8_t> o;
  o.reserve(n + n / 8 + 1024);
  if (parallel) avr::pb_put_metadata_version(&o, avr::kParallelModelTag);
  size_t prev_end = 0;
  for (size_t i = 0; i < pf.slices.size(); i++) {
    const avr::SliceInfo& s = pf.slices[i];
    avr::PbBlock b;
    if (found[i]) {
      avr::PbBlock lit;
      lit.has_literal = true;
      lit.literal = in + prev_end;
      lit.literal_len = (size_t)(found[i] - (in + prev_end));
      avr::pb_put_block(&o, lit);
      prev_end = (size_t)(found[i] - in) + s.size;
      b.has_size = true;
      b.size = (int64_t)s.size;
      b.has_parity = true;
      b.length_parity = s.size & 1;
      if (s.size > 1) b.has_last_byte = true, b.last_byte.assign(1, (char)s.payload()[s.size - 1]);
      b.has_cabac = true;
      b.cabac = recoded[i].first;
      b.cabac_len = recoded[i].second;
    } else {
      b.has_skip = true;
      b.skip_coded = true;
      b.has_size = true;
      b.size = (int64_t)s.size;
    }
    avr::pb_put_block(&o, b);
  }
  avr::PbBlock lit;
  lit.has_literal = true;
  lit.literal = in + prev_end;
  lit.literal_len = n - prev_end;
  avr::pb_put_block(&o, lit);
  *out = (uint8_t*)malloc(o.size() ? o.size() : 1);
  if (!*out) return AVR_ERR_OUT_OF_MEMORY;
  memcpy(*out, o.data(), o.size());
  *out_len = o.size();
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
  avr::EngineTables t;
  build_tables(&t);
  if (!check_reciprocals(t)) return AVR_ERR_DEVICE;
  if (c->tables.reserve(sizeof(t)) != hipSuccess) return AVR_ERR_OUT_OF_MEMORY;
  if (hipMemcpy(c->tables.p, &t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess) return AVR_ERR_DEVICE;
  *out = c.release();
  return AVR_OK;
}

void avr_destroy(avr_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (DevBuf* b : {&c->tables, &c->est, &c->frames, &c->frame_meta, &c->in, &c->out, &c->descs, &c->res, &c->packed,
                    &c->offsets})
    b->release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* avr_last_error(const avr_ctx* c) { return c ? c->err.c_str() : "no context"; }

void avr_free(void* p) { free(p); }

int avr_compress_file(avr_ctx* c, const uint8_t* in, size_t n, int model, uint8_t** out, size_t* out_len) {
  if (!c || !in || !out || !out_len || (model != AVR_MODEL_REFERENCE && model != AVR_MODEL_PARALLEL))
    return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  ParsedFile pf;
  if (int r = parse_file(c, in, n, &pf)) return r;
  // 1) every candidate slice through the parallel kernel: per-slice parse + restore check (and
  //    the parallel model's output)
  Plan plan;
  std::vector<int> cand_of(pf.slices.size(), -1);
  for (size_t i = 0; i < pf.slices.size(); i++) {
    const avr::SliceInfo& s = pf.slices[i];
    if (!recodable_candidate(s)) continue;
    avr_slice_desc d = desc_from_header(s);
    append_aligned(&plan.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
    d.payload_size = (uint32_t)s.size;
    d.read_limit = (uint32_t)s.read_limit;
    d.out_capacity = (uint32_t)(s.size * 2 + 256);
    plan.max_w = std::max(plan.max_w, d.mb_width);
    cand_of[i] = (int)plan.descs.size();
    plan.descs.push_back(d);
  }
  std::vector<avr_slice_result> res;
  std::vector<uint8_t> outb;
  if (int r = run_plan(c, 0, false, plan, &res, &outb)) return r;
  std::vector<char> ok(pf.slices.size(), 0);
  for (size_t i = 0; i < pf.slices.size(); i++) ok[i] = cand_of[i] >= 0 && res[cand_of[i]].status == 0;
  // 2) segmentation (find_next_coded_block_and_emit_literal, recode.cpp:1275-1297)
  std::vector<const uint8_t*> found = segment(in, n, pf, ok);
  // 3) reference model: re-run the coded slices through the sequential kernel in file order;
  //    a slice that fails there is demoted to skip_coded and the pass repeated.
  std::vector<std::vector<uint8_t>> recoded(pf.slices.size());
  if (model == AVR_MODEL_REFERENCE) {
    for (int attempt = 0; attempt < 8; attempt++) {
      Plan rp;
      std::vector<int> idx;
      for (size_t i = 0; i < pf.slices.size(); i++) {
        const avr::SliceInfo& s = pf.slices[i];
        avr_slice_desc d = desc_from_header(s);
        d.coded = found[i] != nullptr;
        if (d.coded) {
          append_aligned(&rp.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
          d.payload_size = (uint32_t)s.size;
          d.read_limit = (uint32_t)s.read_limit;
          d.out_capacity = (uint32_t)(s.size * 4 + 4096);
        }
        rp.max_w = std::max(rp.max_w, d.mb_width);
        idx.push_back((int)i);
        rp.descs.push_back(d);
      }
      std::vector<avr_slice_result> rr;
      std::vector<uint8_t> ro;
      if (int r = run_plan(c, 0, true, rp, &rr, &ro)) return r;
      bool again = false;
      for (size_t k = 0; k < idx.size(); k++) {
        const int i = idx[k];
        if (!found[i]) continue;
        if (rr[k].status != 0) {
          found[i] = nullptr;
          again = true;
          continue;
        }
        recoded[i].assign(ro.begin() + rp.descs[k].out_offset, ro.begin() + rp.descs[k].out_offset + rr[k].out_len);
      }
      if (!again) break;
      // a demoted slice changes the literal gaps of later ones: redo the segmentation
      for (size_t i = 0; i < pf.slices.size(); i++) ok[i] = ok[i] && found[i] != nullptr;
      found = segment(in, n, pf, ok);
      if (attempt == 7) return fail(c, AVR_ERR_DEVICE, "reference-model pass did not converge");
    }
  } else {
    for (size_t i = 0; i < pf.slices.size(); i++)
      if (found[i]) {
        const int k = cand_of[i];
        recoded[i].assign(outb.begin() + plan.descs[k].out_offset,
                          outb.begin() + plan.descs[k].out_offset + res[k].out_len);
      }
  }
  // 4) container (compressor::run, recode.cpp:1115-1125)
  std::vector<std::pair<const uint8_t*, size_t>> blobs(pf.slices.size(), {nullptr, 0});
  for (size_t i = 0; i < pf.slices.size(); i++) blobs[i] = {recoded[i].data(), recoded[i].size()};
  return emit_container(in, n, pf, found, blobs, model == AVR_MODEL_PARALLEL, out, out_len);
}

int avr_assemble_container(const uint8_t* file, size_t n, int n_slices, const int32_t* status, const uint8_t* recoded,
                           const uint64_t* offsets, const uint32_t* lens, uint8_t** out, size_t* out_len) {
  if (!file || !out || !out_len || n_slices < 0 || (n_slices && (!status || !offsets || !lens)))
    return AVR_ERR_INVALID_ARGUMENT;
  ParsedFile pf;
  if (int r = parse_file(nullptr, file, n, &pf)) return r;
  if ((size_t)n_slices != pf.slices.size()) return AVR_ERR_INVALID_ARGUMENT;
  std::vector<char> ok(pf.slices.size(), 0);
  std::vector<std::pair<const uint8_t*, size_t>> blobs(pf.slices.size(), {nullptr, 0});
  for (size_t i = 0; i < pf.slices.size(); i++) {
    ok[i] = recodable_candidate(pf.slices[i]) && status[i] == 0;
    if (ok[i]) {
      if (!recoded) return AVR_ERR_INVALID_ARGUMENT;
      blobs[i] = {recoded + offsets[i], lens[i]};
    }
  }
  return emit_container(file, n, pf, segment(file, n, pf, ok), blobs, true, out, out_len);
}

int avr_decompress_file(avr_ctx* c, const uint8_t* in, size_t n, uint8_t** out, size_t* out_len) {
  if (!c || !in || !out || !out_len) return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  std::vector<avr::PbBlock> blocks;
  std::string version;
  if (!avr::pb_parse(in, n, &blocks, &version)) return fail(c, AVR_ERR_FORMAT, "not a Recoded protobuf");
  const bool parallel = version == avr::kParallelModelTag;
  // read_packet (recode.cpp:1359-1409): literals and surrogate blocks form the stream
  std::vector<uint8_t> stream;
  uint64_t seq = 1;
  for (auto& b : blocks) {
    if ((int)b.has_literal + (int)b.has_cabac + (int)b.has_skip != 1)
      return fail(c, AVR_ERR_FORMAT, "Invalid input block: must have exactly one type");
    if (b.has_literal) {
      stream.insert(stream.end(), b.literal, b.literal + b.literal_len);
    } else if (b.has_cabac) {
      if (!b.has_size) return fail(c, AVR_ERR_FORMAT, "CABAC block requires size field.");
      if (b.size < avr::kSurrogateMarkerBytes)
        return fail(c, AVR_ERR_FORMAT, "Invalid coded block size for surrogate: " + std::to_string(b.size));
      uint8_t mk[8];
      avr::surrogate_marker(seq++, mk);
      stream.insert(stream.end(), mk, mk + 8);
      stream.insert(stream.end(), (size_t)b.size - 8, (uint8_t)'X');
    } else if (!b.skip_coded) {
      return fail(c, AVR_ERR_FORMAT, "Unknown input block type");
    }
  }
  ParsedFile pf;
  if (int r = parse_file(c, stream.data(), stream.size(), &pf)) return r;
  // recognize_coded_block (recode.cpp:1546-1573): slices claim coded blocks in order
  Plan plan;
  std::vector<int> block_of_desc;
  size_t next_coded = 0;
  uint64_t seq_check = 1;
  for (auto& s : pf.slices) {
    while (next_coded < blocks.size() && !blocks[next_coded].has_cabac && !blocks[next_coded].has_skip) next_coded++;
    if (next_coded >= blocks.size())
      return fail(c, AVR_ERR_FORMAT, "Coded block expected, but not recorded in the compressed data.");
    const avr::PbBlock& b = blocks[next_coded];
    if ((size_t)b.size != s.size) return fail(c, AVR_ERR_FORMAT, "Invalid surrogate block size.");
    avr_slice_desc d = desc_from_header(s);
    if (b.has_cabac) {
      uint8_t mk[8];
      avr::surrogate_marker(seq_check++, mk);
      if (memcmp(s.payload(), mk, 8) != 0) return fail(c, AVR_ERR_FORMAT, "Invalid surrogate marker in coded block.");
      append_aligned(&plan.arena, b.cabac, b.cabac_len, 16, &d.payload_offset);
      d.payload_size = (uint32_t)b.cabac_len;
      d.read_limit = (uint32_t)b.cabac_len;
      d.out_capacity = (uint32_t)(b.size + 64);
    } else {
      d.coded = 0;
    }
    plan.max_w = std::max(plan.max_w, d.mb_width);
    if (parallel && !d.coded) {
      next_coded++;
      continue;
    }
    block_of_desc.push_back((int)next_coded);
    plan.descs.push_back(d);
    next_coded++;
  }
  std::vector<avr_slice_result> res;
  std::vector<uint8_t> outb;
  if (int r = run_plan(c, 1, !parallel, plan, &res, &outb)) return r;
  std::vector<std::vector<uint8_t>> regen(blocks.size());
  std::vector<char> done(blocks.size(), 0);
  for (size_t k = 0; k < plan.descs.size(); k++) {
    const int bi = block_of_desc[k];
    if (!plan.descs[k].coded) continue;
    if (res[k].status != 0)
      return fail(c, AVR_ERR_FORMAT, "slice " + std::to_string(k) + " failed to decode (" + std::to_string(res[k].status) + ")");
    const avr::PbBlock& b = blocks[bi];
    std::vector<uint8_t> v(outb.begin() + plan.descs[k].out_offset,
                           outb.begin() + plan.descs[k].out_offset + res[k].out_len);
    // x264 padding correction (recode.cpp:1345-1356)
    if (b.has_parity && b.has_last_byte && !b.last_byte.empty()) {
      if ((int)b.length_parity != (int)(v.size() & 1)) v.push_back((uint8_t)b.last_byte[0]);
      else if (!v.empty()) v.back() = (uint8_t)b.last_byte[0];
    }
    regen[bi] = std::move(v);
    done[bi] = 1;
  }
  std::vector<uint8_t> o;
  o.reserve(stream.size());
  for (size_t i = 0; i < blocks.size(); i++) {
    if (blocks[i].has_literal) o.insert(o.end(), blocks[i].literal, blocks[i].literal + blocks[i].literal_len);
    else if (blocks[i].has_cabac) {
      if (!done[i]) return fail(c, AVR_ERR_FORMAT, "Not all blocks were decoded.");
      o.insert(o.end(), regen[i].begin(), regen[i].end());
    }
  }
  *out = (uint8_t*)malloc(o.size() ? o.size() : 1);
  if (!*out) return AVR_ERR_OUT_OF_MEMORY;
  memcpy(*out, o.data(), o.size());
  *out_len = o.size();
  return AVR_OK;
}

int avr_roundtrip_file(avr_ctx* c, const uint8_t* in, size_t n, int model, uint8_t** compressed,
                       size_t* compressed_len, avr_file_stats* stats) {
  if (!c || !in) return AVR_ERR_INVALID_ARGUMENT;
  uint8_t *comp = nullptr, *dec = nullptr;
  size_t cn = 0, dn = 0;
  const double t0 = now_s();
  if (int r = avr_compress_file(c, in, n, model, &comp, &cn)) return r;
  const double t1 = now_s();
  int r = avr_decompress_file(c, comp, cn, &dec, &dn);
  const double t2 = now_s();
  if (r) {
    free(comp);
    return r;
  }
  const bool same = dn == n && memcmp(dec, in, n) == 0;
  free(dec);
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->file_bytes = n;
    stats->compress_s = t1 - t0;
    stats->decompress_s = t2 - t1;
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

static int batch(avr_ctx* c, int mode, const avr_slice_desc* d_desc, int n, int max_w, int max_h,
                 const uint8_t* d_in, uint8_t* d_out, avr_slice_result* d_res, int model, void* stream) {
  if (!c || n < 0 || (n && (!d_desc || !d_in || !d_out || !d_res)) || max_w <= 0 || max_h <= 0 ||
      (model != AVR_MODEL_REFERENCE && model != AVR_MODEL_PARALLEL))
    return AVR_ERR_INVALID_ARGUMENT;
  if (avr::shared_bytes(max_w) > 160 * 1024) return fail(c, AVR_ERR_UNSUPPORTED, "picture too wide for the LDS ring");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  if (model == AVR_MODEL_REFERENCE) {
    HIP_TRY(c, c->est.reserve(sizeof(uint16_t) * avr::kEstGlobal));
    HIP_TRY(c, c->frames.reserve((size_t)2 * max_w * max_h * 52 + 64));
    HIP_TRY(c, c->frame_meta.reserve(64));
    HIP_TRY(c, avr::launch_slices(mode, true, c->tables.as<avr::EngineTables>(), d_desc, n, max_w, d_in, d_out, d_res,
                                  c->est.as<uint16_t>(), c->frames.as<uint8_t>(), c->frame_meta.as<int>(), s));
    return AVR_OK;
  }
  const int chunk = std::max(1, std::min(n, kMaxSlicesPerLaunch));
  HIP_TRY(c, c->est.reserve(sizeof(uint16_t) * (size_t)avr::kEstGlobal * chunk));
  for (int s0 = 0; s0 < n; s0 += chunk) {
    const int m = std::min(chunk, n - s0);
    HIP_TRY(c, avr::launch_slices(mode, false, c->tables.as<avr::EngineTables>(), d_desc + s0, m, max_w, d_in, d_out,
                                  d_res + s0, c->est.as<uint16_t>(), nullptr, nullptr, s));
  }
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

int avr_parse_stream(const uint8_t* file, size_t n, avr_slice_desc** descs, int* n_slices, uint8_t** arena,
                     size_t* arena_len, size_t* work_len, int* max_w, int* max_h) {
  if (!file || !descs || !n_slices || !arena || !arena_len || !work_len || !max_w || !max_h)
    return AVR_ERR_INVALID_ARGUMENT;
  *descs = nullptr;
  *arena = nullptr;
  ParsedFile pf;
  if (int r = parse_file(nullptr, file, n, &pf)) return r;
  Plan plan;
  uint64_t work = 0;
  int mh = 1;
  for (const avr::SliceInfo& s : pf.slices) {
    avr_slice_desc d = desc_from_header(s);
    append_aligned(&plan.arena, s.payload(), s.read_limit, 16, &d.payload_offset);
    d.payload_size = (uint32_t)s.size;
    d.read_limit = (uint32_t)s.read_limit;
    d.coded = recodable_candidate(s);
    d.out_offset = work;
    d.out_capacity = (uint32_t)(s.size * 2 + 256);
    work += ((uint64_t)d.out_capacity + 15) & ~15ull;
    plan.max_w = std::max(plan.max_w, d.mb_width);
    mh = std::max(mh, d.mb_height);
    plan.descs.push_back(d);
  }
  plan.arena.resize(plan.arena.size() + 16, 0);
  const size_t dn = sizeof(avr_slice_desc) * plan.descs.size();
  *descs = (avr_slice_desc*)malloc(dn ? dn : 1);
  *arena = (uint8_t*)malloc(plan.arena.size());
  if (!*descs || !*arena) {
    free(*descs);
    free(*arena);
    *descs = nullptr;
    *arena = nullptr;
    return AVR_ERR_OUT_OF_MEMORY;
  }
  if (dn) memcpy(*descs, plan.descs.data(), dn);
  memcpy(*arena, plan.arena.data(), plan.arena.size());
  *n_slices = (int)plan.descs.size();
  *arena_len = plan.arena.size();
  *work_len = work;
  *max_w = plan.max_w;
  *max_h = mh;
  return AVR_OK;
}

int avr_pack_outputs(avr_ctx* c, const avr_slice_desc* d_desc, const avr_slice_result* d_res, int n,
                     const uint8_t* d_out, uint8_t* d_packed, uint64_t* d_offsets, void* stream) {
  if (!c || n < 0 || (n && (!d_desc || !d_res || !d_out || !d_packed || !d_offsets))) return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, avr::launch_pack(d_desc, d_res, n, d_out, d_packed, d_offsets, (hipStream_t)stream));
  return AVR_OK;
}

int avr_synthesize_stream(avr_ctx* c, const avr_synth_params* p, int n, uint8_t** out, size_t* out_len) {
  if (!c || !p || n <= 0 || !out || !out_len || p->mb_width <= 0 || p->mb_height <= 0 || p->slice_type < 0 ||
      p->slice_type > 2 || p->chroma_format_idc < 1 || p->chroma_format_idc > 3)
    return AVR_ERR_INVALID_ARGUMENT;
  HIP_TRY(c, hipSetDevice(c->device));
  Plan plan;
  const int mbs = p->mb_width * p->mb_height;
  for (int i = 0; i < n; i++) {
    avr_slice_desc d;
    memset(&d, 0, sizeof(d));
    d.slice_type = p->slice_type;
    d.slice_qp = p->slice_qp;
    d.cabac_init_idc = p->slice_type == 2 ? -1 : 0;
    d.mb_width = p->mb_width;
    d.mb_height = p->mb_height;
    d.num_ref_idx_l0 = p->slice_type == 2 ? 0 : std::max(1, p->num_ref_idx_l0);
    d.num_ref_idx_l1 = p->slice_type == 1 ? std::max(1, p->num_ref_idx_l1) : 0;
    d.chroma_array_type = p->chroma_format_idc;
    d.transform_8x8_mode = p->transform_8x8_mode;
    d.direct_8x8_inference = 1;
    d.x264_build = -1;
    d.picture_id = i;
    d.coded = 1;
    d.payload_offset = p->seed * 0x100000001B3ull + (uint64_t)i;  // generator seed
    d.payload_size = (uint32_t)mbs;                               // generator: macroblocks to emit
    d.out_capacity = (uint32_t)std::min<uint64_t>((uint64_t)mbs * 384 + 4096, 0x7fffffffu);
    plan.descs.push_back(d);
  }
  plan.max_w = p->mb_width;
  plan.arena.assign(16, 0);
  std::vector<avr_slice_result> res;
  std::vector<uint8_t> outb;
  if (int r = run_plan(c, 2, false, plan, &res, &outb)) return r;
  std::vector<uint8_t> stream;
  avr::synth_write_parameter_sets(&stream, *p);
  for (int i = 0; i < n; i++) {
    if (res[i].status != 0) return fail(c, AVR_ERR_DEVICE, "generator failed on slice " + std::to_string(i));
    avr::synth_write_slice(&stream, *p, i, outb.data() + plan.descs[i].out_offset, res[i].out_len);
  }
  *out = (uint8_t*)malloc(stream.size());
  if (!*out) return AVR_ERR_OUT_OF_MEMORY;
  memcpy(*out, stream.data(), stream.size());
  *out_len = stream.size();
  return AVR_OK;
}

}  // extern "C"

// Debug only (not part of include/avrecode.h): section cycle counters (32 slots) of an AVR_PROFILE build of
// the parallel kernels (mode 0 compress, 1 decompress, 2 generate), read and cleared.
extern "C" int avr_debug_profile(int mode, unsigned long long* out16) {
  hipError_t e = mode == 0 ? avr::profile_parallel_compress(out16)
               : mode == 1 ? avr::profile_parallel_decompress(out16)
                           : avr::profile_parallel_generate(out16);
  return e == hipSuccess ? AVR_OK : AVR_ERR_DEVICE;
}
