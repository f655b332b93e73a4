// Host front end: demux, NAL/parameter-set/slice-header parsing, recode.proto wire codec.
// See avr_front.h.  ITU-T H.264 7.3.2.1.1 (SPS), 7.3.2.2 (PPS), 7.3.3 (slice header), D.2.7
// (user data SEI); FFmpeg 2.8 NAL unescaping and RBSP length rules (the fork's behaviour that
// decides init_decoder's (buf, size), recode.cpp:143).
#include "avr_front.h"

#include <algorithm>
#include <cstring>

namespace avr {

const char* const kParallelModelTag = "avrecode-amd:P64";     // parallel model, arithmetic_code<uint64_t, uint8_t>
const char* const kParallel32ModelTag = "avrecode-amd:P32";   // parallel model, P32 coder (avr_engine.h)
const char* const kChainedModelTag = "avrecode-amd:R16";      // reference model in chains of 16 coded slices

int model_of_version(const std::string& v) {
  if (v == kParallelModelTag) return 1;
  if (v == kParallel32ModelTag) return 2;
  if (v == kChainedModelTag) return 3;
  return v.rfind("avrecode-amd:", 0) == 0 ? -1 : 0;
}
const char* version_of_model(int model) {
  return model == 1 ? kParallelModelTag : model == 2 ? kParallel32ModelTag : model == 3 ? kChainedModelTag : nullptr;
}

namespace {

class Bits {
 public:
  Bits(const uint8_t* p, size_t n) : p_(p), nbits_(n * 8) {}
  uint32_t u1() {
    if (pos_ >= nbits_) {
      err_ = true;
      pos_++;
      return 0;
    }
    uint32_t v = (p_[pos_ >> 3] >> (7 - (pos_ & 7))) & 1;
    pos_++;
    return v;
  }
  uint32_t u(int n) {
    uint32_t v = 0;
    while (n--) v = (v << 1) | u1();
    return v;
  }
  uint32_t ue() {
    int lz = 0;
    while (!u1()) {
      if (++lz > 31 || err_) {
        err_ = true;
        return 0;
      }
    }
    return ((1u << lz) - 1) + u(lz);
  }
  int32_t se() {
    uint32_t k = ue();
    return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
  }
  bool more_rbsp(size_t len) const {
    while (len > 0 && p_[len - 1] == 0) len--;
    if (!len) return false;
    int tz = __builtin_ctz(p_[len - 1]);
    return pos_ < (len - 1) * 8 + (7 - tz);
  }
  size_t pos() const { return pos_; }
  bool err() const { return err_; }

 private:
  const uint8_t* p_;
  size_t nbits_, pos_ = 0;
  bool err_ = false;
};

void skip_scaling_list(Bits& b, int size) {
  int last = 8, next = 8;
  for (int j = 0; j < size; j++) {
    if (next) next = (last + b.se() + 256) % 256;
    last = next ? next : last;
  }
}

// Emulation prevention removed (7.4.1): every 00 00 03 drops its 03, scanning left to right (the
// byte after a dropped 03 starts the next match).  The 03 bytes are found by memchr and the runs
// between them copied whole: a multi-GB stream unescapes at memory speed, not byte by byte.
std::vector<uint8_t> unescape(const uint8_t* src, size_t n) {
  std::vector<uint8_t> out(n);
  size_t i = 0, o = 0;
  while (i < n) {
    // the first 00 00 03 at or after i: a 03 at p >= i + 2 with two zeros before it
    size_t j = n;
    for (size_t k = i + 2; k < n;) {
      const uint8_t* p = (const uint8_t*)memchr(src + k, 3, n - k);
      if (!p) break;
      const size_t q = (size_t)(p - src);
      if (src[q - 1] == 0 && src[q - 2] == 0) {
        j = q - 2;
        break;
      }
      k = q + 1;
    }
    const size_t run = (j < n ? j + 2 : n) - i;   // the bytes before the 03 (both zeros included)
    memcpy(out.data() + o, src + i, run);
    o += run;
    i = j < n ? j + 3 : n;
  }
  out.resize(o);
  return out;
}

// Does unescape() remove anything: is there a 00 00 03 in the n bytes at src?
bool has_epb(const uint8_t* src, size_t n) {
  for (size_t k = 2; k < n;) {
    const uint8_t* p = (const uint8_t*)memchr(src + k, 3, n - k);
    if (!p) return false;
    const size_t q = (size_t)(p - src);
    if (src[q - 1] == 0 && src[q - 2] == 0) return true;
    k = q + 1;
  }
  return false;
}

// FFmpeg 2.8 decode_nal_units: trailing zero bytes dropped, stop bit excluded.
size_t rbsp_bit_length(const uint8_t* rbsp, size_t n) {
  while (n > 0 && rbsp[n - 1] == 0) n--;
  if (!n) return 0;
  return 8 * n - (size_t)(__builtin_ctz(rbsp[n - 1]) + 1);
}

bool parse_sps(const uint8_t* r, size_t n, Sps* sps_table) {
  Bits b(r, n);
  Sps s;
  s.profile_idc = (int)b.u(8);
  b.u(16);
  uint32_t id = b.ue();
  if (id > 31) return false;
  const int p = s.profile_idc;
  if (p == 100 || p == 110 || p == 122 || p == 244 || p == 44 || p == 83 || p == 86 || p == 118 || p == 128 ||
      p == 138 || p == 139 || p == 134 || p == 135) {
    s.chroma_format_idc = (int)b.ue();
    if (s.chroma_format_idc == 3) s.separate_colour_plane = (int)b.u1();
    b.ue();
    b.ue();
    b.u1();
    if (b.u1())
      for (int i = 0; i < (s.chroma_format_idc != 3 ? 8 : 12); i++)
        if (b.u1()) skip_scaling_list(b, i < 6 ? 16 : 64);
  }
  // spec ranges (7.4.2.1.1): log2_max_frame_num_minus4, log2_max_pic_order_cnt_lsb_minus4 <= 12,
  // pic_order_cnt_type <= 2; anything else is a corrupt SPS (and would make u(n) loop)
  const uint32_t lfn = b.ue();
  if (lfn > 12) return false;
  s.log2_max_frame_num = 4 + (int)lfn;
  s.poc_type = (int)b.ue();
  if (s.poc_type > 2) return false;
  if (s.poc_type == 0) {
    const uint32_t lpoc = b.ue();
    if (lpoc > 12) return false;
    s.log2_max_poc_lsb = 4 + (int)lpoc;
  } else if (s.poc_type == 1) {
    s.delta_pic_order_always_zero = (int)b.u1();
    b.se();
    b.se();
    uint32_t k = b.ue();
    if (k > 255) return false;
    for (uint32_t i = 0; i < k && !b.err(); i++) b.se();
  }
  b.ue();
  b.u1();
  const uint32_t wm1 = b.ue(), hm1 = b.ue();
  if (wm1 >= 1024 || hm1 >= 1024) return false;
  s.mb_width = 1 + (int)wm1;
  int map_h = 1 + (int)hm1;
  s.frame_mbs_only = (int)b.u1();
  if (!s.frame_mbs_only) s.mb_aff = (int)b.u1();
  s.direct_8x8_inference = (int)b.u1();
  s.mb_height = (2 - s.frame_mbs_only) * map_h;
  // bound the picture (level 6.2 allows 139264 macroblocks per frame) so that mb_width * mb_height
  // and the device frame sizing (W * H * 52 bytes) cannot overflow
  if ((int64_t)s.mb_width * s.mb_height > 139264) return false;
  if (b.err()) return false;
  s.valid = true;
  sps_table[id] = s;
  return true;
}

bool parse_pps(const uint8_t* r, size_t n, const Sps* sps_table, Pps* pps_table) {
  Bits b(r, n);
  Pps q;
  uint32_t id = b.ue();
  if (id > 255) return false;
  q.sps_id = (int)b.ue();
  if (q.sps_id > 31) return false;
  q.entropy_coding_mode = (int)b.u1();
  q.bottom_field_pic_order_present = (int)b.u1();
  q.num_slice_groups = 1 + (int)b.ue();
  if (q.num_slice_groups > 1) {  // FMO: never CABAC; unusable here
    pps_table[id] = q;
    return true;
  }
  q.num_ref_idx_default[0] = 1 + (int)b.ue();
  q.num_ref_idx_default[1] = 1 + (int)b.ue();
  q.weighted_pred = (int)b.u1();
  q.weighted_bipred_idc = (int)b.u(2);
  q.pic_init_qp = 26 + b.se();
  b.se();
  b.se();
  q.deblocking_filter_control_present = (int)b.u1();
  b.u1();  // constrained_intra_pred_flag (CABAC parse unaffected without data partitioning)
  q.redundant_pic_cnt_present = (int)b.u1();
  if (b.more_rbsp(n)) {
    q.transform_8x8_mode = (int)b.u1();
    if (b.u1()) {
      const Sps& s = sps_table[q.sps_id];
      int cf = s.valid ? s.chroma_format_idc : 1;
      for (int i = 0; i < 6 + ((cf != 3) ? 2 : 6) * q.transform_8x8_mode; i++)
        if (b.u1()) skip_scaling_list(b, i < 6 ? 16 : 64);
    }
    b.se();
  }
  if (b.err()) return false;
  q.valid = true;
  pps_table[id] = q;
  return true;
}

int parse_x264_build(const uint8_t* r, size_t n) {
  size_t p = 0;
  while (p + 2 <= n) {
    int type = 0, size = 0;
    while (p < n && r[p] == 0xff) type += 255, p++;
    if (p >= n) break;
    type += r[p++];
    while (p < n && r[p] == 0xff) size += 255, p++;
    if (p >= n) break;
    size += r[p++];
    if (p + (size_t)size > n) break;
    static const char tag[] = "x264 - core ";
    if (type == 5 && size > 16 + (int)sizeof(tag) - 1 && !memcmp(r + p + 16, tag, sizeof(tag) - 1)) {
      int build = 0, digits = 0;
      for (size_t k = p + 16 + sizeof(tag) - 1; k < p + size && r[k] >= '0' && r[k] <= '9'; k++, digits++)
        build = build * 10 + (r[k] - '0');
      if (digits && build > 0) return build;
    }
    p += (size_t)size;
  }
  return -1;
}

bool parse_slice_header(const Sps* sps_table, const Pps* pps_table, const uint8_t* r, size_t n, int type,
                        int ref_idc, SliceHeader* h) {
  Bits b(r, n);
  *h = SliceHeader();
  h->nal_unit_type = type;
  h->nal_ref_idc = ref_idc;
  h->first_mb = (int)b.ue();
  int st = (int)b.ue();
  if (st > 9) return false;
  h->slice_type = st % 5;
  h->pps_id = (int)b.ue();
  if (h->pps_id > 255 || !pps_table[h->pps_id].valid) return false;
  const Pps& pps = pps_table[h->pps_id];
  const Sps& sps = sps_table[pps.sps_id];
  if (!sps.valid) return false;
  h->entropy_coding_mode = pps.entropy_coding_mode;
  if (sps.separate_colour_plane) b.u(2);
  h->frame_num = (int)b.u(sps.log2_max_frame_num);
  if (!sps.frame_mbs_only) {
    h->field_pic = (int)b.u1();
    if (h->field_pic) h->bottom_field = (int)b.u1();
  }
  h->mbaff = sps.mb_aff && !h->field_pic;
  // first_mb_in_slice counts macroblock pairs in an MBAFF frame (7.4.3)
  if (h->mbaff) h->first_mb *= 2;
  if (type == 5) h->idr_pic_id = (int)b.ue();
  if (sps.poc_type == 0) {
    h->poc_lsb = (int)b.u(sps.log2_max_poc_lsb);
    if (pps.bottom_field_pic_order_present && !h->field_pic) b.se();
  }
  if (sps.poc_type == 1 && !sps.delta_pic_order_always_zero) {
    b.se();
    if (pps.bottom_field_pic_order_present && !h->field_pic) b.se();
  }
  if (pps.redundant_pic_cnt_present) b.ue();
  const bool is_p = h->slice_type == 0 || h->slice_type == 3, is_b = h->slice_type == 1;
  const bool is_i = h->slice_type == 2 || h->slice_type == 4;
  if (is_b) b.u1();
  h->num_ref_idx[0] = pps.num_ref_idx_default[0];
  h->num_ref_idx[1] = pps.num_ref_idx_default[1];
  if ((is_p || is_b) && b.u1()) {
    h->num_ref_idx[0] = 1 + (int)b.ue();
    if (is_b) h->num_ref_idx[1] = 1 + (int)b.ue();
  }
  if (!is_b) h->num_ref_idx[1] = 0;
  if (is_i) h->num_ref_idx[0] = 0;
  if (!is_i) {
    for (int l = 0; l < (is_b ? 2 : 1); l++)
      if (b.u1())
        for (int guard = 0; guard < 1000 && !b.err(); guard++) {
          uint32_t idc = b.ue();
          if (idc == 3) break;
          if (idc > 5) return false;
          b.ue();
        }
  }
  const int cat = sps.separate_colour_plane ? 0 : sps.chroma_format_idc;
  if ((pps.weighted_pred && is_p) || (pps.weighted_bipred_idc == 1 && is_b)) {
    b.ue();
    if (cat) b.ue();
    for (int l = 0; l < (is_b ? 2 : 1); l++)
      for (int i = 0; i < h->num_ref_idx[l] && !b.err(); i++) {
        if (b.u1()) b.se(), b.se();
        if (cat && b.u1()) b.se(), b.se(), b.se(), b.se();
      }
  }
  if (ref_idc) {
    if (type == 5) {
      b.u1();
      b.u1();
    } else if (b.u1()) {
      for (int guard = 0; guard < 1000 && !b.err(); guard++) {
        uint32_t op = b.ue();
        if (!op) break;
        if (op > 6) return false;
        if (op == 1 || op == 3) b.ue();
        if (op == 2) b.ue();
        if (op == 3 || op == 6) b.ue();
        if (op == 4) b.ue();
      }
    }
  }
  h->cabac_init_idc = (pps.entropy_coding_mode && !is_i) ? (int)b.ue() : -1;
  h->slice_qp = pps.pic_init_qp + b.se();
  if (h->slice_type == 3 || h->slice_type == 4) {
    if (h->slice_type == 3) b.u1();
    b.se();
  }
  if (pps.deblocking_filter_control_present && b.ue() != 1) b.se(), b.se();
  if (b.err()) return false;
  h->cabac_start = (b.pos() + 7) / 8;
  h->chroma_array_type = cat;
  h->transform_8x8_mode = pps.transform_8x8_mode;
  h->direct_8x8_inference = sps.direct_8x8_inference;
  h->mb_width = sps.mb_width;
  h->mb_height = sps.mb_height;
  // macroblocks in this picture: a field has half the frame's rows
  const int pic_mbs = sps.mb_width * (h->field_pic ? sps.mb_height / 2 : sps.mb_height);
  h->supported = pps.entropy_coding_mode && !sps.separate_colour_plane &&
                 (is_p || is_b || h->slice_type == 2) && h->cabac_init_idc <= 2 &&
                 h->first_mb < pic_mbs && h->num_ref_idx[0] <= 32 && h->num_ref_idx[1] <= 32 &&
                 sps.mb_width <= 1024;
  return true;
}

uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) << 32 | rd32(p + 4); }
constexpr uint32_t fourcc(const char* s) { return (uint32_t)s[0] << 24 | (uint32_t)s[1] << 16 | (uint32_t)s[2] << 8 | s[3]; }

struct Box {
  uint32_t type;
  size_t body, end;
};
bool read_box(const uint8_t* f, size_t off, size_t lim, Box* b) {
  if (off + 8 > lim) return false;
  uint64_t sz = rd32(f + off);
  b->type = rd32(f + off + 4);
  size_t hdr = 8;
  if (sz == 1) {
    if (off + 16 > lim) return false;
    sz = rd64(f + off + 8);
    hdr = 16;
  } else if (sz == 0) {
    sz = lim - off;
  }
  // sz > lim - off, not off + sz > lim: a 64-bit size must not wrap the end below the body
  if (sz < hdr || off >= lim || sz > (uint64_t)(lim - off)) return false;
  b->body = off + hdr;
  b->end = off + (size_t)sz;
  return true;
}

struct Track {
  bool video = false;
  size_t avcc = 0, avcc_len = 0;
  size_t stsz = 0, stsz_len = 0, stco = 0, stco_len = 0, stsc = 0, stsc_len = 0;
  bool co64 = false;
};

void walk_track(const uint8_t* f, size_t off, size_t lim, Track* t, int depth) {
  Box b;
  while (read_box(f, off, lim, &b)) {
    if (b.type == fourcc("mdia") || b.type == fourcc("minf") || b.type == fourcc("stbl")) {
      if (depth < 8) walk_track(f, b.body, b.end, t, depth + 1);
    } else if (b.type == fourcc("hdlr")) {
      if (b.end - b.body >= 12 && rd32(f + b.body + 8) == fourcc("vide")) t->video = true;
    } else if (b.type == fourcc("stsd")) {
      size_t p = b.body + 8;
      Box e;
      if (read_box(f, p, b.end, &e) && (e.type == fourcc("avc1") || e.type == fourcc("avc3"))) {
        size_t c = e.body + 78;
        Box cb;
        while (read_box(f, c, e.end, &cb)) {
          if (cb.type == fourcc("avcC")) {
            t->avcc = cb.body;
            t->avcc_len = cb.end - cb.body;
          }
          c = cb.end;
        }
      }
    } else if (b.type == fourcc("stsz")) {
      t->stsz = b.body, t->stsz_len = b.end - b.body;
    } else if (b.type == fourcc("stco") || b.type == fourcc("co64")) {
      t->stco = b.body, t->stco_len = b.end - b.body, t->co64 = b.type == fourcc("co64");
    } else if (b.type == fourcc("stsc")) {
      t->stsc = b.body, t->stsc_len = b.end - b.body;
    }
    off = b.end;
  }
}

}  // namespace

int mp4_layout(const uint8_t* f, size_t n, Mp4Layout* L) {
  *L = Mp4Layout();
  Track video;
  bool found = false, moov = false;
  Box b;
  for (size_t off = 0; read_box(f, off, n, &b); off = b.end) {
    if (b.type != fourcc("moov")) continue;
    moov = true;
    Box tb;
    for (size_t c = b.body; read_box(f, c, b.end, &tb); c = tb.end) {
      if (tb.type != fourcc("trak")) continue;
      Track t;
      walk_track(f, tb.body, tb.end, &t, 0);
      if (t.video && t.avcc && !found) video = t, found = true;
    }
  }
  if (!moov) return 0;   // not within [0, n) (yet)
  if (!found || !video.stsz || !video.stco || !video.stsc || video.avcc_len < 7) return -1;
  const uint8_t* a = f + video.avcc;
  L->len_size = (a[4] & 3) + 1;
  size_t p = 5;
  for (int pass = 0; pass < 2; pass++) {
    if (p >= video.avcc_len) break;
    int cnt = pass == 0 ? (a[p++] & 31) : a[p++];
    for (int i = 0; i < cnt && p + 2 <= video.avcc_len; i++) {
      size_t l = (size_t)a[p] << 8 | a[p + 1];
      p += 2;
      if (p + l > video.avcc_len) return -1;
      L->param_sets.push_back({video.avcc + p, l});
      p += l;
    }
  }
  if (video.stsz_len < 12 || video.stco_len < 8 || video.stsc_len < 8) return -1;
  const uint8_t *stsz = f + video.stsz, *stco = f + video.stco, *stsc = f + video.stsc;
  const uint32_t fixed = rd32(stsz + 4), nsamples = rd32(stsz + 8), nchunks = rd32(stco + 4), nstsc = rd32(stsc + 4);
  if (!fixed && 12 + 4ull * nsamples > video.stsz_len) return -1;
  if (8 + (video.co64 ? 8ull : 4ull) * nchunks > video.stco_len || 8 + 12ull * nstsc > video.stsc_len) return -1;
  uint32_t sample = 0;
  for (uint32_t e = 0; e < nstsc && sample < nsamples; e++) {
    const uint32_t first = rd32(stsc + 8 + 12 * e), per = rd32(stsc + 12 + 12 * e);
    const uint32_t next_first = e + 1 < nstsc ? rd32(stsc + 8 + 12 * (e + 1)) : nchunks + 1;
    // chunk numbers are 1-based and increase from entry to entry (ISO/IEC 14496-12 8.7.4)
    if (first == 0 || next_first <= first) return -1;
    const uint32_t last = next_first - 1;
    for (uint32_t c = first; c <= last && c <= nchunks && sample < nsamples; c++) {
      size_t coff = video.co64 ? (size_t)rd64(stco + 8 + 8 * (c - 1)) : rd32(stco + 8 + 4 * (c - 1));
      for (uint32_t s = 0; s < per && sample < nsamples; s++, sample++) {
        size_t ssz = fixed ? fixed : rd32(stsz + 12 + 4 * sample);
        if (coff > SIZE_MAX / 2 || ssz > SIZE_MAX / 2) return -1;
        L->samples.push_back({coff, ssz});
        coff += ssz;
      }
    }
  }
  return 1;
}

void mp4_sample_nals(const uint8_t* f, const NalRef& smp, int len_size, std::vector<NalRef>* nals) {
  for (size_t q = smp.offset, qe = smp.offset + smp.size; q + (size_t)len_size <= qe;) {
    size_t l = 0;
    for (int k = 0; k < len_size; k++) l = l << 8 | f[q + k];
    q += (size_t)len_size;
    if (!l || q + l > qe) break;
    nals->push_back({q, l});
    q += l;
  }
}

namespace {

bool demux_mp4(const uint8_t* f, size_t n, std::vector<NalRef>* nals) {
  Mp4Layout L;
  if (mp4_layout(f, n, &L) != 1) return false;
  *nals = L.param_sets;
  for (const NalRef& smp : L.samples) {
    if (smp.offset > n || smp.size > n - smp.offset) return false;
    mp4_sample_nals(f, smp, L.len_size, nals);
  }
  return true;
}

// The first j >= k with f[j] = f[j + 1] = 0 and f[j + 2] = 1 (or 0 too, with zero3), j + 3 <= n; n
// when there is none.  memchr finds the zeros: start codes are found at memory speed.
size_t scan_start(const uint8_t* f, size_t n, size_t k, bool zero3) {
  while (k + 3 <= n) {
    const uint8_t* p = (const uint8_t*)memchr(f + k, 0, n - 2 - k);
    if (!p) return n;
    const size_t j = (size_t)(p - f);
    if (f[j + 1] == 0 && (f[j + 2] == 1 || (zero3 && f[j + 2] == 0))) return j;
    k = j + 1;
  }
  return n;
}

// scan_start over f with skip ranges: the same answer, without reading the ranges (a start code
// needs a 0x00 at j and j + 1 and a 0x00 / 0x01 at j + 2, and the ranges hold none of those --
// the surrogate fill is 'X', its marker stays outside the range).  *r: the first range not yet
// passed (scans only move forward).
size_t scan_start_skip(const uint8_t* f, size_t n, size_t k, bool zero3, const SkipRanges& sk, size_t* r) {
  while (k + 3 <= n) {
    while (*r < sk.size() && sk[*r].second <= k) ++*r;
    if (*r < sk.size() && sk[*r].first <= k) {   // inside a range: continue at its end
      k = sk[*r].second;
      continue;
    }
    const size_t lim = *r < sk.size() ? std::min(n, sk[*r].first + 2) : n;   // a code may end 2 bytes in
    const size_t j = scan_start(f, lim, k, zero3);
    if (j < lim) return j;
    if (lim == n) return n;
    k = std::max(k, lim - 2);
    if (*r < sk.size() && k < sk[*r].second) k = sk[*r].second;
  }
  return n;
}

void demux_annexb(const uint8_t* f, size_t n, std::vector<NalRef>* nals, const SkipRanges* skips) {
  size_t r = 0;
  auto scan = [&](size_t k, bool zero3) {
    return skips ? scan_start_skip(f, n, k, zero3, *skips, &r) : scan_start(f, n, k, zero3);
  };
  size_t i = scan(0, false);
  while (i + 3 <= n) {
    const size_t start = i + 3, j = scan(start, true);
    size_t end = j + 3 <= n ? j : n;
    while (end > start && f[end - 1] == 0) end--;
    if (end > start) nals->push_back({start, end - start});
    i = scan(j, false);
  }
}

}  // namespace

bool is_mp4(const uint8_t* file, size_t n) {
  return n >= 8 && (rd32(file + 4) == fourcc("ftyp") || rd32(file + 4) == fourcc("moov") ||
                    rd32(file + 4) == fourcc("mdat") || rd32(file + 4) == fourcc("free"));
}

bool demux(const uint8_t* file, size_t n, std::vector<NalRef>* nals, const SkipRanges* skips) {
  nals->clear();
  if (is_mp4(file, n)) return demux_mp4(file, n, nals) && !nals->empty();
  demux_annexb(file, n, nals, skips);
  return !nals->empty();   // nothing H.264 in it: av_decoder::run throws (recode.cpp:92-93)
}

// has_epb over the NAL's bytes outside the skip ranges: exact, since a 00 00 03 cannot touch a
// range's bytes (neither 0x00 nor 0x03 occurs in them)
bool StreamParser::nal_has_epb(const uint8_t* src, size_t n) const {
  if (!skips_ || src < skip_base_) return has_epb(src, n);
  const size_t a = (size_t)(src - skip_base_), b = a + n;
  const SkipRanges& sk = *skips_;
  size_t r = (size_t)(std::upper_bound(sk.begin(), sk.end(), std::make_pair(a, ~(size_t)0)) - sk.begin());
  if (r > 0 && sk[r - 1].second > a) r--;   // a range that starts before the NAL and reaches into it
  size_t k = a;
  for (; r < sk.size() && sk[r].first < b; r++) {
    if (sk[r].first > k && has_epb(skip_base_ + k, sk[r].first - k)) return true;
    k = std::max(k, sk[r].second);
  }
  return k < b && has_epb(skip_base_ + k, b - k);
}

bool StreamParser::next(const uint8_t* nal, size_t n, SliceInfo* s, bool views) {
  if (n < 2) return false;
  const int type = nal[0] & 0x1f, ref_idc = (nal[0] >> 5) & 3;
  if (type != 1 && type != 5 && type != 6 && type != 7 && type != 8) return false;
  // a slice NAL without emulation-prevention bytes is its own RBSP: no copy when views are allowed
  const bool view = views && (type == 1 || type == 5) && !nal_has_epb(nal + 1, n - 1);
  std::vector<uint8_t> rbsp = view ? std::vector<uint8_t>() : unescape(nal + 1, n - 1);
  const uint8_t* rd = view ? nal + 1 : rbsp.data();
  const size_t rn = view ? n - 1 : rbsp.size();
  if (type == 6) {
    int b = parse_x264_build(rbsp.data(), rbsp.size());
    if (b > 0) x264_build_ = b;
    return false;
  }
  if (type == 7) {
    parse_sps(rbsp.data(), rbsp.size(), sps_);
    return false;
  }
  if (type == 8) {
    parse_pps(rbsp.data(), rbsp.size(), sps_, pps_);
    return false;
  }
  SliceHeader h;
  if (!parse_slice_header(sps_, pps_, rd, rn, type, ref_idc, &h) || !h.entropy_coding_mode)
    return false;
  h.x264_build = x264_build_;
  const SliceHeader& p = prev_;
  const bool new_pic = !have_prev_ || h.first_mb == 0 || h.first_mb <= p.first_mb || h.frame_num != p.frame_num ||
                       h.pps_id != p.pps_id || h.poc_lsb != p.poc_lsb ||
                       (h.nal_unit_type == 5) != (p.nal_unit_type == 5) || h.idr_pic_id != p.idr_pic_id ||
                       (h.nal_ref_idc == 0) != (p.nal_ref_idc == 0) || h.field_pic != p.field_pic ||
                       h.bottom_field != p.bottom_field;
  // picture_id stands in for the frame_num the fork hands frame_spec: the second
  // field of a field pair shares its frame_num with the first, so it keeps the first's id and the
  // model keeps filling the same frame (the fields interleave in its frame-sized buffer)
  const bool second_field = new_pic && have_prev_ && h.field_pic && p.field_pic && h.frame_num == p.frame_num &&
                            h.bottom_field != p.bottom_field && !second_field_;
  if (new_pic && !second_field) picture_id_++;
  if (new_pic) second_field_ = second_field;
  prev_ = h;
  have_prev_ = true;
  s->h = h;
  s->picture_id = picture_id_;
  const size_t bits = rbsp_bit_length(rd, rn);
  const size_t end = (bits + 7) / 8;
  s->size = end > h.cabac_start ? end - h.cabac_start : 0;
  s->read_limit = rn > h.cabac_start + s->size ? s->size + 1 : s->size;
  s->verbatim = rn == n - 1;
  if (view) {
    s->view = rd;
    s->view_len = rn;
  } else {
    s->rbsp = std::move(rbsp);
  }
  return true;
}

// ----------------------------------------------------------------------------- protobuf
namespace {
void varint(std::vector<uint8_t>* o, uint64_t v) {
  while (v >= 0x80) {
    o->push_back((uint8_t)(v | 0x80));
    v >>= 7;
  }
  o->push_back((uint8_t)v);
}
void bytes_field(std::vector<uint8_t>* o, int field, const uint8_t* p, size_t n) {
  varint(o, (uint64_t)field << 3 | 2);
  varint(o, n);
  o->insert(o->end(), p, p + n);
}
bool rd_varint(const uint8_t** p, const uint8_t* e, uint64_t* v) {
  *v = 0;
  for (int s = 0; s < 64; s += 7) {
    if (*p >= e) return false;
    uint8_t c = *(*p)++;
    *v |= (uint64_t)(c & 0x7f) << s;
    if (!(c & 0x80)) return true;
  }
  return false;
}
bool skip_field(const uint8_t** p, const uint8_t* e, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return rd_varint(p, e, &v);
    case 1: if (e - *p < 8) return false; *p += 8; return true;
    case 2: if (!rd_varint(p, e, &v) || (uint64_t)(e - *p) < v) return false; *p += v; return true;
    case 5: if (e - *p < 4) return false; *p += 4; return true;
    default: return false;
  }
}
}  // namespace

void pb_put_block(std::vector<uint8_t>* o, const PbBlock& b) {
  std::vector<uint8_t> m;
  if (b.has_size) varint(&m, 1 << 3), varint(&m, (uint64_t)b.size);
  if (b.has_literal) bytes_field(&m, 2, b.literal, b.literal_len);
  if (b.has_skip) varint(&m, 3 << 3), varint(&m, b.skip_coded ? 1 : 0);
  if (b.has_cabac) bytes_field(&m, 4, b.cabac, b.cabac_len);
  if (b.has_parity) varint(&m, 5 << 3), varint(&m, b.length_parity ? 1 : 0);
  if (b.has_last_byte) bytes_field(&m, 6, (const uint8_t*)b.last_byte.data(), b.last_byte.size());
  if (b.has_seams) bytes_field(&m, 16, b.seams, b.seams_len);
  bytes_field(o, 2, m.data(), m.size());
}

namespace {
size_t varint_size(uint64_t v) {
  size_t k = 1;
  while (v >= 0x80) v >>= 7, k++;
  return k;
}
size_t bytes_field_size(int field, size_t n) { return varint_size((uint64_t)field << 3 | 2) + varint_size(n) + n; }
size_t block_inner_size(const PbBlock& b) {
  size_t m = 0;
  if (b.has_size) m += varint_size(1 << 3) + varint_size((uint64_t)b.size);
  if (b.has_literal) m += bytes_field_size(2, b.literal_len);
  if (b.has_skip) m += varint_size(3 << 3) + 1;
  if (b.has_cabac) m += bytes_field_size(4, b.cabac_len);
  if (b.has_parity) m += varint_size(5 << 3) + 1;
  if (b.has_last_byte) m += bytes_field_size(6, b.last_byte.size());
  if (b.has_seams) m += bytes_field_size(16, b.seams_len);
  return m;
}
size_t put_varint(uint8_t* o, size_t at, uint64_t v) {
  while (v >= 0x80) {
    o[at++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  o[at++] = (uint8_t)v;
  return at;
}
size_t put_bytes(uint8_t* o, size_t at, int field, const uint8_t* p, size_t n, std::vector<PbCopy>* copies) {
  at = put_varint(o, at, (uint64_t)field << 3 | 2);
  at = put_varint(o, at, n);
  if (copies && n) copies->push_back({at, p, n});
  else if (n) memcpy(o + at, p, n);
  return at + n;
}
}  // namespace

size_t pb_block_size(const PbBlock& b) { return bytes_field_size(2, block_inner_size(b)); }

// pb_put_block's bytes, field for field
size_t pb_write_block(uint8_t* o, size_t at, const PbBlock& b, std::vector<PbCopy>* copies) {
  at = put_varint(o, at, 2 << 3 | 2);
  at = put_varint(o, at, block_inner_size(b));
  if (b.has_size) at = put_varint(o, at, 1 << 3), at = put_varint(o, at, (uint64_t)b.size);
  if (b.has_literal) at = put_bytes(o, at, 2, b.literal, b.literal_len, copies);
  if (b.has_skip) at = put_varint(o, at, 3 << 3), at = put_varint(o, at, b.skip_coded ? 1 : 0);
  if (b.has_cabac) at = put_bytes(o, at, 4, b.cabac, b.cabac_len, copies);
  if (b.has_parity) at = put_varint(o, at, 5 << 3), at = put_varint(o, at, b.length_parity ? 1 : 0);
  if (b.has_last_byte) at = put_bytes(o, at, 6, (const uint8_t*)b.last_byte.data(), b.last_byte.size(), nullptr);
  if (b.has_seams) at = put_bytes(o, at, 16, b.seams, b.seams_len, copies);
  return at;
}

void pb_put_metadata_version(std::vector<uint8_t>* o, const std::string& version) {
  std::vector<uint8_t> m;
  bytes_field(&m, 1, (const uint8_t*)version.data(), version.size());
  bytes_field(o, 1, m.data(), m.size());
}

bool pb_read_version(const uint8_t* in, size_t n, std::string* version) {
  version->clear();
  const uint8_t *p = in, *e = in + n;
  while (p < e) {
    uint64_t tag, len;
    if (!rd_varint(&p, e, &tag)) return false;
    if ((tag & 7) != 2 || (tag >> 3) != 1) {
      if (!skip_field(&p, e, (int)(tag & 7))) return false;
      continue;
    }
    if (!rd_varint(&p, e, &len) || (uint64_t)(e - p) < len) return false;
    const uint8_t *q = p, *qe = p + len;
    p += len;
    while (q < qe) {
      uint64_t t2, l2;
      if (!rd_varint(&q, qe, &t2)) return false;
      if ((t2 & 7) != 2) {
        if (!skip_field(&q, qe, (int)(t2 & 7))) return false;
        continue;
      }
      if (!rd_varint(&q, qe, &l2) || (uint64_t)(qe - q) < l2) return false;
      if ((t2 >> 3) == 1) version->assign((const char*)q, l2);
      q += l2;
    }
  }
  return true;
}

bool pb_parse(const uint8_t* in, size_t n, std::vector<PbBlock>* blocks, std::string* version, bool* has_metadata) {
  blocks->clear();
  version->clear();
  if (has_metadata) *has_metadata = false;
  const uint8_t *p = in, *e = in + n;
  while (p < e) {
    uint64_t tag, len;
    if (!rd_varint(&p, e, &tag)) return false;
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if (wt != 2 || (field != 1 && field != 2)) {
      if (!skip_field(&p, e, wt)) return false;
      continue;
    }
    if (!rd_varint(&p, e, &len) || (uint64_t)(e - p) < len) return false;
    const uint8_t *q = p, *qe = p + len;
    p += len;
    if (field == 1) {  // Metadata
      if (has_metadata) *has_metadata = true;
      while (q < qe) {
        uint64_t t2, l2;
        if (!rd_varint(&q, qe, &t2)) return false;
        if ((t2 & 7) != 2) {
          if (!skip_field(&q, qe, (int)(t2 & 7))) return false;
          continue;
        }
        if (!rd_varint(&q, qe, &l2) || (uint64_t)(qe - q) < l2) return false;
        if ((t2 >> 3) == 1) version->assign((const char*)q, l2);
        q += l2;
      }
      continue;
    }
    PbBlock b;
    while (q < qe) {
      uint64_t t2, v;
      if (!rd_varint(&q, qe, &t2)) return false;
      const int f2 = (int)(t2 >> 3), w2 = (int)(t2 & 7);
      if (w2 == 0 && (f2 == 1 || f2 == 3 || f2 == 5)) {
        if (!rd_varint(&q, qe, &v)) return false;
        if (f2 == 1) b.has_size = true, b.size = (int64_t)v;
        if (f2 == 3) b.has_skip = true, b.skip_coded = v != 0;
        if (f2 == 5) b.has_parity = true, b.length_parity = v != 0;
      } else if (w2 == 2 && (f2 == 2 || f2 == 4 || f2 == 6 || f2 == 16)) {
        if (!rd_varint(&q, qe, &v) || (uint64_t)(qe - q) < v) return false;
        if (f2 == 2) b.has_literal = true, b.literal = q, b.literal_len = v;
        if (f2 == 4) b.has_cabac = true, b.cabac = q, b.cabac_len = v;
        if (f2 == 6) b.has_last_byte = true, b.last_byte.assign((const char*)q, v);
        if (f2 == 16) b.has_seams = true, b.seams = q, b.seams_len = v;
        q += v;
      } else if (!skip_field(&q, qe, w2)) {
        return false;
      }
    }
    blocks->push_back(b);
  }
  return true;
}

void surrogate_marker(uint64_t seq, uint8_t out[8]) {  // next_surrogate_marker (recode.cpp:1527-1535)
  for (int i = 0; i < kSurrogateMarkerBytes; i++) {
    out[i] = (uint8_t)(seq % 255 + 1);
    seq /= 255;
  }
}

}  // namespace avr
