/*
 * Oracle: H.264 front end.  TEST INFRASTRUCTURE ONLY (see avr_oracle.h).
 *
 * Restates what the reference obtains from FFmpeg (recode.cpp:73-135 av_decoder: avformat demux +
 * h264 NAL/parameter-set/slice-header parsing in the libavcodec-hooks fork):
 *   - MP4 (ISO BMFF, avc1/avcC length-prefixed samples) and Annex-B start-code demux,
 *   - NAL unescaping (FFmpeg 2.8 ff_h264_decode_nal) and the RBSP bit-length rule that decides
 *     the (buf,size) FFmpeg hands to init_decoder (recode.cpp:143, 1136),
 *   - SPS / PPS / slice header per ITU-T H.264 7.3.2.1.1, 7.3.2.2, 7.3.3.
 */
#include <stdlib.h>
#include <string.h>

#include "avr_oracle.h"

/* ------------------------------------------------------------------------------ bit reader */
typedef struct {
  const uint8_t *p;
  size_t nbits, pos;
  int err;
} br_t;
static void br_init(br_t *b, const uint8_t *p, size_t n) { b->p = p; b->nbits = n * 8; b->pos = 0; b->err = 0; }
static uint32_t br_u1(br_t *b) {
  if (b->pos >= b->nbits) { b->err = 1; b->pos++; return 0; }
  uint32_t v = (b->p[b->pos >> 3] >> (7 - (b->pos & 7))) & 1;
  b->pos++;
  return v;
}
static uint32_t br_u(br_t *b, int n) {
  uint32_t v = 0;
  for (int i = 0; i < n; i++) v = (v << 1) | br_u1(b);
  return v;
}
static uint32_t br_ue(br_t *b) {
  int lz = 0;
  while (!br_u1(b)) {
    if (++lz > 31 || b->err) { b->err = 1; return 0; }
  }
  return ((1u << lz) - 1) + br_u(b, lz);
}
static int32_t br_se(br_t *b) {
  uint32_t k = br_ue(b);
  return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
}
/* more_rbsp_data(): true if there is a 1 bit after pos other than the final stop bit */
static int br_more_rbsp(const br_t *b, size_t rbsp_len) {
  size_t n = rbsp_len;
  while (n > 0 && b->p[n - 1] == 0) n--;
  if (n == 0) return 0;
  uint8_t last = b->p[n - 1];
  int tz = 0;
  while (!(last & (1 << tz))) tz++;
  size_t stop = (n - 1) * 8 + (7 - tz);
  return b->pos < stop;
}

/* ----------------------------------------------------------------------------------- NALs */
size_t avr_nal_unescape(const uint8_t *src, size_t n, uint8_t *dst) {
  size_t si = 0, di = 0;
  while (si < n) {
    if (si + 2 < n && src[si] == 0 && src[si + 1] == 0 && src[si + 2] == 3) {
      dst[di++] = 0;
      dst[di++] = 0;
      si += 3;
      continue;
    }
    dst[di++] = src[si++];
  }
  return di;
}

/* FFmpeg 2.8 h264.c decode_nal_units: strip trailing zero bytes, then
 * bit_length = 8*len - decode_rbsp_trailing(last byte) (stop bit and the zeros after it) */
size_t avr_rbsp_bit_length(const uint8_t *rbsp, size_t n) {
  while (n > 0 && rbsp[n - 1] == 0) n--;
  if (n == 0) return 0;
  uint8_t v = rbsp[n - 1];
  int r;
  for (r = 1; r < 9; r++) {
    if (v & 1) break;
    v >>= 1;
  }
  return 8 * n - (size_t)r;
}

/* ------------------------------------------------------------------------------ SPS/PPS */
static void skip_scaling_list(br_t *b, int size) {
  int last = 8, next = 8;
  for (int j = 0; j < size; j++) {
    if (next != 0) {
      int delta = br_se(b);
      next = (last + delta + 256) % 256;
    }
    last = next == 0 ? last : next;
  }
}

int avr_parse_sps(avr_param_sets_t *ps, const uint8_t *rbsp, size_t n) {
  br_t b;
  br_init(&b, rbsp, n);
  avr_sps_t s;
  memset(&s, 0, sizeof(s));
  s.profile_idc = (int)br_u(&b, 8);
  br_u(&b, 8); /* constraint flags */
  br_u(&b, 8); /* level */
  uint32_t id = br_ue(&b);
  if (id > 31) return -1;
  s.chroma_format_idc = 1;
  s.bit_depth_luma = s.bit_depth_chroma = 8;
  int p = s.profile_idc;
  if (p == 100 || p == 110 || p == 122 || p == 244 || p == 44 || p == 83 || p == 86 || p == 118 ||
      p == 128 || p == 138 || p == 139 || p == 134 || p == 135) {
    s.chroma_format_idc = (int)br_ue(&b);
    if (s.chroma_format_idc == 3) s.separate_colour_plane = (int)br_u1(&b);
    s.bit_depth_luma = 8 + (int)br_ue(&b);
    s.bit_depth_chroma = 8 + (int)br_ue(&b);
    br_u1(&b); /* qpprime_y_zero_transform_bypass_flag */
    if (br_u1(&b)) {
      int cnt = s.chroma_format_idc != 3 ? 8 : 12;
      for (int i = 0; i < cnt; i++)
        if (br_u1(&b)) skip_scaling_list(&b, i < 6 ? 16 : 64);
    }
  }
  s.log2_max_frame_num = 4 + (int)br_ue(&b);
  s.poc_type = (int)br_ue(&b);
  if (s.poc_type == 0) {
    s.log2_max_poc_lsb = 4 + (int)br_ue(&b);
  } else if (s.poc_type == 1) {
    s.delta_pic_order_always_zero = (int)br_u1(&b);
    br_se(&b);
    br_se(&b);
    uint32_t k = br_ue(&b);
    for (uint32_t i = 0; i < k && !b.err; i++) br_se(&b);
  }
  br_ue(&b); /* max_num_ref_frames */
  br_u1(&b); /* gaps_in_frame_num_value_allowed_flag */
  s.mb_width = 1 + (int)br_ue(&b);
  int map_units_h = 1 + (int)br_ue(&b);
  s.frame_mbs_only = (int)br_u1(&b);
  if (!s.frame_mbs_only) s.mb_aff = (int)br_u1(&b);
  s.direct_8x8_inference = (int)br_u1(&b);
  s.mb_height = (2 - s.frame_mbs_only) * map_units_h;
  if (b.err) return -1;
  s.valid = 1;
  ps->sps[id] = s;
  return (int)id;
}

int avr_parse_pps(avr_param_sets_t *ps, const uint8_t *rbsp, size_t n) {
  br_t b;
  br_init(&b, rbsp, n);
  avr_pps_t q;
  memset(&q, 0, sizeof(q));
  uint32_t id = br_ue(&b);
  if (id > 255) return -1;
  q.sps_id = (int)br_ue(&b);
  if (q.sps_id > 31) return -1;
  q.entropy_coding_mode = (int)br_u1(&b);
  q.bottom_field_pic_order_present = (int)br_u1(&b);
  q.num_slice_groups = 1 + (int)br_ue(&b);
  if (q.num_slice_groups > 1) {
    /* FMO is Baseline/Extended only (never CABAC); stop parsing, mark the PPS unusable */
    q.valid = 0;
    ps->pps[id] = q;
    return (int)id;
  }
  q.num_ref_idx_default[0] = 1 + (int)br_ue(&b);
  q.num_ref_idx_default[1] = 1 + (int)br_ue(&b);
  q.weighted_pred = (int)br_u1(&b);
  q.weighted_bipred_idc = (int)br_u(&b, 2);
  q.pic_init_qp = 26 + br_se(&b);
  br_se(&b); /* pic_init_qs */
  br_se(&b); /* chroma_qp_index_offset */
  q.deblocking_filter_control_present = (int)br_u1(&b);
  q.constrained_intra_pred = (int)br_u1(&b);
  q.redundant_pic_cnt_present = (int)br_u1(&b);
  if (br_more_rbsp(&b, n)) {
    q.transform_8x8_mode = (int)br_u1(&b);
    if (br_u1(&b)) {
      const avr_sps_t *s = &ps->sps[q.sps_id];
      int cf = s->valid ? s->chroma_format_idc : 1;
      int cnt = 6 + ((cf != 3) ? 2 : 6) * q.transform_8x8_mode;
      for (int i = 0; i < cnt; i++)
        if (br_u1(&b)) skip_scaling_list(&b, i < 6 ? 16 : 64);
    }
    br_se(&b); /* second_chroma_qp_index_offset */
  }
  if (b.err) return -1;
  q.valid = 1;
  ps->pps[id] = q;
  return (int)id;
}

/* ------------------------------------------------------------------------------- SEI */
int avr_parse_sei_x264_build(const uint8_t *rbsp, size_t n) {
  size_t p = 0;
  while (p + 2 <= n) {
    int type = 0, size = 0;
    while (p < n && rbsp[p] == 0xff) { type += 255; p++; }
    if (p >= n) break;
    type += rbsp[p++];
    while (p < n && rbsp[p] == 0xff) { size += 255; p++; }
    if (p >= n) break;
    size += rbsp[p++];
    if (p + (size_t)size > n) break;
    if (type == 5 && size > 16) {
      const uint8_t *u = rbsp + p + 16;
      size_t ul = (size_t)size - 16;
      static const char tag[] = "x264 - core ";
      if (ul > sizeof(tag) - 1 && memcmp(u, tag, sizeof(tag) - 1) == 0) {
        int build = 0;
        size_t k = sizeof(tag) - 1;
        int digits = 0;
        while (k < ul && u[k] >= '0' && u[k] <= '9') { build = build * 10 + (u[k] - '0'); k++; digits++; }
        if (digits && build > 0) return build;
      }
    }
    p += (size_t)size;
  }
  return -1;
}

/* ------------------------------------------------------------------------- slice header */
int avr_parse_slice_header(const avr_param_sets_t *ps, const uint8_t *rbsp, size_t n,
                           int nal_unit_type, int nal_ref_idc, avr_slice_hdr_t *h) {
  br_t b;
  br_init(&b, rbsp, n);
  memset(h, 0, sizeof(*h));
  h->x264_build = -1;
  h->nal_unit_type = nal_unit_type;
  h->nal_ref_idc = nal_ref_idc;
  h->first_mb = (int)br_ue(&b);
  int st = (int)br_ue(&b);
  if (st > 9) return -1;
  h->slice_type = st % 5;
  h->pps_id = (int)br_ue(&b);
  if (h->pps_id > 255 || !ps->pps[h->pps_id].valid) return -1;
  const avr_pps_t *pps = &ps->pps[h->pps_id];
  const avr_sps_t *sps = &ps->sps[pps->sps_id];
  if (!sps->valid) return -1;
  if (sps->separate_colour_plane) br_u(&b, 2);
  h->frame_num = (int)br_u(&b, sps->log2_max_frame_num);
  if (!sps->frame_mbs_only) {
    h->field_pic = (int)br_u1(&b);
    if (h->field_pic) h->bottom_field = (int)br_u1(&b);
  }
  h->mbaff = sps->mb_aff && !h->field_pic;
  if (h->mbaff) h->first_mb *= 2; /* first_mb_in_slice counts macroblock pairs (7.4.3) */
  if (nal_unit_type == 5) h->idr_pic_id = (int)br_ue(&b);
  if (sps->poc_type == 0) {
    h->poc_lsb = (int)br_u(&b, sps->log2_max_poc_lsb);
    if (pps->bottom_field_pic_order_present && !h->field_pic) br_se(&b);
  }
  if (sps->poc_type == 1 && !sps->delta_pic_order_always_zero) {
    br_se(&b);
    if (pps->bottom_field_pic_order_present && !h->field_pic) br_se(&b);
  }
  if (pps->redundant_pic_cnt_present) br_ue(&b);
  if (h->slice_type == AVR_SLICE_B) h->direct_spatial = (int)br_u1(&b);
  h->num_ref_idx_active[0] = pps->num_ref_idx_default[0];
  h->num_ref_idx_active[1] = pps->num_ref_idx_default[1];
  if (h->slice_type == AVR_SLICE_P || h->slice_type == AVR_SLICE_SP || h->slice_type == AVR_SLICE_B) {
    if (br_u1(&b)) {
      h->num_ref_idx_active[0] = 1 + (int)br_ue(&b);
      if (h->slice_type == AVR_SLICE_B) h->num_ref_idx_active[1] = 1 + (int)br_ue(&b);
    }
  }
  if (h->slice_type != AVR_SLICE_B) h->num_ref_idx_active[1] = 0;
  if (h->slice_type == AVR_SLICE_I || h->slice_type == AVR_SLICE_SI) h->num_ref_idx_active[0] = 0;
  /* ref_pic_list_modification() (nal 20/21 MVC variants are not video we parse) */
  if (h->slice_type != AVR_SLICE_I && h->slice_type != AVR_SLICE_SI) {
    for (int l = 0; l < (h->slice_type == AVR_SLICE_B ? 2 : 1); l++) {
      if (br_u1(&b)) {
        for (int guard = 0; guard < 1000 && !b.err; guard++) {
          uint32_t idc = br_ue(&b);
          if (idc == 3) break;
          if (idc > 5) return -1;
          br_ue(&b);
        }
      }
    }
  }
  int chroma_array_type = sps->separate_colour_plane ? 0 : sps->chroma_format_idc;
  if ((pps->weighted_pred && (h->slice_type == AVR_SLICE_P || h->slice_type == AVR_SLICE_SP)) ||
      (pps->weighted_bipred_idc == 1 && h->slice_type == AVR_SLICE_B)) {
    br_ue(&b); /* luma_log2_weight_denom */
    if (chroma_array_type != 0) br_ue(&b);
    for (int l = 0; l < (h->slice_type == AVR_SLICE_B ? 2 : 1); l++) {
      for (int i = 0; i < h->num_ref_idx_active[l] && !b.err; i++) {
        if (br_u1(&b)) { br_se(&b); br_se(&b); }
        if (chroma_array_type != 0 && br_u1(&b)) { br_se(&b); br_se(&b); br_se(&b); br_se(&b); }
      }
    }
  }
  if (nal_ref_idc != 0) { /* dec_ref_pic_marking() */
    if (nal_unit_type == 5) {
      br_u1(&b);
      br_u1(&b);
    } else if (br_u1(&b)) {
      for (int guard = 0; guard < 1000 && !b.err; guard++) {
        uint32_t op = br_ue(&b);
        if (op == 0) break;
        if (op > 6) return -1;
        if (op == 1 || op == 3) br_ue(&b);
        if (op == 2) br_ue(&b);
        if (op == 3 || op == 6) br_ue(&b);
        if (op == 4) br_ue(&b);
      }
    }
  }
  if (pps->entropy_coding_mode && h->slice_type != AVR_SLICE_I && h->slice_type != AVR_SLICE_SI)
    h->cabac_init_idc = (int)br_ue(&b);
  else
    h->cabac_init_idc = -1;
  h->slice_qp = pps->pic_init_qp + br_se(&b);
  if (h->slice_type == AVR_SLICE_SP || h->slice_type == AVR_SLICE_SI) {
    if (h->slice_type == AVR_SLICE_SP) br_u1(&b);
    br_se(&b);
  }
  if (pps->deblocking_filter_control_present) {
    uint32_t idc = br_ue(&b);
    if (idc != 1) { br_se(&b); br_se(&b); }
  }
  if (b.err) return -1;
  /* slice_data(): cabac_alignment_one_bit until aligned */
  h->cabac_start = (b.pos + 7) / 8;
  h->chroma_array_type = chroma_array_type;
  h->transform_8x8_mode = pps->transform_8x8_mode;
  h->direct_8x8_inference = sps->direct_8x8_inference;
  h->constrained_intra_pred = pps->constrained_intra_pred;
  h->mb_width = sps->mb_width;
  h->mb_height = sps->mb_height;
  /* macroblocks in this picture: a field has half the frame's rows */
  int pic_mbs = sps->mb_width * (h->field_pic ? sps->mb_height / 2 : sps->mb_height);
  h->supported = pps->entropy_coding_mode && !sps->separate_colour_plane &&
                 h->slice_type != AVR_SLICE_SP && h->slice_type != AVR_SLICE_SI &&
                 (h->cabac_init_idc <= 2) && h->first_mb < pic_mbs &&
                 h->num_ref_idx_active[0] <= 32 && h->num_ref_idx_active[1] <= 32;
  return 0;
}

/* --------------------------------------------------------------------------------- demux */
static uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
static uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) << 32 | rd32(p + 4); }

typedef struct {
  const uint8_t *avcc;
  size_t avcc_len, avcc_off;
  const uint8_t *stsz, *stco, *stsc;
  size_t stsz_len, stco_len, stsc_len;
  int co64;
  int is_video;
} trak_t;

static int box_children(const uint8_t *f, size_t off, size_t end, trak_t *t, int depth);

static int parse_box(const uint8_t *f, size_t off, size_t end, size_t *next, uint32_t *type, size_t *body,
                     size_t *body_end) {
  if (off + 8 > end) return -1;
  uint64_t sz = rd32(f + off);
  *type = rd32(f + off + 4);
  size_t hdr = 8;
  if (sz == 1) {
    if (off + 16 > end) return -1;
    sz = rd64(f + off + 8);
    hdr = 16;
  } else if (sz == 0) {
    sz = end - off;
  }
  if (sz < hdr || off + sz > end) return -1;
  *body = off + hdr;
  *body_end = off + (size_t)sz;
  *next = off + (size_t)sz;
  return 0;
}

#define FOURCC(a, b, c, d) ((uint32_t)(a) << 24 | (uint32_t)(b) << 16 | (uint32_t)(c) << 8 | (uint32_t)(d))

static int box_children(const uint8_t *f, size_t off, size_t end, trak_t *t, int depth) {
  while (off + 8 <= end) {
    uint32_t type;
    size_t body, bend, next;
    if (parse_box(f, off, end, &next, &type, &body, &bend)) return -1;
    switch (type) {
      case FOURCC('m', 'd', 'i', 'a'):
      case FOURCC('m', 'i', 'n', 'f'):
      case FOURCC('s', 't', 'b', 'l'):
        if (depth < 8) box_children(f, body, bend, t, depth + 1);
        break;
      case FOURCC('h', 'd', 'l', 'r'):
        if (bend - body >= 12 && rd32(f + body + 8) == FOURCC('v', 'i', 'd', 'e')) t->is_video = 1;
        break;
      case FOURCC('s', 't', 's', 'd'): {
        size_t p = body + 8; /* version/flags + entry_count */
        if (p + 8 <= bend) {
          uint32_t esz = rd32(f + p), etype = rd32(f + p + 4);
          if (etype == FOURCC('a', 'v', 'c', '1') || etype == FOURCC('a', 'v', 'c', '3')) {
            size_t c = p + 8 + 78, cend = p + esz;
            if (cend > bend) cend = bend;
            while (c + 8 <= cend) {
              uint32_t ct;
              size_t cb, cbe, cn;
              if (parse_box(f, c, cend, &cn, &ct, &cb, &cbe)) break;
              if (ct == FOURCC('a', 'v', 'c', 'C')) {
                t->avcc = f + cb;
                t->avcc_len = cbe - cb;
                t->avcc_off = cb;
              }
              c = cn;
            }
          }
        }
        break;
      }
      case FOURCC('s', 't', 's', 'z'): t->stsz = f + body; t->stsz_len = bend - body; break;
      case FOURCC('s', 't', 'c', 'o'): t->stco = f + body; t->stco_len = bend - body; t->co64 = 0; break;
      case FOURCC('c', 'o', '6', '4'): t->stco = f + body; t->stco_len = bend - body; t->co64 = 1; break;
      case FOURCC('s', 't', 's', 'c'): t->stsc = f + body; t->stsc_len = bend - body; break;
      default: break;
    }
    off = next;
  }
  return 0;
}

typedef struct {
  avr_nal_t *v;
  int n, cap;
} nal_vec_t;
static void nv_push(nal_vec_t *nv, size_t off, size_t size) {
  if (nv->n == nv->cap) {
    nv->cap = nv->cap ? nv->cap * 2 : 256;
    nv->v = (avr_nal_t *)realloc(nv->v, (size_t)nv->cap * sizeof(avr_nal_t));
  }
  nv->v[nv->n].offset = off;
  nv->v[nv->n].size = size;
  nv->n++;
}

static int demux_mp4(const uint8_t *f, size_t n, nal_vec_t *nv) {
  size_t off = 0;
  trak_t video;
  memset(&video, 0, sizeof(video));
  int found = 0;
  while (off + 8 <= n) {
    uint32_t type;
    size_t body, bend, next;
    if (parse_box(f, off, n, &next, &type, &body, &bend)) break;
    if (type == FOURCC('m', 'o', 'o', 'v')) {
      size_t c = body;
      while (c + 8 <= bend) {
        uint32_t ct;
        size_t cb, cbe, cn;
        if (parse_box(f, c, bend, &cn, &ct, &cb, &cbe)) break;
        if (ct == FOURCC('t', 'r', 'a', 'k')) {
          trak_t t;
          memset(&t, 0, sizeof(t));
          box_children(f, cb, cbe, &t, 0);
          if (t.is_video && t.avcc && !found) { video = t; found = 1; }
        }
        c = cn;
      }
    }
    off = next;
  }
  if (!found || !video.stsz || !video.stco || !video.stsc || video.avcc_len < 7) return -1;
  const uint8_t *a = video.avcc;
  int len_size = (a[4] & 3) + 1;
  size_t p = 5;
  int nsps = a[p++] & 31;
  for (int i = 0; i < nsps && p + 2 <= video.avcc_len; i++) {
    size_t l = (size_t)a[p] << 8 | a[p + 1];
    p += 2;
    if (p + l > video.avcc_len) return -1;
    nv_push(nv, video.avcc_off + p, l);
    p += l;
  }
  if (p < video.avcc_len) {
    int npps = a[p++];
    for (int i = 0; i < npps && p + 2 <= video.avcc_len; i++) {
      size_t l = (size_t)a[p] << 8 | a[p + 1];
      p += 2;
      if (p + l > video.avcc_len) return -1;
      nv_push(nv, video.avcc_off + p, l);
      p += l;
    }
  }
  /* sample table */
  if (video.stsz_len < 12 || video.stco_len < 8 || video.stsc_len < 8) return -1;
  uint32_t fixed_size = rd32(video.stsz + 4), nsamples = rd32(video.stsz + 8);
  uint32_t nchunks = rd32(video.stco + 4), nstsc = rd32(video.stsc + 4);
  if (fixed_size == 0 && 12 + 4ull * nsamples > video.stsz_len) return -1;
  if (8 + (video.co64 ? 8ull : 4ull) * nchunks > video.stco_len || 8 + 12ull * nstsc > video.stsc_len) return -1;
  uint32_t sample = 0;
  for (uint32_t e = 0; e < nstsc && sample < nsamples; e++) {
    const uint8_t *ent = video.stsc + 8 + 12 * e;
    uint32_t first = rd32(ent), per = rd32(ent + 4);
    uint32_t last = e + 1 < nstsc ? rd32(video.stsc + 8 + 12 * (e + 1)) - 1 : nchunks;
    for (uint32_t c = first; c <= last && c <= nchunks && sample < nsamples; c++) {
      size_t coff = video.co64 ? (size_t)rd64(video.stco + 8 + 8 * (c - 1)) : rd32(video.stco + 8 + 4 * (c - 1));
      for (uint32_t s = 0; s < per && sample < nsamples; s++, sample++) {
        size_t ssz = fixed_size ? fixed_size : rd32(video.stsz + 12 + 4 * sample);
        if (coff + ssz > n) return -1;
        size_t q = coff, qe = coff + ssz;
        while (q + (size_t)len_size <= qe) {
          size_t l = 0;
          for (int k = 0; k < len_size; k++) l = l << 8 | f[q + k];
          q += (size_t)len_size;
          if (l == 0 || q + l > qe) break;
          nv_push(nv, q, l);
          q += l;
        }
        coff += ssz;
      }
    }
  }
  return 0;
}

static int demux_annexb(const uint8_t *f, size_t n, nal_vec_t *nv) {
  size_t i = 0;
  /* find first start code */
  while (i + 3 <= n && !(f[i] == 0 && f[i + 1] == 0 && f[i + 2] == 1)) i++;
  while (i + 3 <= n) {
    size_t start = i + 3, j = start;
    while (j + 3 <= n && !(f[j] == 0 && f[j + 1] == 0 && (f[j + 2] == 1 || f[j + 2] == 0))) j++;
    size_t end = j + 3 <= n ? j : n;
    /* trailing_zero_8bits before the next start code */
    while (end > start && f[end - 1] == 0) end--;
    if (end > start) nv_push(nv, start, end - start);
    i = j;
    while (i + 3 <= n && !(f[i] == 0 && f[i + 1] == 0 && f[i + 2] == 1)) i++;
  }
  return 0;
}

int avr_demux(const uint8_t *file, size_t n, avr_nal_t **out) {
  nal_vec_t nv = {NULL, 0, 0};
  int is_mp4 = n >= 8 && (rd32(file + 4) == FOURCC('f', 't', 'y', 'p') || rd32(file + 4) == FOURCC('m', 'o', 'o', 'v') ||
                          rd32(file + 4) == FOURCC('m', 'd', 'a', 't') || rd32(file + 4) == FOURCC('f', 'r', 'e', 'e'));
  int r = is_mp4 ? demux_mp4(file, n, &nv) : demux_annexb(file, n, &nv);
  if (r || nv.n == 0) { /* no H.264 in it: the reference's avformat_open_input fails */
    free(nv.v);
    *out = NULL;
    return -1;
  }
  *out = nv.v;
  return nv.n;
}
