/*
 * Test driver (TEST INFRASTRUCTURE): plays the libavcodec-hooks caller against the C-ABI hooks
 * layer of libavrecode.so.  The oracle's slice_data() parser (oracle/oracle_walker.c) stands in for
 * the fork's H.264 decoder: it walks every CABAC slice of the stream, pulling each bin through
 * avr_hook_get / _bypass / _terminate and reporting the model events (mb_xy, begin/end_sub_mb,
 * begin/end_coding_type) exactly where the fork would.  The parse is driven by the device's bins,
 * so a wrong bin desynchronises it (and the layer checks the caller's context states).
 *
 * Built by tests/test_hooks.py into tests/native/_build/libhooks_driver.so.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/avrecode.h"
#include "../../oracle/avr_oracle.h"

/* Perturbations (hooks_set_perturb): a caller whose hook placement differs from the device's parse
 * in one event, which the layer must reject with AVR_ERR_FORMAT:
 *   1  the k-th begin_coding_type(SIG_MAP) one bin late
 *   2  frame_spec repeats picture k-1's frame_num for picture k
 *   3  the k-th mb_xy reports x ^ 1
 *   4  the k-th begin_sub_mb / end_sub_mb pair reports scan8 index ^ 1 */
static int g_perturb, g_k;
/* frame_spec's first argument: the driver's decode-order picture counter (default), or the slice
 * header's frame_num as the fork passes it (hooks_set_frame_num_syntax(1)), which consecutive
 * pictures share after a non-reference picture */
static int g_syntax_fn;
void hooks_set_frame_num_syntax(int on) { g_syntax_fn = on; }
static long g_maps, g_mbs, g_subs, g_sub_bad;
static int g_delayed;   /* a begin_coding_type(SIG_MAP) waiting for the next bin */
static void *g_session;
/* streaming compress (hooks_compress_stream): the bytes of `g_file` handed to the session so far;
 * before each slice's init_decoder the driver feeds through the end of that slice's NAL unit, in two
 * pieces, as a demuxer's read_packet would (recode.cpp:1127-1131) */
static const uint8_t *g_file;
static size_t g_fed, g_file_len;
static int g_feed_err;
/* hooks_set_feed_chunk(k): the demuxer reads fixed k-byte pieces (the last one shorter), so a
 * slice's bytes arrive with whatever follows them in its piece (0: exactly through the NAL unit) */
static size_t g_chunk;
void hooks_set_feed_chunk(size_t k) { g_chunk = k; }
/* per-slice wall time of the last drive() (feed + init_decoder + the slice's walk), seconds */
static double *g_times;
static long g_ntimes, g_captimes;
int hooks_slice_times(double *out, int cap) {
  for (long i = 0; i < g_ntimes && i < cap; i++) out[i] = g_times[i];
  return (int)g_ntimes;
}
/* per slice of the last drive(): avr_debug_hooks_regenerated after its init_decoder (decompress) */
int avr_debug_hooks_regenerated(const avr_hooks_session *hs);
static long *g_regen;
static long g_nregen, g_capregen;
int hooks_slice_regen(long *out, int cap) {
  for (long i = 0; i < g_nregen && i < cap; i++) out[i] = g_regen[i];
  return (int)g_nregen;
}
static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}
static void feed_to(size_t end) {
  if (g_file && g_chunk) {
    end = (end + g_chunk - 1) / g_chunk * g_chunk;
    if (end > g_file_len) end = g_file_len;
  }
  if (!g_file || end <= g_fed) return;
  size_t mid = g_fed + (end - g_fed) / 2;
  if (avr_hooks_feed((avr_hooks_session *)g_session, g_file + g_fed, mid - g_fed) != AVR_OK) g_feed_err = 1;
  if (avr_hooks_feed((avr_hooks_session *)g_session, g_file + mid, end - mid) != AVR_OK) g_feed_err = 1;
  g_fed = end;
}
void hooks_set_perturb(int mode, int k) { g_perturb = mode; g_k = k; g_maps = g_mbs = g_subs = 0; g_delayed = 0; }

static void flush_delayed(void) {
  if (g_delayed) { g_delayed = 0; avr_hook_begin_coding_type(g_session, AVR_PIP_SIGNIFICANCE_MAP, 0, 0, 0); }
}
static int fwd_get(void *o, uint8_t *state, int ctx_idx) {
  (void)ctx_idx;
  int b = avr_hook_get(o, state);   /* the delayed begin lands after this bin */
  flush_delayed();
  return b;
}
static int fwd_bypass(void *o) { int b = avr_hook_get_bypass(o); flush_delayed(); return b; }
static int fwd_terminate(void *o) { int b = avr_hook_get_terminate(o); flush_delayed(); return b; }

/* The model hooks go to the session (AVCodecHooks.opaque); the cabac hooks to the slice object. */
static void m_frame_spec(void *o, int f, int w, int h) {
  (void)o;
  if (g_perturb == 2 && f == g_k) f = g_k - 1;
  avr_hook_frame_spec(g_session, f, w, h);
}
static void m_mb_xy(void *o, int x, int y) {
  (void)o;
  if (g_perturb == 3 && g_mbs++ == g_k) x ^= 1;
  avr_hook_mb_xy(g_session, x, y);
}
static void m_begin_sub(void *o, int a, int b, int c, int d, int e) {
  (void)o;
  g_sub_bad = g_perturb == 4 && g_subs++ == g_k;
  avr_hook_begin_sub_mb(g_session, a, g_sub_bad ? b ^ 1 : b, c, d, e);
}
static void m_end_sub(void *o, int a, int b, int c, int d, int e) {
  (void)o;
  avr_hook_end_sub_mb(g_session, a, g_sub_bad ? b ^ 1 : b, c, d, e);
}
static void m_begin_ct(void *o, avr_coding_type ct, int z, int p0, int p1) {
  (void)o;
  if (g_perturb == 1 && ct == PIP_SIGNIFICANCE_MAP && g_maps++ == g_k) { g_delayed = 1; return; }
  avr_hook_begin_coding_type(g_session, (int)ct, z, p0, p1);
}
static void m_end_ct(void *o, avr_coding_type ct) {
  (void)o;
  flush_delayed();
  avr_hook_end_coding_type(g_session, (int)ct);
}

/* Decode every CABAC slice of `stream` through the hooks (the fork's av_decoder loop,
 * recode.cpp:114-135).  Returns the number of slices walked, or < 0. */
static long drive(const uint8_t *stream, size_t n) {
  avr_nal_t *nals;
  int nn = avr_demux(stream, n, &nals);
  if (nn < 0) return -1;
  avr_param_sets_t *ps = (avr_param_sets_t *)calloc(1, sizeof(avr_param_sets_t));
  int x264_build = -1, have_prev = 0, picture_id = 0, second_field = 0;
  avr_slice_hdr_t prev;
  long walked = 0;
  memset(&prev, 0, sizeof(prev));
  g_ntimes = 0;
  g_nregen = 0;
  for (int i = 0; i < nn; i++) {
    const uint8_t *nal = stream + nals[i].offset;
    size_t len = nals[i].size;
    if (len < 2) continue;
    int type = nal[0] & 0x1f, ref_idc = (nal[0] >> 5) & 3;
    if (type != 1 && type != 5 && type != 6 && type != 7 && type != 8) continue;
    uint8_t *rbsp = (uint8_t *)malloc(len);
    size_t rl = avr_nal_unescape(nal + 1, len - 1, rbsp);
    if (type == 6) { int b = avr_parse_sei_x264_build(rbsp, rl); if (b > 0) x264_build = b; free(rbsp); continue; }
    if (type == 7) { avr_parse_sps(ps, rbsp, rl); free(rbsp); continue; }
    if (type == 8) { avr_parse_pps(ps, rbsp, rl); free(rbsp); continue; }
    avr_slice_hdr_t h;
    if (avr_parse_slice_header(ps, rbsp, rl, type, ref_idc, &h) != 0 || !ps->pps[h.pps_id].entropy_coding_mode) {
      free(rbsp);
      continue;
    }
    h.x264_build = x264_build;
    int new_pic = !have_prev || h.first_mb == 0 || h.first_mb <= prev.first_mb || h.frame_num != prev.frame_num ||
                  h.pps_id != prev.pps_id || h.poc_lsb != prev.poc_lsb ||
                  (h.nal_unit_type == 5) != (prev.nal_unit_type == 5) || h.idr_pic_id != prev.idr_pic_id ||
                  (h.nal_ref_idc == 0) != (prev.nal_ref_idc == 0) || h.field_pic != prev.field_pic ||
                  h.bottom_field != prev.bottom_field;
    /* frame_spec's frame: the two fields of a frame share frame_num, so the second field stays
     * in the first one's frame (update_frame_spec, recode.cpp:824-843) */
    int second = new_pic && have_prev && h.field_pic && prev.field_pic && h.frame_num == prev.frame_num &&
                 h.bottom_field != prev.bottom_field && !second_field;
    if (new_pic && !second) picture_id++;
    if (new_pic) second_field = second;
    prev = h;
    have_prev = 1;
    size_t bits = avr_rbsp_bit_length(rbsp, rl);
    size_t end = (bits + 7) / 8;
    size_t size = end > h.cabac_start ? end - h.cabac_start : 0;
    const double t0 = now_s();
    m_frame_spec(NULL, g_syntax_fn ? h.frame_num : picture_id, h.mb_width, h.mb_height);
    feed_to(nals[i].offset + nals[i].size);
    void *slice = avr_hook_init_decoder(g_session, NULL, rbsp + h.cabac_start, (int)size);
    if (g_nregen == g_capregen) {
      g_capregen = g_capregen ? 2 * g_capregen : 1024;
      g_regen = (long *)realloc(g_regen, sizeof(long) * (size_t)g_capregen);
    }
    g_regen[g_nregen++] = avr_debug_hooks_regenerated(g_session);
    if (slice) {
      avr_hooks_t hk = {slice, fwd_get, fwd_bypass, fwd_terminate, m_frame_spec, m_mb_xy,
                        m_begin_sub, m_end_sub, m_begin_ct, m_end_ct};
      /* the walker's own frame_spec call (the fork's, at the slice start) passes the same value */
      if (avr_walk_slice(&h, &hk, g_syntax_fn ? h.frame_num : picture_id) != 0) { free(rbsp); walked = -2; break; }
      walked++;
    }
    if (g_ntimes == g_captimes) {
      g_captimes = g_captimes ? 2 * g_captimes : 1024;
      g_times = (double *)realloc(g_times, sizeof(double) * (size_t)g_captimes);
    }
    g_times[g_ntimes++] = now_s() - t0;
    free(rbsp);
  }
  free(ps);
  free(nals);
  return walked;
}

/* compress `file` through the hooks; *out = the container.  Returns avr status (or -100 - x on a
 * driver failure); *walked = slices walked through the hooks. */
int hooks_compress(const uint8_t *file, size_t n, int model, uint8_t **out, size_t *out_len, long *walked) {
  avr_ctx *c;
  int r = avr_create(0, &c);
  if (r) return r;
  avr_hooks_session *s;
  r = avr_hooks_compress_begin(c, file, n, model, &s);
  if (r) { avr_destroy(c); return r; }
  g_session = s;
  *walked = drive(file, n);
  r = avr_hooks_end(s, out, out_len);
  avr_hooks_destroy(s);
  avr_destroy(c);
  return *walked < 0 ? -100 + (int)*walked : r;
}

/* the same through a streaming session: the file's bytes reach the session only as the slices
 * that need them are decoded (the rest after the last slice). */
int hooks_compress_stream(const uint8_t *file, size_t n, int model, uint8_t **out, size_t *out_len, long *walked) {
  avr_ctx *c;
  int r = avr_create(0, &c);
  if (r) return r;
  avr_hooks_session *s;
  r = avr_hooks_compress_stream_begin(c, model, &s);
  if (r) { avr_destroy(c); return r; }
  g_session = s;
  g_file = file;
  g_file_len = n;
  g_fed = 0;
  g_feed_err = 0;
  /* MP4 read through a non-seekable read_packet (recode.cpp:84-90): the mov demuxer reads up to
   * the moov box before the first packet -- for moov-last files, the whole file; a moov-first
   * ("faststart") file then streams sample by sample */
  if (n >= 8 && memcmp(file + 4, "ftyp", 4) == 0) {
    size_t off = 0, moov_end = n;
    while (off + 8 <= n) {
      size_t sz = (size_t)file[off] << 24 | (size_t)file[off + 1] << 16 | (size_t)file[off + 2] << 8 | file[off + 3];
      if (sz < 8 || sz > n - off) break;
      if (!memcmp(file + off + 4, "moov", 4)) { moov_end = off + sz; break; }
      if (!memcmp(file + off + 4, "mdat", 4)) break;   /* media first: the moov box is last */
      off += sz;
    }
    feed_to(moov_end);
  }
  *walked = drive(file, n);
  feed_to(n);
  g_file = NULL;
  r = avr_hooks_end(s, out, out_len);
  avr_hooks_destroy(s);
  avr_destroy(c);
  if (g_feed_err) return -200;
  return *walked < 0 ? -100 + (int)*walked : r;
}

/* decompress a container through the hooks; *out = the original file. */
int hooks_decompress(const uint8_t *avrc, size_t n, uint8_t **out, size_t *out_len, long *walked) {
  avr_ctx *c;
  int r = avr_create(0, &c);
  if (r) return r;
  avr_hooks_session *s;
  const uint8_t *stream;
  size_t stream_len;
  r = avr_hooks_decompress_begin(c, avrc, n, &s, &stream, &stream_len);
  if (r) { avr_destroy(c); return r; }
  g_session = s;
  *walked = drive(stream, stream_len);
  r = avr_hooks_end(s, out, out_len);
  if (r) fprintf(stderr, "hooks_decompress: %s\n", avr_last_error(c));
  avr_hooks_destroy(s);
  avr_destroy(c);
  return *walked < 0 ? -100 + (int)*walked : r;
}
