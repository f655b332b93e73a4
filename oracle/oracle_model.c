/*
 * Oracle: h264_model (recode.cpp:615-1059) and the scan geometry it uses (recode.cpp:233-471).
 * TEST INFRASTRUCTURE ONLY (see avr_oracle.h).
 *
 * Restated line by line.  Differences from the reference, all output-neutral except (3):
 *  (1) the neighbour / coefficient priors computed at recode.cpp:708-791 are dead (794-797) and
 *      are not computed (they would assert on 4:2:2 chroma DC at recode.cpp:500);
 *  (2) reverse_scan_8 (recode.cpp:279-312) is derived from scan_8 instead of tabulated; the
 *      entries get_neighbor_sub_mb can reach are identical;
 *  (3) decompress side only: the nnz-bit key uses is_8x8 || size > 32 (see model_finished_queueing).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_model.h"

static const uint8_t scan_8[51] = { /* recode.cpp:263-277 */
  4 + 1 * 8,  5 + 1 * 8,  4 + 2 * 8,  5 + 2 * 8,  6 + 1 * 8,  7 + 1 * 8,  6 + 2 * 8,  7 + 2 * 8,
  4 + 3 * 8,  5 + 3 * 8,  4 + 4 * 8,  5 + 4 * 8,  6 + 3 * 8,  7 + 3 * 8,  6 + 4 * 8,  7 + 4 * 8,
  4 + 6 * 8,  5 + 6 * 8,  4 + 7 * 8,  5 + 7 * 8,  6 + 6 * 8,  7 + 6 * 8,  6 + 7 * 8,  7 + 7 * 8,
  4 + 8 * 8,  5 + 8 * 8,  4 + 9 * 8,  5 + 9 * 8,  6 + 8 * 8,  7 + 8 * 8,  6 + 9 * 8,  7 + 9 * 8,
  4 + 11 * 8, 5 + 11 * 8, 4 + 12 * 8, 5 + 12 * 8, 6 + 11 * 8, 7 + 11 * 8, 6 + 12 * 8, 7 + 12 * 8,
  4 + 13 * 8, 5 + 13 * 8, 4 + 14 * 8, 5 + 14 * 8, 6 + 13 * 8, 7 + 13 * 8, 6 + 14 * 8, 7 + 14 * 8,
  0 + 0 * 8,  0 + 5 * 8,  0 + 10 * 8,
};

/* reverse_scan_8 semantics: the block living at scan8 cell (row, col), possibly in the left / upper
 * neighbour macroblock.  Planes occupy rows 1-4 (Y), 6-9 (U), 11-14 (V), columns 4-7; column 3 is
 * the left neighbour's right column, rows 0/5/10 the upper neighbour's bottom row. */
static int rev_scan8(int row, int col, int *left, int *up) {
  *left = *up = 0;
  int plane_top = row <= 4 ? 1 : row <= 9 ? 6 : 11;
  if (row == plane_top - 1) { *up = 1; row = plane_top + 3; }
  if (col == 3) { *left = 1; col = 7; }
  int cell = row * 8 + col;
  for (int k = 0; k < 48; k++)
    if (scan_8[k] == cell) return k;
  return -1;
}

/* get_neighbor_sub_mb (recode.cpp:419-471) */
static int get_neighbor_sub_mb(int above, int sub_mb_size, int mb_x, int mb_y, int scan8_index, int *ox,
                               int *oy, int *oidx) {
  *ox = mb_x;
  *oy = mb_y;
  *oidx = scan8_index;
  if (scan8_index >= 16 * 3) {
    if (above) {
      if (mb_y > 0) { *oy = mb_y - 1; return 1; }
      return 0;
    }
    if (mb_x > 0) { *ox = mb_x - 1; return 1; }
    return 0;
  }
  int s = scan_8[scan8_index];
  int left, up;
  int idx = rev_scan8((s >> 3) + (above ? -1 : 0), (s & 7) + (above ? 0 : -1), &left, &up);
  if (left) {
    if (mb_x == 0) return 0;
    mb_x--;
  }
  if (up) {
    if (mb_y == 0) return 0;
    mb_y--;
  }
  if (sub_mb_size >= 32) idx = idx / 4 * 4;
  *oidx = idx;
  *ox = mb_x;
  *oy = mb_y;
  return 1;
}
/* exported for tests/test_oracle_geometry.py: compared with the reference's get_neighbor_sub_mb
 * compiled from recode.cpp:419-471 (tests/golden/geometry.json) */
int oracle_get_neighbor_sub_mb(int above, int sub_mb_size, int mb_x, int mb_y, int scan8_index, int *out3) {
  return get_neighbor_sub_mb(above, sub_mb_size, mb_x, mb_y, scan8_index, &out3[0], &out3[1], &out3[2]);
}
const uint8_t *oracle_scan_8(void) { return scan_8; }

/* ------------------------------------------------------------------------- FrameBuffer */
static void fb_bzero(framebuf_t *f) {
  size_t n = (size_t)f->width * f->height;
  memset(f->meta, 0, n * sizeof(blockmeta_t));
  memset(f->image, 0, n * sizeof(mbblock_t));
}
static void fb_init(framebuf_t *f, uint32_t w, uint32_t h) {
  free(f->meta);
  free(f->image);
  f->width = w;
  f->height = h;
  f->meta = (blockmeta_t *)calloc((size_t)w * h, sizeof(blockmeta_t));
  f->image = (mbblock_t *)calloc((size_t)w * h, sizeof(mbblock_t));
}
blockmeta_t *model_meta(avr_model_t *m, int which, int x, int y) {
  framebuf_t *f = &m->frames[which];
  return &f->meta[x + y * f->width];
}
static mbblock_t *model_block(avr_model_t *m, int x, int y) {
  framebuf_t *f = &m->frames[m->cur_frame];
  return &f->image[x + y * f->width];
}

static FILE *keylog_file(void);
avr_model_t *avr_model_new(void) {
  if (keylog_file()) { model_key_t mark = ~(model_key_t)0; fwrite(&mark, sizeof(mark), 1, keylog_file()); }
  avr_model_t *m = (avr_model_t *)calloc(1, sizeof(avr_model_t));
  m->coding_type = PIP_UNKNOWN;
  m->sub_mb_cat = -1;
  m->sub_mb_size = -1;
  m->cap = 1 << 16;
  m->keys = (model_key_t *)malloc(m->cap * sizeof(model_key_t));
  m->vals = (estimator_t *)malloc(m->cap * sizeof(estimator_t));
  m->used = (uint8_t *)calloc(m->cap, 1);
  return m;
}
void avr_model_bills(const avr_model_t *m, size_t bill[8], size_t cabac_bill[8]) {
  for (int i = 0; i < 8; i++) {
    bill[i] += m->bill[i];
    cabac_bill[i] += m->cabac_bill[i];
  }
}

void avr_model_free(avr_model_t *m) {
  if (!m) return;
  for (int i = 0; i < 2; i++) { free(m->frames[i].meta); free(m->frames[i].image); }
  free(m->keys);
  free(m->vals);
  free(m->used);
  free(m);
}

/* Experiment hooks (a per-file prior for the parallel model's per-context
 * estimators; measured by scripts/prior_experiment.py, not part of any format):
 *   AVR_ORACLE_STATS=path  count every coded bin of a per-context key (kind < 1026, the
 *                          model's default keys, recode.cpp:677-683) by context and value; the
 *                          counts (u64[1026][2]) are written to path at exit
 *   AVR_ORACLE_PRIOR=path  a new per-context estimator starts from path's (u16[1026][2]: pos,
 *                          neg) instead of {1, 1} (recode.cpp:1057) */
static uint64_t g_stats[1026][2];
static int g_stats_on = -1;
static uint16_t g_prior[1026][2];
static int g_prior_on = -1;
static void stats_write(void) {
  const char *p = getenv("AVR_ORACLE_STATS");
  FILE *f = p ? fopen(p, "wb") : NULL;
  if (f) { fwrite(g_stats, sizeof(g_stats), 1, f); fclose(f); }
}
static int stats_on(void) {
  if (g_stats_on < 0) {
    g_stats_on = getenv("AVR_ORACLE_STATS") != NULL;
    if (g_stats_on) atexit(stats_write);
  }
  return g_stats_on;
}
static int prior_on(void) {
  if (g_prior_on < 0) {
    const char *p = getenv("AVR_ORACLE_PRIOR");
    FILE *f = p ? fopen(p, "rb") : NULL;
    g_prior_on = f && fread(g_prior, sizeof(g_prior), 1, f) == 1;
    if (f) fclose(f);
  }
  return g_prior_on;
}
static inline int default_kind(model_key_t key) { return (key & 0xffffffffffffull) == 0 && (key >> 48) < 1026; }

static inline size_t hash_key(model_key_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return (size_t)k;
}
static estimator_t *estimator(avr_model_t *m, model_key_t key) {
  if (m->count * 2 >= m->cap) {
    size_t oc = m->cap;
    model_key_t *ok = m->keys;
    estimator_t *ov = m->vals;
    uint8_t *ou = m->used;
    m->cap *= 2;
    m->keys = (model_key_t *)malloc(m->cap * sizeof(model_key_t));
    m->vals = (estimator_t *)malloc(m->cap * sizeof(estimator_t));
    m->used = (uint8_t *)calloc(m->cap, 1);
    for (size_t i = 0; i < oc; i++) {
      if (!ou[i]) continue;
      size_t j = hash_key(ok[i]) & (m->cap - 1);
      while (m->used[j]) j = (j + 1) & (m->cap - 1);
      m->used[j] = 1;
      m->keys[j] = ok[i];
      m->vals[j] = ov[i];
    }
    free(ok);
    free(ov);
    free(ou);
  }
  size_t j = hash_key(key) & (m->cap - 1);
  while (m->used[j]) {
    if (m->keys[j] == key) return &m->vals[j];
    j = (j + 1) & (m->cap - 1);
  }
  m->used[j] = 1;
  m->keys[j] = key;
  m->vals[j].pos = 1; /* struct estimator { int pos = 1, neg = 1; } (recode.cpp:1057) */
  m->vals[j].neg = 1;
  if (prior_on() && default_kind(key) && g_prior[key >> 48][0]) {
    m->vals[j].pos = g_prior[key >> 48][0];
    m->vals[j].neg = g_prior[key >> 48][1];
  }
  m->count++;
  return &m->vals[j];
}

/* --------------------------------------------------------------------- get_model_key (676-815) */
static const uint8_t sig_coeff_flag_offset_8x8_frame[63] = { /* recode.cpp:686-690 */
  0, 1, 2, 3, 4, 5, 5, 4, 4, 3, 3, 4, 4, 4, 5, 5, 4, 4, 4, 4, 3, 3, 6, 7, 7, 7, 8, 9, 10, 9, 8, 7,
  7, 6, 11, 12, 13, 11, 6, 7, 8, 9, 14, 10, 9, 8, 6, 11, 12, 13, 11, 6, 9, 14, 10, 9, 11, 12, 13, 11, 14, 10, 12};
static const int cat_lookup[14] = {105 + 0, 105 + 15, 105 + 29, 105 + 44, 105 + 47, 402, 484 + 0,
                                   484 + 15, 484 + 29, 660, 528 + 0, 528 + 15, 528 + 29, 718}; /* 696 */
static const uint8_t sig_coeff_offset_dc[7] = {0, 0, 1, 1, 2, 2, 2};                 /* 697 */

model_key_t model_get_key(avr_model_t *m, int ctx_kind) {
  switch (m->coding_type) {
    case PIP_SIGNIFICANCE_NZ:
    case PIP_UNKNOWN:
    case PIP_UNREACHABLE:
    case PIP_RESIDUALS:
      return mk_key(ctx_kind, 0, 0);
    case PIP_SIGNIFICANCE_MAP: {
      int zigzag_offset = m->zigzag_index;
      if (m->sub_mb_is_dc && m->sub_mb_chroma422) {
        zigzag_offset = sig_coeff_offset_dc[m->zigzag_index];
      } else if (m->sub_mb_size > 32) {
        zigzag_offset = sig_coeff_flag_offset_8x8_frame[m->zigzag_index];
      }
      int nnz = model_meta(m, m->cur_frame, m->mb_x, m->mb_y)->num_nonzeros[m->scan8_index];
      return mk_key(K_SIGNIF, 64 * nnz + m->nonzeros_observed,
                    m->sub_mb_is_dc + zigzag_offset * 2 + 16 * 2 * cat_lookup[m->sub_mb_cat]);
    }
    case PIP_SIGNIFICANCE_EOB: {
      int nnz = model_meta(m, m->cur_frame, m->mb_x, m->mb_y)->num_nonzeros[m->scan8_index];
      return mk_key(K_FAKE_EOB, nnz == m->nonzeros_observed, 0);
    }
    default:
      abort(); /* "Unreachable" (recode.cpp:813-814) */
  }
}

/* Analysis aid (test infrastructure): AVR_ORACLE_KEYLOG=<file> appends every probability query's
 * model key (u64) to <file>; used offline to size the device's estimator cache. */
static FILE *keylog_file(void) {
  static int init;
  static FILE *f;
  if (!init) {
    init = 1;
    const char *p = getenv("AVR_ORACLE_KEYLOG");
    if (p && *p) f = fopen(p, "wb");
  }
  return f;
}

/* probability_for_model_key (816-820) */
uint64_t model_p1(avr_model_t *m, uint64_t range, model_key_t key) {
  FILE *kl = keylog_file();
  if (kl) fwrite(&key, sizeof(key), 1, kl);
  estimator_t *e = estimator(m, key);
  return m->p32 ? pc_p1((uint32_t)range, e->pos, e->neg) : rc_p1(range, e->pos, e->neg);
}

/* update_frame_spec (824-843) */
void model_update_frame_spec(avr_model_t *m, int frame_num, int mb_width, int mb_height) {
  framebuf_t *f = m->frames;
  int c = m->cur_frame;
  if (f[c].width != (uint32_t)mb_width || f[c].height != (uint32_t)mb_height ||
      !(f[c].frame_num == frame_num && f[c].width && f[c].height)) {
    c = m->cur_frame = !m->cur_frame;
    if (f[c].width != (uint32_t)mb_width || f[c].height != (uint32_t)mb_height) {
      fb_init(&f[c], (uint32_t)mb_width, (uint32_t)mb_height);
      if (f[!c].width != (uint32_t)mb_width || f[!c].height != (uint32_t)mb_height)
        fb_init(&f[!c], (uint32_t)mb_width, (uint32_t)mb_height);
    } else {
      fb_bzero(&f[c]);
    }
    f[c].frame_num = frame_num;
  }
}

/* finished_queueing (845-930).  cb is the compressor's put or the decompressor's get lambda. */
void model_finished_queueing(avr_model_t *m, int ct, nz_cb_t cb, void *ctx) {
  if (ct != PIP_SIGNIFICANCE_MAP) return;
  int last = m->coding_type;
  m->coding_type = PIP_SIGNIFICANCE_NZ;
  blockmeta_t *meta = model_meta(m, m->cur_frame, m->mb_x, m->mb_y);
  int nonzero_bits[6];
  for (int i = 0; i < 6; i++) nonzero_bits[i] = (meta->num_nonzeros[m->scan8_index] & (1 << i)) >> i;
  const uint32_t serialized_bits = m->sub_mb_size > 16 ? 6 : m->sub_mb_size > 4 ? 4 : 2;
  uint32_t serialized_so_far = 0, left_nonzero = 0, above_nonzero = 0;
  int nx, ny, nidx;
  int has_left = get_neighbor_sub_mb(0, m->sub_mb_size, m->mb_x, m->mb_y, m->scan8_index, &nx, &ny, &nidx);
  if (has_left) left_nonzero = model_meta(m, m->cur_frame, nx, ny)->num_nonzeros[nidx];
  int has_above = get_neighbor_sub_mb(1, m->sub_mb_size, m->mb_x, m->mb_y, m->scan8_index, &nx, &ny, &nidx);
  if (has_above) above_nonzero = model_meta(m, m->cur_frame, nx, ny)->num_nonzeros[nidx];
  /* DEVIATION (3): the compressor calls this after end_coding_type has set is_8x8 for the current
   * block (recode.cpp:1208-1212), the decompressor before it (recode.cpp:1478-1480).  The
   * reference therefore keys the first 8x8 block of every macroblock differently on the two sides
   * and cannot decode its own output for 8x8-transform streams.  The compressor side (whose output
   * is the container) is kept verbatim; the decompressor reproduces the compressor's key. */
  int is_8x8 = meta->is_8x8 || (m->decompress_side && m->sub_mb_size > 32 && !getenv("AVR_REFERENCE_8X8_BUG"));
  uint32_t i = 0;
  do {
    uint32_t cur_bit = 1u << i;
    int left_bit = 2;
    if (has_left) left_bit = left_nonzero >= cur_bit;
    int above_bit = 2;
    if (above_nonzero) above_bit = above_nonzero >= cur_bit; /* sic: not has_above (881) */
    int prev = model_meta(m, !m->cur_frame, m->mb_x, m->mb_y)->num_nonzeros[m->scan8_index] >= cur_bit;
    model_key_t key = mk_key(K_NZBIT + (int)i, (int)serialized_so_far + 64 * prev + 128 * left_bit + 384 * above_bit,
                             is_8x8 + m->sub_mb_is_dc * 2 + m->sub_mb_chroma422 + m->sub_mb_cat * 4);
    cb(ctx, m, key, &nonzero_bits[i]);
    if (nonzero_bits[i]) serialized_so_far |= cur_bit;
  } while (++i < serialized_bits);
  (void)has_above;
  meta->num_nonzeros[m->scan8_index] = 0;
  for (int k = 0; k < 6; k++) meta->num_nonzeros[m->scan8_index] |= (uint8_t)(nonzero_bits[k] << k);
  m->coding_type = last;
}

/* end_coding_type (931-950) */
void model_end_coding_type(avr_model_t *m, int ct) {
  if (ct == PIP_SIGNIFICANCE_MAP) {
    uint8_t num_nonzeros = 0;
    mbblock_t *b = model_block(m, m->mb_x, m->mb_y);
    for (int i = 0; i < m->sub_mb_size; i++)
      if (b->residual[m->scan8_index * 16 + i] != 0) num_nonzeros++;
    blockmeta_t *meta = model_meta(m, m->cur_frame, m->mb_x, m->mb_y);
    meta->is_8x8 = meta->is_8x8 || (m->sub_mb_size > 32);
    meta->coded = 1;
    meta->num_nonzeros[m->scan8_index] = num_nonzeros;
  }
  m->coding_type = PIP_UNKNOWN;
}

/* begin_coding_type (951-974) */
int model_begin_coding_type(avr_model_t *m, int ct) {
  int begin_queueing = 0;
  m->coding_type = ct;
  if (ct == PIP_SIGNIFICANCE_MAP) {
    model_meta(m, m->cur_frame, m->mb_x, m->mb_y)->num_nonzeros[m->scan8_index] = 0;
    m->nonzeros_observed = 0;
    m->zigzag_index = 0;
    begin_queueing = 1;
  }
  return begin_queueing;
}

/* reset_mb_significance_state_tracking (975-979) */
void model_reset_sig_tracking(avr_model_t *m) {
  m->zigzag_index = 0;
  m->nonzeros_observed = 0;
  m->coding_type = PIP_SIGNIFICANCE_MAP;
}

/* update_state_tracking (980-1026) */
void model_update_tracking(avr_model_t *m, int symbol) {
  mbblock_t *b;
  switch (m->coding_type) {
    case PIP_SIGNIFICANCE_NZ:
      break;
    case PIP_SIGNIFICANCE_MAP:
      b = model_block(m, m->mb_x, m->mb_y);
      b->residual[m->scan8_index * 16 + m->zigzag_index] = (uint16_t)symbol;
      m->nonzeros_observed += symbol;
      if (m->zigzag_index + 1 == m->sub_mb_size) {
        m->coding_type = PIP_UNREACHABLE;
        m->zigzag_index = 0;
      } else if (symbol) {
        m->coding_type = PIP_SIGNIFICANCE_EOB;
      } else {
        ++m->zigzag_index;
        if (m->zigzag_index + 1 == m->sub_mb_size) {
          b->residual[m->scan8_index * 16 + m->zigzag_index] = 1;
          ++m->nonzeros_observed;
          m->coding_type = PIP_UNREACHABLE;
          m->zigzag_index = 0;
        }
      }
      break;
    case PIP_SIGNIFICANCE_EOB:
      b = model_block(m, m->mb_x, m->mb_y);
      if (symbol) {
        m->zigzag_index = 0;
        m->coding_type = PIP_UNREACHABLE;
      } else if (m->zigzag_index + 2 == m->sub_mb_size) {
        b->residual[m->scan8_index * 16 + m->zigzag_index + 1] = 1;
        m->coding_type = PIP_UNREACHABLE;
      } else {
        m->coding_type = PIP_SIGNIFICANCE_MAP;
        ++m->zigzag_index;
      }
      break;
    case PIP_RESIDUALS:
    case PIP_UNKNOWN:
      break;
    default:
      abort(); /* PIP_UNREACHABLE: assert(false) (1021-1024) */
  }
}

/* update_state_for_model_key (1030-1047) */
void model_update_key(avr_model_t *m, int symbol, model_key_t key) {
  if (m->coding_type == PIP_SIGNIFICANCE_EOB) {
    int nnz = model_meta(m, m->cur_frame, m->mb_x, m->mb_y)->num_nonzeros[m->scan8_index];
    if (symbol != (nnz == m->nonzeros_observed)) abort(); /* assert (1033) */
  }
  estimator_t *e = estimator(m, key);
  if (stats_on() && default_kind(key)) g_stats[key >> 48][symbol != 0]++;
  if (symbol) e->pos++;
  else e->neg++;
  if ((m->coding_type != PIP_SIGNIFICANCE_MAP && e->pos + e->neg > 0x60) ||
      (m->coding_type == PIP_SIGNIFICANCE_MAP && e->pos + e->neg > 0x50)) {
    e->pos = (e->pos + 1) / 2;
    e->neg = (e->neg + 1) / 2;
  }
  model_update_tracking(m, symbol);
}

void model_update_state(avr_model_t *m, int symbol, int ctx_kind) {
  model_update_key(m, symbol, model_get_key(m, ctx_kind));
}
