/*
 * Oracle: CABAC slice_data() walker.  TEST INFRASTRUCTURE ONLY (see avr_oracle.h).
 *
 * This is the part of the libavcodec-hooks FFmpeg fork that CALLS the reference's hot path: the
 * H.264 CABAC syntax parse (FFmpeg libavcodec/h264_cabac.c ff_h264_decode_mb_cabac and helpers,
 * ITU-T H.264 7.3.4 slice_data, 7.3.5 macroblock_layer, 9.3.3.1 ctxIdxInc derivations).  The fork
 * is an un-vendored submodule (.gitmodules:1-4), so this is a restatement of the published
 * algorithm.  Every bin goes through hooks->get / get_bypass / get_terminate exactly as the fork
 * routes ff_get_cabac* through coding_hooks (recode.cpp:149-160), and the model hooks are placed as
 * the reference's asserts require (recode.cpp:185-189, 933-934, 1021-1022):
 *   mb_xy before every macroblock, begin_sub_mb/end_sub_mb around every residual block (before
 *   its coded_block_flag), begin_coding_type(SIG_MAP) immediately before the first
 *   significant_coeff_flag and end_coding_type(SIG_MAP) right after the map.
 * frame_spec is called once per slice with a decode-order picture counter.
 *
 * Supported: progressive frames, field pictures and MBAFF frames, CABAC, ChromaArrayType 0..3,
 * 8x8 transform, I/P/B slices.  I_PCM returns an error (the reference throws, recode.cpp:161-163).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "avr_oracle.h"

int avr_walk_se, avr_walk_se_bin, avr_walk_se_limit, avr_walk_mbs_done, avr_walk_last_mb;

enum {
  SE_SKIP = 1, SE_MBTYPE, SE_SUBMBTYPE, SE_T8X8, SE_PREVINTRA, SE_REMINTRA, SE_CHROMAPRED, SE_REF,
  SE_MVD_PREFIX, SE_MVD_SUFFIX, SE_CBP, SE_QPDELTA, SE_CBF, SE_SIG, SE_LAST, SE_LEVEL_PREFIX,
  SE_LEVEL_SUFFIX, SE_SIGN, SE_EOS, SE_PCM_FLAG, SE_FIELD
};

/* scan8 (recode.cpp:263-277 == FFmpeg h264dec.h scan8) */
static const uint8_t scan8[51] = {
  4 + 1 * 8,  5 + 1 * 8,  4 + 2 * 8,  5 + 2 * 8,  6 + 1 * 8,  7 + 1 * 8,  6 + 2 * 8,  7 + 2 * 8,
  4 + 3 * 8,  5 + 3 * 8,  4 + 4 * 8,  5 + 4 * 8,  6 + 3 * 8,  7 + 3 * 8,  6 + 4 * 8,  7 + 4 * 8,
  4 + 6 * 8,  5 + 6 * 8,  4 + 7 * 8,  5 + 7 * 8,  6 + 6 * 8,  7 + 6 * 8,  6 + 7 * 8,  7 + 7 * 8,
  4 + 8 * 8,  5 + 8 * 8,  4 + 9 * 8,  5 + 9 * 8,  6 + 8 * 8,  7 + 8 * 8,  6 + 9 * 8,  7 + 9 * 8,
  4 + 11 * 8, 5 + 11 * 8, 4 + 12 * 8, 5 + 12 * 8, 6 + 11 * 8, 7 + 11 * 8, 6 + 12 * 8, 7 + 12 * 8,
  4 + 13 * 8, 5 + 13 * 8, 4 + 14 * 8, 5 + 14 * 8, 6 + 13 * 8, 7 + 13 * 8, 6 + 14 * 8, 7 + 14 * 8,
  0 + 0 * 8,  0 + 5 * 8,  0 + 10 * 8,
};

/* ctxIdxOffset per ctxBlockCat (Table 9-34; frame coded) */
static const int16_t cbf_base[14] = {85, 89, 93, 97, 101, 1012, 460, 464, 468, 1016, 472, 476, 480, 1020};
static const int16_t sig_base[14] = {105 + 0, 105 + 15, 105 + 29, 105 + 44, 105 + 47, 402, 484 + 0,
                                     484 + 15, 484 + 29, 660, 528 + 0, 528 + 15, 528 + 29, 718};
static const int16_t last_base[14] = {166 + 0, 166 + 15, 166 + 29, 166 + 44, 166 + 47, 417, 572 + 0,
                                      572 + 15, 572 + 29, 690, 616 + 0, 616 + 15, 616 + 29, 748};
static const int16_t abs_base[14] = {227 + 0, 227 + 10, 227 + 20, 227 + 30, 227 + 39, 426, 952 + 0,
                                     952 + 10, 952 + 20, 708, 982 + 0, 982 + 10, 982 + 20, 766};
/* field-coded macroblocks (field pictures, MBAFF field pairs): Table 9-34's field ctxIdxOffsets
 * (FFmpeg h264_cabac.c significant_coeff_flag_offset[1] / last_coeff_flag_offset[1]) */
static const int16_t sig_base_fld[14] = {277 + 0, 277 + 15, 277 + 29, 277 + 44, 277 + 47, 436, 776 + 0,
                                         776 + 15, 776 + 29, 675, 820 + 0, 820 + 15, 820 + 29, 733};
static const int16_t last_base_fld[14] = {338 + 0, 338 + 15, 338 + 29, 338 + 44, 338 + 47, 451, 864 + 0,
                                          864 + 15, 864 + 29, 699, 908 + 0, 908 + 15, 908 + 29, 757};
/* Table 9-43 ctxIdxInc of significant_coeff_flag in 8x8 field blocks (== recode.cpp:691-694) */
static const uint8_t sig8x8_fld[63] = {
  0, 1, 1, 2, 2, 3, 3, 4, 5, 6, 7, 7, 7, 8, 4, 5, 6, 9, 10, 10, 8, 11, 12, 11, 9, 9, 10, 10, 8, 11, 12, 11,
  9, 9, 10, 10, 8, 11, 12, 11, 9, 9, 10, 10, 8, 13, 13, 9, 9, 10, 10, 8, 13, 13, 9, 9, 10, 10, 14, 14, 14, 14, 14};
/* Table 9-43 ctxIdxInc for significant / last in 8x8 frame blocks (== recode.cpp:686-690) */
static const uint8_t sig8x8[63] = {
  0, 1, 2, 3, 4, 5, 5, 4, 4, 3, 3, 4, 4, 4, 5, 5, 4, 4, 4, 4, 3, 3, 6, 7, 7, 7, 8, 9, 10, 9, 8, 7,
  7, 6, 11, 12, 13, 11, 6, 7, 8, 9, 14, 10, 9, 8, 6, 11, 12, 13, 11, 6, 9, 14, 10, 9, 11, 12, 13, 11, 14, 10, 12};
static const uint8_t last8x8[63] = {
  0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
  3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8};

typedef struct {
  uint8_t decoded, skip, intra, i16, direct16, t8x8, chroma_pred;
  uint8_t fld;             /* field macroblock (field picture, or a field pair of an MBAFF frame) */
  uint16_t cbp;            /* FFmpeg cbp_table: luma b0-3, chroma b4-5, chroma DC cbf b6-7, luma DC cbf b8-10 */
  uint8_t nnz[3][16];      /* coefficient count per 4x4 block, raster x4 + 4*y4 per plane */
  uint8_t mvd[2][16][2];   /* min(|mvd|,70) per list, raster 4x4, component */
  int8_t ref[2][4];        /* per 8x8, -1 = list not used / intra */
  uint8_t direct8[4];
} wmb_t;

typedef struct {
  const avr_slice_hdr_t *h;
  const avr_hooks_t *hk;
  uint8_t state[1024];
  wmb_t *mbs;
  int W, H;
  wmb_t *cur, *left, *top;
  int last_dqp_nz;
  int is_b;
  int err;
  int fld;           /* the current macroblock is field coded (field picture, or an MBAFF field pair) */
  /* MBAFF (FFmpeg FRAME_MBAFF): mbs is indexed by frame macroblock (x + frame row * W), pairs of
   * a top and a bottom macroblock; neighbours follow ITU-T H.264 Table 6-4 (6.4.12.2) */
  int mbaff, x, pr, bottom;
  wmb_t *lpair, *apair;   /* top macroblocks of the left / upper pair when in the slice, else NULL */
} walker_t;

/* ---------------------------------------------------------------- neighbours (6.4.11, 6.4.12) */
/* The macroblock holding the left neighbour of row yN (luma or chroma samples, maxH rows) of the
 * current macroblock, and that row (*yM) in it: mbAddrA of Table 6-4 for xN < 0.  Progressive
 * and field pictures: the macroblock to the left, same row. */
static wmb_t *nb_left(walker_t *w, int yN, int maxH, int *yM) {
  *yM = yN;
  if (!w->mbaff) return w->left;
  if (!w->lpair) return NULL;
  wmb_t *T = w->lpair, *B = w->lpair + w->W;
  const int afrm = !T->fld;
  if (!w->cur->fld) {   /* frame macroblock */
    if (afrm) return w->bottom ? B : T;
    *yM = w->bottom ? (yN + maxH) >> 1 : yN >> 1;
    return (yN & 1) ? B : T;
  }
  if (afrm) {           /* field macroblock, frame pair to the left */
    const int y2 = (yN << 1) + w->bottom;
    if (yN < maxH / 2) { *yM = y2; return T; }
    *yM = y2 - maxH;
    return B;
  }
  return w->bottom ? B : T;
}
/* mbAddrB of Table 6-4 (yN < 0): the macroblock above; its bottom row is the neighbour row */
static wmb_t *nb_above(walker_t *w) {
  if (!w->mbaff) return w->top;
  if (!w->cur->fld) {
    if (w->bottom) return w->cur - w->W;   /* the top macroblock of this pair */
    return w->apair ? w->apair + w->W : NULL;
  }
  if (!w->apair) return NULL;
  if (w->bottom) return w->apair + w->W;
  return w->apair->fld ? w->apair : w->apair + w->W;
}
/* the macroblock neighbours A / B of 6.4.11.1 (luma locations (-1, 0) and (0, -1)) */
static wmb_t *mb_a(walker_t *w) {
  int yM;
  return nb_left(w, 0, 16, &yM);
}
/* A neighbour's ref_idx / vertical |mvd| as seen from the current macroblock (FFmpeg
 * fill_decode_caches MAP_F2F: a frame neighbour of a field macroblock counts double references
 * and half the vertical motion, a field neighbour of a frame macroblock the opposite;
 * 9.3.3.1.1.6-7) */
static int nb_ref(const walker_t *w, const wmb_t *m, int list, int b8) {
  int r = m->ref[list][b8];
  if (w->mbaff && r >= 0 && m->fld != w->cur->fld) r = w->cur->fld ? r * 2 : r >> 1;
  return r;
}
static int nb_mvd(const walker_t *w, const wmb_t *m, int list, int idx, int comp) {
  int v = m->mvd[list][idx][comp];
  if (w->mbaff && comp == 1 && m->fld != w->cur->fld) v = w->cur->fld ? v >> 1 : v << 1;
  return v;
}

static inline int bin(walker_t *w, int se, int k, int ctx) {
  avr_walk_se = se;
  avr_walk_se_bin = k;
  return w->hk->get(w->hk->opaque, &w->state[ctx], ctx);
}
static inline int byp(walker_t *w, int se, int k) {
  avr_walk_se = se;
  avr_walk_se_bin = k;
  return w->hk->get_bypass(w->hk->opaque);
}
static inline int term(walker_t *w, int se) {
  avr_walk_se = se;
  avr_walk_se_bin = 0;
  return w->hk->get_terminate(w->hk->opaque);
}
static inline int imin(int a, int b) { return a < b ? a : b; }

/* ---------------------------------------------------------------------------- mb_type */
typedef struct {
  int intra, i16, pcm, i16_pred, i16_cbp;  /* i16_cbp: luma(0/15) | chroma<<4 */
  int nparts;                              /* 1, 2 or 4 (8x8 sub-macroblocks) */
  int vertical;                            /* 2 partitions: 0 = 16x8, 1 = 8x16 */
  int pred[2];                             /* 1 = L0, 2 = L1, 3 = Bi */
  int direct16;
} mbtype_t;

/* decode_cabac_intra_mb_type (I: ctxIdxOffset 3; P prefix 17; B prefix 32) */
static int intra_mb_type(walker_t *w, int base, int intra_slice, mbtype_t *t) {
  memset(t, 0, sizeof(*t));
  t->intra = 1;
  int ctx = 0;
  if (intra_slice) {
    const wmb_t *a = mb_a(w), *b = nb_above(w);
    if (a && a->i16) ctx++;  /* condTerm: available && mb_type != I_NxN */
    if (b && b->i16) ctx++;
    if (!bin(w, SE_MBTYPE, 0, base + ctx)) return 0; /* I_NxN */
    base += 2;
  } else {
    if (!bin(w, SE_MBTYPE, 0, base)) return 0;
  }
  if (term(w, SE_PCM_FLAG)) { t->pcm = 1; return 0; }
  t->i16 = 1;
  int cbp_luma = bin(w, SE_MBTYPE, 2, base + 1) ? 15 : 0;
  int chroma = 0;
  if (bin(w, SE_MBTYPE, 3, base + 2)) chroma = 1 + bin(w, SE_MBTYPE, 4, base + 2 + intra_slice);
  int pred = 2 * bin(w, SE_MBTYPE, 5, base + 3 + intra_slice);
  pred += bin(w, SE_MBTYPE, 6, base + 3 + 2 * intra_slice);
  t->i16_pred = pred;
  t->i16_cbp = cbp_luma | (chroma << 4);
  return 0;
}

static const uint8_t b_pairs[9][2] = {{1, 1}, {2, 2}, {1, 2}, {2, 1}, {1, 3}, {2, 3}, {3, 1}, {3, 2}, {3, 3}};

static void decode_mb_type(walker_t *w, mbtype_t *t) {
  const avr_slice_hdr_t *h = w->h;
  memset(t, 0, sizeof(*t));
  if (h->slice_type == AVR_SLICE_I) {
    intra_mb_type(w, 3, 1, t);
    return;
  }
  if (h->slice_type == AVR_SLICE_P) {
    if (!bin(w, SE_MBTYPE, 0, 14)) {
      int mt;
      if (!bin(w, SE_MBTYPE, 1, 15)) mt = 3 * bin(w, SE_MBTYPE, 2, 16);   /* 16x16 / 8x8 */
      else mt = 2 - bin(w, SE_MBTYPE, 2, 17);                           /* 8x16 / 16x8 */
      if (mt == 0) { t->nparts = 1; t->pred[0] = 1; }
      else if (mt == 1) { t->nparts = 2; t->vertical = 0; t->pred[0] = t->pred[1] = 1; }
      else if (mt == 2) { t->nparts = 2; t->vertical = 1; t->pred[0] = t->pred[1] = 1; }
      else t->nparts = 4;
      return;
    }
    intra_mb_type(w, 17, 0, t);
    return;
  }
  /* B */
  int ctx = 0;
  const wmb_t *a = mb_a(w), *b = nb_above(w);
  if (a && !a->direct16) ctx++;  /* condTerm: available && not B_Skip/B_Direct_16x16 */
  if (b && !b->direct16) ctx++;
  if (!bin(w, SE_MBTYPE, 0, 27 + ctx)) { t->direct16 = 1; t->nparts = 4; return; }
  if (!bin(w, SE_MBTYPE, 1, 27 + 3)) {
    t->nparts = 1;
    t->pred[0] = 1 + bin(w, SE_MBTYPE, 2, 27 + 5);
    return;
  }
  int bits = bin(w, SE_MBTYPE, 2, 27 + 4) << 3;
  bits |= bin(w, SE_MBTYPE, 3, 27 + 5) << 2;
  bits |= bin(w, SE_MBTYPE, 4, 27 + 5) << 1;
  bits |= bin(w, SE_MBTYPE, 5, 27 + 5);
  int mt;
  if (bits < 8) mt = bits + 3;
  else if (bits == 13) { intra_mb_type(w, 32, 0, t); return; }
  else if (bits == 14) mt = 11;
  else if (bits == 15) mt = 22;
  else { bits = (bits << 1) | bin(w, SE_MBTYPE, 6, 27 + 5); mt = bits - 4; }
  if (mt == 3) { t->nparts = 1; t->pred[0] = 3; return; }
  if (mt == 22) { t->nparts = 4; return; }
  int k = mt - 4;
  t->nparts = 2;
  t->vertical = k & 1;
  t->pred[0] = b_pairs[k >> 1][0];
  t->pred[1] = b_pairs[k >> 1][1];
}

/* sub_mb_type: returns parts (1,2,4), shape (0 = 8x4 / 1 = 4x8 when 2 parts), pred, direct */
typedef struct { int nparts, vertical, pred, direct; } submb_t;
static void decode_sub_mb_type(walker_t *w, submb_t *s) {
  memset(s, 0, sizeof(*s));
  if (!w->is_b) {
    int t;
    if (bin(w, SE_SUBMBTYPE, 0, 21)) t = 0;
    else if (!bin(w, SE_SUBMBTYPE, 1, 22)) t = 1;
    else if (bin(w, SE_SUBMBTYPE, 2, 23)) t = 2;
    else t = 3;
    s->pred = 1;
    s->nparts = t == 0 ? 1 : t == 3 ? 4 : 2;
    s->vertical = t == 2;
    return;
  }
  int t;
  if (!bin(w, SE_SUBMBTYPE, 0, 36)) t = 0;
  else if (!bin(w, SE_SUBMBTYPE, 1, 37)) t = 1 + bin(w, SE_SUBMBTYPE, 2, 39);
  else {
    t = 3;
    if (bin(w, SE_SUBMBTYPE, 2, 38)) {
      if (bin(w, SE_SUBMBTYPE, 3, 39)) t = 11 + bin(w, SE_SUBMBTYPE, 4, 39);
      else {
        t += 4;
        t += 2 * bin(w, SE_SUBMBTYPE, 4, 39);
        t += bin(w, SE_SUBMBTYPE, 5, 39);
      }
    } else {
      t += 2 * bin(w, SE_SUBMBTYPE, 3, 39);
      t += bin(w, SE_SUBMBTYPE, 4, 39);
    }
  }
  if (t == 0) { s->direct = 1; s->nparts = 1; return; }
  if (t <= 3) { s->nparts = 1; s->pred = t; return; }
  if (t <= 9) { int k = t - 4; s->nparts = 2; s->vertical = k & 1; s->pred = (k >> 1) + 1; return; }
  s->nparts = 4;
  s->pred = t - 9;
}

/* ------------------------------------------------------------------------ ref / mvd */
static int ref_neighbor_gt0(walker_t *w, int list, int x4, int y4, int left) {
  const wmb_t *m;
  int b8, yM;
  if (left) {
    if (x4 > 0) { m = w->cur; b8 = (y4 >> 1) * 2 + ((x4 - 1) >> 1); }
    else { m = nb_left(w, 4 * y4, 16, &yM); b8 = (yM >> 3) * 2 + 1; }
  } else {
    if (y4 > 0) { m = w->cur; b8 = ((y4 - 1) >> 1) * 2 + (x4 >> 1); }
    else { m = nb_above(w); b8 = 2 + (x4 >> 1); }
  }
  if (!m) return 0;
  if (w->is_b && m->direct8[b8]) return 0;
  return nb_ref(w, m, list, b8) > 0;
}

static int decode_ref(walker_t *w, int list, int x4, int y4) {
  int ctx = ref_neighbor_gt0(w, list, x4, y4, 1) + 2 * ref_neighbor_gt0(w, list, x4, y4, 0);
  int ref = 0;
  /* an MBAFF field macroblock addresses each reference field: twice the references (FFmpeg
   * ref_count << MB_MBAFF) */
  avr_walk_se_limit = (w->h->num_ref_idx_active[list] << (w->mbaff && w->cur->fld)) - 1;
  while (bin(w, SE_REF, ref, 54 + ctx)) {
    ref++;
    ctx = (ctx >> 2) + 4;
    if (ref >= 32) { w->err = -3; return 0; }
  }
  return ref;
}

static int mvd_neighbor(walker_t *w, int list, int comp, int x4, int y4, int left) {
  if (left) {
    if (x4 > 0) return w->cur->mvd[list][y4 * 4 + x4 - 1][comp];
    int yM;
    const wmb_t *m = nb_left(w, 4 * y4, 16, &yM);
    return m ? nb_mvd(w, m, list, (yM >> 2) * 4 + 3, comp) : 0;
  }
  if (y4 > 0) return w->cur->mvd[list][(y4 - 1) * 4 + x4][comp];
  const wmb_t *m = nb_above(w);
  return m ? nb_mvd(w, m, list, 12 + x4, comp) : 0;
}

/* decode_cabac_mb_mvd: ctxIdxOffset 40 (x) / 47 (y); returns |mvd| clipped to 70 */
static int decode_mvd(walker_t *w, int list, int comp, int x4, int y4) {
  int base = comp ? 47 : 40;
  int amvd = mvd_neighbor(w, list, comp, x4, y4, 1) + mvd_neighbor(w, list, comp, x4, y4, 0);
  int inc = amvd < 3 ? 0 : amvd <= 32 ? 1 : 2;
  if (!bin(w, SE_MVD_PREFIX, 0, base + inc)) return 0;
  int mvd = 1;
  int ctx = base + 3;
  while (mvd < 9 && bin(w, SE_MVD_PREFIX, mvd, ctx)) {
    if (mvd < 4) ctx++;
    mvd++;
  }
  if (mvd >= 9) {
    int k = 3;
    while (byp(w, SE_MVD_SUFFIX, k - 3)) {
      mvd += 1 << k;
      k++;
      if (k > 24) { w->err = -4; return 0; }
    }
    while (k--) mvd += byp(w, SE_MVD_SUFFIX, 100) << k;
  }
  byp(w, SE_SIGN, 0);
  return mvd < 70 ? mvd : 70;
}

static void fill_mvd(wmb_t *m, int list, int x4, int y4, int pw, int ph, int mx, int my) {
  for (int y = y4; y < y4 + ph; y++)
    for (int x = x4; x < x4 + pw; x++) {
      m->mvd[list][y * 4 + x][0] = (uint8_t)mx;
      m->mvd[list][y * 4 + x][1] = (uint8_t)my;
    }
}

/* ------------------------------------------------------------------------ residual */
/* FFmpeg ff_h264_decode_mb_cabac, CHROMA444 && IS_8x8DCT: a neighbour macroblock that does not
 * use the 8x8 transform contributes (x264_build < 151 ? intra ? 64 : 0 : 0) — the x264 < r151
 * 4:4:4 coded_block_flag behaviour FFmpeg reproduces for such streams. */
static int nnz_444_8x8_override(walker_t *w, const wmb_t *nb, int *v) {
  if (w->h->chroma_array_type != 3 || !w->cur->t8x8 || nb->t8x8) return 0;
  unsigned build = (unsigned)w->h->x264_build;
  *v = build < 151u ? (w->cur->intra ? 64 : 0) : 0;
  return 1;
}
static int nnz_at(walker_t *w, int p, int pw, int ph, int x4, int y4, int left) {
  int v;
  if (left) {
    if (x4 > 0) return w->cur->nnz[p][y4 * 4 + x4 - 1];
    int yM;   /* rows of 4x4 blocks: 4 y4 samples of a plane 4 ph high */
    const wmb_t *m = nb_left(w, 4 * y4, 4 * ph, &yM);
    if (!m) return w->cur->intra ? 64 : 0;
    if (nnz_444_8x8_override(w, m, &v)) return v;
    return m->nnz[p][(yM >> 2) * 4 + pw - 1];
  }
  if (y4 > 0) return w->cur->nnz[p][(y4 - 1) * 4 + x4];
  const wmb_t *m = nb_above(w);
  if (!m) return w->cur->intra ? 64 : 0;
  if (nnz_444_8x8_override(w, m, &v)) return v;
  return m->nnz[p][(ph - 1) * 4 + x4];
}

static uint16_t nb_cbp(walker_t *w, const wmb_t *m) {
  if (m) return m->cbp;
  return w->cur->intra ? 0x7CF : 0x00F;
}
/* the left neighbours' coded_block_pattern as FFmpeg's left_cbp: chroma and DC bits of A, luma
 * bit 1 from the 8x8 block left of the current 8x8 block 0, bit 3 left of block 2 (6.4.11.2) */
static uint16_t nb_cbp_left(walker_t *w) {
  int y0, y2;
  const wmb_t *m0 = nb_left(w, 0, 16, &y0), *m2 = nb_left(w, 8, 16, &y2);
  const uint16_t c0 = nb_cbp(w, m0), c2 = nb_cbp(w, m2);
  return (uint16_t)((c0 & 0x7F0) | (((c0 >> ((y0 >> 3) * 2 + 1)) & 1) << 1) | (((c2 >> ((y2 >> 3) * 2 + 1)) & 1) << 3));
}

/* one residual_block_cabac(); n = FFmpeg block index (scan8 index), p/x4/y4 its position */
static void residual_block(walker_t *w, int cat, int n, int max, int is_dc, int chroma422, int p, int pw,
                           int ph, int x4, int y4) {
  const avr_hooks_t *hk = w->hk;
  if (w->err) return;
  hk->begin_sub_mb(hk->opaque, cat, n, max, is_dc, chroma422);
  int coded = 1;
  if (max != 64 || w->h->chroma_array_type == 3) {
    int nza, nzb;
    if (is_dc) {
      int bit = cat == 3 ? (0x40 << (n - 49)) : (0x100 << (n - 48));
      nza = (nb_cbp(w, mb_a(w)) & bit) != 0;
      nzb = (nb_cbp(w, nb_above(w)) & bit) != 0;
    } else {
      nza = nnz_at(w, p, pw, ph, x4, y4, 1) > 0;
      nzb = nnz_at(w, p, pw, ph, x4, y4, 0) > 0;
    }
    coded = bin(w, SE_CBF, 0, cbf_base[cat] + nza + 2 * nzb);
  }
  int cnt = 0;
  if (coded) {
    int numc8x8 = w->h->chroma_array_type == 2 ? 2 : 1;
    hk->begin_coding_type(hk->opaque, PIP_SIGNIFICANCE_MAP, 0, 0, 0);
    int last;
    for (last = 0; last < max - 1; last++) {
      int sctx, lctx;
      if (max == 64) { sctx = w->fld ? sig8x8_fld[last] : sig8x8[last]; lctx = last8x8[last]; }
      else if (cat == 3) { sctx = lctx = imin(last / numc8x8, 2); }
      else sctx = lctx = last;
      if (bin(w, SE_SIG, last, (w->fld ? sig_base_fld : sig_base)[cat] + sctx)) {
        cnt++;  /* only the count matters: levels are coded in reverse scan order */
        if (bin(w, SE_LAST, last, (w->fld ? last_base_fld : last_base)[cat] + lctx)) { last = max; break; }
      }
    }
    if (last == max - 1) cnt++;
    hk->end_coding_type(hk->opaque, PIP_SIGNIFICANCE_MAP);
    int gt1 = 0, eq1 = 0;
    for (int i = cnt - 1; i >= 0 && !w->err; i--) {
      int absl;
      if (!bin(w, SE_LEVEL_PREFIX, 0, abs_base[cat] + (gt1 ? 0 : imin(4, 1 + eq1)))) {
        absl = 1;
      } else {
        int c1 = abs_base[cat] + 5 + imin(4 - (cat == 3), gt1);
        absl = 2;
        while (absl < 15 && bin(w, SE_LEVEL_PREFIX, absl - 1, c1)) absl++;
        if (absl >= 15) {
          int k = 0;
          while (byp(w, SE_LEVEL_SUFFIX, k)) {
            if (++k > 30) { w->err = -5; break; }
          }
          int v = 1;
          while (k-- > 0) v += v + byp(w, SE_LEVEL_SUFFIX, 100);
          absl = 14 + v;
        }
      }
      byp(w, SE_SIGN, 0);
      if (absl == 1) eq1++;
      else gt1++;
    }
  }
  if (is_dc) {
    if (cnt) w->cur->cbp |= (uint16_t)(cat == 3 ? (0x40 << (n - 49)) : (0x100 << (n - 48)));
  } else if (max == 64) {
    for (int dy = 0; dy < 2; dy++)
      for (int dx = 0; dx < 2; dx++) w->cur->nnz[p][(y4 + dy) * 4 + x4 + dx] = (uint8_t)cnt;
  } else {
    w->cur->nnz[p][y4 * 4 + x4] = (uint8_t)cnt;
  }
  hk->end_sub_mb(hk->opaque, cat, n, max, is_dc, chroma422);
}

static void blk_pos(int n, int *x4, int *y4) {
  int s = scan8[n];
  int row = s >> 3;
  *x4 = (s & 7) - 4;
  *y4 = row <= 4 ? row - 1 : row <= 9 ? row - 6 : row - 11;
}

static void luma_residual(walker_t *w, int p, const mbtype_t *t, int cbp) {
  static const int cat_dc[3] = {0, 6, 10}, cat_ac[3] = {1, 7, 11}, cat_4x4[3] = {2, 8, 12}, cat_8x8[3] = {5, 9, 13};
  int x4, y4;
  if (t->i16) {
    residual_block(w, cat_dc[p], 48 + p, 16, 1, 0, p, 4, 4, 0, 0);
    if (cbp & 15) {
      for (int i = 0; i < 16; i++) {
        blk_pos(16 * p + i, &x4, &y4);
        residual_block(w, cat_ac[p], 16 * p + i, 15, 0, 0, p, 4, 4, x4, y4);
      }
    }
    return;
  }
  for (int i8 = 0; i8 < 4; i8++) {
    if (!(cbp & (1 << i8))) continue;
    if (w->cur->t8x8) {
      blk_pos(16 * p + 4 * i8, &x4, &y4);
      residual_block(w, cat_8x8[p], 16 * p + 4 * i8, 64, 0, 0, p, 4, 4, x4, y4);
    } else {
      for (int i4 = 0; i4 < 4; i4++) {
        int n = 16 * p + 4 * i8 + i4;
        blk_pos(n, &x4, &y4);
        residual_block(w, cat_4x4[p], n, 16, 0, 0, p, 4, 4, x4, y4);
      }
    }
  }
}

static void residual(walker_t *w, const mbtype_t *t, int cbp) {
  int cat_ = w->h->chroma_array_type;
  luma_residual(w, 0, t, cbp);
  if (cat_ == 3) {
    luma_residual(w, 1, t, cbp);
    luma_residual(w, 2, t, cbp);
  } else if (cat_ == 1 || cat_ == 2) {
    int c422 = cat_ == 2;
    int ph = c422 ? 4 : 2;
    if (cbp & 0x30) {
      for (int c = 0; c < 2; c++) residual_block(w, 3, 49 + c, c422 ? 8 : 4, 1, c422, 1 + c, 2, ph, 0, 0);
    }
    if (cbp & 0x20) {
      for (int c = 0; c < 2; c++) {
        for (int i8 = 0; i8 < (c422 ? 2 : 1); i8++) {
          for (int i = 0; i < 4; i++) {
            int n = 16 + 16 * c + 8 * i8 + i;
            int x4, y4;
            blk_pos(n, &x4, &y4);
            residual_block(w, 4, n, 15, 0, 0, 1 + c, 2, ph, x4, y4);
          }
        }
      }
    }
  }
}

/* ------------------------------------------------------------------------ macroblock */
/* a skipped macroblock (P_Skip / B_Skip) */
static void mb_skipped(walker_t *w) {
  wmb_t *cur = w->cur;
  cur->skip = 1;
  if (w->is_b) {
    cur->direct16 = 1;
    memset(cur->direct8, 1, 4);
  } else {
    memset(cur->ref[0], 0, 4);
  }
  w->last_dqp_nz = 0;
}

static void decode_mb_layer(walker_t *w);
static void decode_mb(walker_t *w) {
  const avr_slice_hdr_t *h = w->h;
  memset(w->cur->ref, -1, sizeof(w->cur->ref));
  if (h->slice_type != AVR_SLICE_I) {
    int ctx = (w->left && !w->left->skip) + (w->top && !w->top->skip);
    if (bin(w, SE_SKIP, 0, (w->is_b ? 24 : 11) + ctx)) {
      mb_skipped(w);
      return;
    }
  }
  decode_mb_layer(w);
}

/* MBAFF (FFmpeg h264_cabac.c decode_cabac_mb_skip): mb_skip_flag's neighbours A / B of the top
 * (bottom = 0) or bottom macroblock of the current pair when the pair is field (fld) or frame
 * coded -- fld may still be the inferred value (7.4.4) */
static int skip_ctx_mbaff(walker_t *w, int bottom, int fld) {
  const wmb_t *a = NULL, *b = NULL;
  const wmb_t *T = w->mbs + w->x + 2 * w->pr * w->W;
  if (w->lpair) a = (bottom && fld == w->lpair->fld) ? w->lpair + w->W : w->lpair;
  if (fld) {
    if (w->apair) b = (!bottom && w->apair->fld) ? w->apair : w->apair + w->W;
  } else {
    b = bottom ? T : (w->apair ? w->apair + w->W : NULL);
  }
  return (w->is_b ? 24 : 11) + (a && !a->skip) + (b && !b->skip);
}
/* mb_field_decoding_flag (FFmpeg decode_cabac_field_decoding_flag): ctxIdx 70 + left pair
 * field (the inferred flag, which is the left pair's within a row) + upper pair field */
static int field_flag(walker_t *w, int inferred) {
  return bin(w, SE_FIELD, 0, 70 + (w->x > 0 && inferred) + (w->apair && w->apair->fld));
}

/* one macroblock pair of an MBAFF frame, FFmpeg's order: top skip; a skipped top takes the bottom's
 * skip flag next and, if the bottom is coded, the pair's field flag; a coded top reads the field
 * flag after its skip flag; the bottom of a pair whose top was coded reads none */
static void decode_pair_mbaff(walker_t *w, int *mbs_done) {
  const avr_slice_hdr_t *h = w->h;
  const avr_hooks_t *hooks = w->hk;
  wmb_t *T = w->mbs + w->x + 2 * w->pr * w->W;
  /* inference (7.4.4): the left pair's flag, else the upper pair's, else frame */
  int fld = w->lpair ? w->lpair->fld : w->apair ? w->apair->fld : 0;
  int skip_top = 0, skip_bottom = 0;
  for (int bottom = 0; bottom < 2 && !w->err; bottom++) {
    wmb_t *cur = T + bottom * w->W;
    w->cur = cur;
    w->bottom = bottom;
    memset(cur->ref, -1, sizeof(cur->ref));
    hooks->mb_xy(hooks->opaque, w->x, 2 * w->pr + bottom);
    cur->fld = (uint8_t)fld;
    w->fld = fld;
    if (h->slice_type != AVR_SLICE_I) {
      int skip;
      if (bottom && skip_top) skip = skip_bottom;
      else skip = bin(w, SE_SKIP, 0, skip_ctx_mbaff(w, bottom, fld));
      if (skip) {
        if (!bottom) {
          skip_top = 1;
          cur->skip = 1;
          skip_bottom = bin(w, SE_SKIP, 0, skip_ctx_mbaff(w, 1, fld));
          if (!skip_bottom) fld = field_flag(w, fld);
          cur->fld = (uint8_t)fld;
          w->fld = fld;
        }
        mb_skipped(w);
        cur->decoded = 1;
        (*mbs_done)++;
        continue;
      }
    }
    if (!bottom) {
      fld = field_flag(w, fld);
      cur->fld = (uint8_t)fld;
      w->fld = fld;
    }
    decode_mb_layer(w);
    if (w->err) return;
    cur->decoded = 1;
    (*mbs_done)++;
  }
}

static void decode_mb_layer(walker_t *w) {
  const avr_slice_hdr_t *h = w->h;
  wmb_t *cur = w->cur;
  mbtype_t t;
  decode_mb_type(w, &t);
  if (w->err) return;
  if (t.pcm) { w->err = -2; return; }  /* I_PCM: skip_bytes hook, unsupported (recode.cpp:161-163) */
  int cbp = 0;
  int no_sub_lt8x8 = 1;
  if (t.intra) {
    cur->intra = 1;
    cur->i16 = (uint8_t)t.i16;
    if (!t.i16) {
      if (h->transform_8x8_mode) cur->t8x8 = (uint8_t)bin(w, SE_T8X8, 0, 399 + (mb_a(w) && mb_a(w)->t8x8) + (nb_above(w) && nb_above(w)->t8x8));
      int nmodes = cur->t8x8 ? 4 : 16;
      for (int i = 0; i < nmodes; i++) {
        if (!bin(w, SE_PREVINTRA, 0, 68)) {
          bin(w, SE_REMINTRA, 0, 69);
          bin(w, SE_REMINTRA, 1, 69);
          bin(w, SE_REMINTRA, 2, 69);
        }
      }
    }
    if (h->chroma_array_type == 1 || h->chroma_array_type == 2) {
      const wmb_t *a = mb_a(w), *b = nb_above(w);
      int ctx = (a && a->intra && a->chroma_pred) + (b && b->intra && b->chroma_pred);
      int mode = 0;
      if (bin(w, SE_CHROMAPRED, 0, 64 + ctx)) {
        mode = 1;
        if (bin(w, SE_CHROMAPRED, 1, 64 + 3)) mode = 2 + bin(w, SE_CHROMAPRED, 2, 64 + 3);
      }
      cur->chroma_pred = (uint8_t)mode;
    }
  } else if (t.nparts == 4) {
    /* P_8x8, B_8x8 or B_Direct_16x16 */
    submb_t sub[4];
    if (t.direct16) {
      cur->direct16 = 1;
      memset(cur->direct8, 1, 4);
      if (!h->direct_8x8_inference) no_sub_lt8x8 = 0;
    } else {
      for (int i = 0; i < 4; i++) {
        decode_sub_mb_type(w, &sub[i]);
        if (sub[i].direct) {
          cur->direct8[i] = 1;
          if (!h->direct_8x8_inference) no_sub_lt8x8 = 0;
        } else if (sub[i].nparts > 1) {
          no_sub_lt8x8 = 0;
        }
      }
      for (int list = 0; list < (w->is_b ? 2 : 1); list++) {
        for (int i = 0; i < 4; i++) {
          if (sub[i].direct || !(sub[i].pred & (1 << list))) continue;
          int ref = (h->num_ref_idx_active[list] << (w->mbaff && cur->fld)) > 1 ? decode_ref(w, list, 2 * (i & 1), 2 * (i >> 1)) : 0;
          cur->ref[list][i] = (int8_t)ref;
        }
      }
      for (int list = 0; list < (w->is_b ? 2 : 1); list++) {
        for (int i = 0; i < 4; i++) {
          if (sub[i].direct || !(sub[i].pred & (1 << list))) continue;
          int x0 = 2 * (i & 1), y0 = 2 * (i >> 1);
          for (int j = 0; j < sub[i].nparts; j++) {
            int px, py, pw, ph;
            if (sub[i].nparts == 1) { px = x0; py = y0; pw = 2; ph = 2; }
            else if (sub[i].nparts == 4) { px = x0 + (j & 1); py = y0 + (j >> 1); pw = ph = 1; }
            else if (!sub[i].vertical) { px = x0; py = y0 + j; pw = 2; ph = 1; }
            else { px = x0 + j; py = y0; pw = 1; ph = 2; }
            int mx = decode_mvd(w, list, 0, px, py);
            int my = decode_mvd(w, list, 1, px, py);
            fill_mvd(cur, list, px, py, pw, ph, mx, my);
          }
        }
      }
    }
  } else {
    /* 16x16, 16x8, 8x16 */
    for (int list = 0; list < (w->is_b ? 2 : 1); list++) {
      for (int i = 0; i < t.nparts; i++) {
        if (!(t.pred[i] & (1 << list))) continue;
        int px = t.nparts == 2 && t.vertical ? 2 * i : 0, py = t.nparts == 2 && !t.vertical ? 2 * i : 0;
        int ref = (h->num_ref_idx_active[list] << (w->mbaff && cur->fld)) > 1 ? decode_ref(w, list, px, py) : 0;
        if (t.nparts == 1) memset(cur->ref[list], ref, 4);
        else if (!t.vertical) { cur->ref[list][2 * i] = cur->ref[list][2 * i + 1] = (int8_t)ref; }
        else { cur->ref[list][i] = cur->ref[list][i + 2] = (int8_t)ref; }
      }
    }
    for (int list = 0; list < (w->is_b ? 2 : 1); list++) {
      for (int i = 0; i < t.nparts; i++) {
        if (!(t.pred[i] & (1 << list))) continue;
        int px = 0, py = 0, pw = 4, ph = 4;
        if (t.nparts == 2) {
          if (t.vertical) { px = 2 * i; pw = 2; }
          else { py = 2 * i; ph = 2; }
        }
        int mx = decode_mvd(w, list, 0, px, py);
        int my = decode_mvd(w, list, 1, px, py);
        fill_mvd(cur, list, px, py, pw, ph, mx, my);
      }
    }
  }
  if (w->err) return;
  if (t.i16) {
    cbp = t.i16_cbp;
  } else {
    uint16_t ca = nb_cbp_left(w), cb = nb_cbp(w, nb_above(w));
    int c = 0;
    c |= bin(w, SE_CBP, 0, 73 + !(ca & 0x02) + 2 * !(cb & 0x04));
    c |= bin(w, SE_CBP, 1, 73 + !(c & 0x01) + 2 * !(cb & 0x08)) << 1;
    c |= bin(w, SE_CBP, 2, 73 + !(ca & 0x08) + 2 * !(c & 0x01)) << 2;
    c |= bin(w, SE_CBP, 3, 73 + !(c & 0x04) + 2 * !(c & 0x02)) << 3;
    if (h->chroma_array_type == 1 || h->chroma_array_type == 2) {
      int a = (ca >> 4) & 3, b = (cb >> 4) & 3;
      int ctx = (a > 0) + 2 * (b > 0);
      if (bin(w, SE_CBP, 4, 77 + ctx)) {
        ctx = 4 + (a == 2) + 2 * (b == 2);
        c |= (1 + bin(w, SE_CBP, 5, 77 + ctx)) << 4;
      }
    }
    cbp = c;
    if ((cbp & 15) && h->transform_8x8_mode && !t.intra && no_sub_lt8x8 &&
        (!cur->direct16 || h->direct_8x8_inference))
      cur->t8x8 = (uint8_t)bin(w, SE_T8X8, 0, 399 + (mb_a(w) && mb_a(w)->t8x8) + (nb_above(w) && nb_above(w)->t8x8));
  }
  cur->cbp = (uint16_t)cbp;
  if ((cbp & 0x3f) || t.i16) {
    int ctx = w->last_dqp_nz ? 1 : 0, val = 0;
    while (bin(w, SE_QPDELTA, val, 60 + ctx)) {
      ctx = ctx < 2 ? 2 : 3;
      if (++val > 102) { w->err = -6; return; }
    }
    w->last_dqp_nz = val != 0;
    residual(w, &t, cbp);
  } else {
    w->last_dqp_nz = 0;
  }
}

/* The upper row's bottom edges as the device walkers keep them (avr_walker.h EdgeCore, one per column;
 * zero where that macroblock is not in the slice): the fields the CABAC context selection of the
 * row below reads (9.3.3.1.1), AVR_EDGE_BYTES each. */
static void edge_row(const walker_t *w, int y, uint8_t *out) {
  const int ph_c = (w->h->chroma_array_type == 2 || w->h->chroma_array_type == 3) ? 4 : 2;
  memset(out, 0, (size_t)AVR_EDGE_BYTES * w->W);
  for (int c = 0; c < w->W; c++) {
    const wmb_t *m = &w->mbs[(size_t)(y - 1) * w->W + c];
    uint8_t *e = out + (size_t)AVR_EDGE_BYTES * c;
    if (!m->decoded) continue;
    e[0] = (uint8_t)(1 | m->skip << 1 | m->intra << 2 | m->i16 << 3 | m->direct16 << 4 | m->t8x8 << 5 |
                     (m->chroma_pred != 0) << 6);
    e[2] = (uint8_t)m->cbp;
    e[3] = (uint8_t)(m->cbp >> 8);
    memcpy(e + 4, &m->nnz[0][12], 4);
    memcpy(e + 8, &m->nnz[1][4 * (ph_c - 1)], 4);
    memcpy(e + 12, &m->nnz[2][4 * (ph_c - 1)], 4);
    for (int l = 0; l < 2; l++)
      for (int i = 0; i < 4; i++) {
        e[16 + 8 * l + 2 * i] = m->mvd[l][12 + i][0];
        e[17 + 8 * l + 2 * i] = m->mvd[l][12 + i][1];
      }
    e[32] = (uint8_t)m->ref[0][2];
    e[33] = (uint8_t)m->ref[0][3];
    e[34] = (uint8_t)m->ref[1][2];
    e[35] = (uint8_t)m->ref[1][3];
    e[36] = m->direct8[2];
    e[37] = m->direct8[3];
  }
}

/* A piece of a split slice (avr_oracle.h): the upper row rebuilt from its edges (the fields the
 * parse reads of an upper neighbour), then the walk from `start` */
static void edge_unrow(walker_t *w, int y, const uint8_t *in) {
  const int ph_c = (w->h->chroma_array_type == 2 || w->h->chroma_array_type == 3) ? 4 : 2;
  for (int c = 0; c < w->W; c++) {
    wmb_t *m = &w->mbs[(size_t)(y - 1) * w->W + c];
    const uint8_t *e = in + (size_t)AVR_EDGE_BYTES * c;
    memset(m, 0, sizeof(*m));
    if (!(e[0] & 1)) continue;
    m->decoded = 1;
    m->skip = (e[0] >> 1) & 1;
    m->intra = (e[0] >> 2) & 1;
    m->i16 = (e[0] >> 3) & 1;
    m->direct16 = (e[0] >> 4) & 1;
    m->t8x8 = (e[0] >> 5) & 1;
    m->chroma_pred = (e[0] >> 6) & 1;
    m->cbp = (uint16_t)(e[2] | e[3] << 8);
    memcpy(&m->nnz[0][12], e + 4, 4);
    memcpy(&m->nnz[1][4 * (ph_c - 1)], e + 8, 4);
    memcpy(&m->nnz[2][4 * (ph_c - 1)], e + 12, 4);
    for (int l = 0; l < 2; l++)
      for (int i = 0; i < 4; i++) {
        m->mvd[l][12 + i][0] = e[16 + 8 * l + 2 * i];
        m->mvd[l][12 + i][1] = e[17 + 8 * l + 2 * i];
      }
    memset(m->ref, -1, sizeof(m->ref));
    m->ref[0][2] = (int8_t)e[32];
    m->ref[0][3] = (int8_t)e[33];
    m->ref[1][2] = (int8_t)e[34];
    m->ref[1][3] = (int8_t)e[35];
    m->direct8[2] = e[36];
    m->direct8[3] = e[37];
  }
}

static int walk(const avr_slice_hdr_t *h, const avr_hooks_t *hooks, int picture_id, const avr_piece_start_t *ps) {
  if (!h->supported) return -1;
  walker_t w;
  memset(&w, 0, sizeof(w));
  w.h = h;
  w.hk = hooks;
  w.W = h->mb_width;
  /* a field picture is its own picture of half the frame's rows (FFmpeg PAFF); the model hooks
   * still see the frame (h->mb_height) and FFmpeg's frame row of each macroblock,
   * sl->mb_y = 2 * field row + bottom_field_flag (h264_slice.c, decode_slice) */
  w.H = h->field_pic ? h->mb_height / 2 : h->mb_height;
  w.fld = h->field_pic;   /* MBAFF: per pair */
  w.is_b = h->slice_type == AVR_SLICE_B;
  w.mbs = (wmb_t *)calloc((size_t)w.W * w.H, sizeof(wmb_t));
  if (!w.mbs) return -1;
  avr_cabac_init_states(w.state, h->slice_type == AVR_SLICE_I ? -1 : h->cabac_init_idc, h->slice_qp);
  hooks->frame_spec(hooks->opaque, picture_id, w.W, h->mb_height);
  int addr = h->first_mb;
  int stop_after = 0;
  if (ps) {
    if (h->field_pic || h->mbaff) { free(w.mbs); return -1; }
    addr = ps->start_mb;
    stop_after = ps->n_mbs;
    if (ps->edge) {
      if (addr % w.W || addr < w.W) { free(w.mbs); return -1; }
      memcpy(w.state, ps->state, 1024);
      w.last_dqp_nz = ps->last_dqp_nz;
      edge_unrow(&w, addr / w.W, ps->edge);
    }
  }
  int ret = 0;
  avr_walk_mbs_done = 0;
  w.mbaff = h->mbaff;
  /* MBAFF: first_mb is the top macroblock of the first pair (2 * first_mb_in_slice); macroblock
   * pairs in raster order, the model hooks see FFmpeg's frame row 2 * pair row + bottom */
  for (int pair = addr / 2; w.mbaff;) {
    w.x = pair % w.W;
    w.pr = pair / w.W;
    if (2 * w.pr + 1 >= w.H) { ret = -7; break; }
    wmb_t *T = w.mbs + w.x + 2 * w.pr * w.W;
    w.lpair = w.x > 0 && T[-1].decoded ? T - 1 : NULL;
    w.apair = w.pr > 0 && T[-2 * w.W].decoded ? T - 2 * w.W : NULL;
    decode_pair_mbaff(&w, &avr_walk_mbs_done);
    if (w.err) { ret = w.err; break; }
    avr_walk_last_mb = 2 * (pair + 1) >= w.W * w.H;
    if (term(&w, SE_EOS)) break;
    pair++;
  }
  for (; !w.mbaff;) {
    if (addr >= w.W * w.H) { ret = -7; break; }
    int x = addr % w.W, y = addr / w.W;
    w.cur = &w.mbs[addr];
    w.left = x > 0 && w.mbs[addr - 1].decoded ? &w.mbs[addr - 1] : NULL;
    w.top = y > 0 && w.mbs[addr - w.W].decoded ? &w.mbs[addr - w.W] : NULL;
    if (hooks->row_start && !h->field_pic && x == 0 && addr != h->first_mb) {
      uint8_t *row = (uint8_t *)malloc((size_t)AVR_EDGE_BYTES * w.W);
      edge_row(&w, y, row);
      hooks->row_start(hooks->opaque, addr, w.state, row, w.last_dqp_nz);
      free(row);
    }
    hooks->mb_xy(hooks->opaque, x, h->field_pic ? 2 * y + h->bottom_field : y);
    decode_mb(&w);
    if (getenv("AVR_WALK_DEBUG"))
      fprintf(stderr, "mb %d skip %d intra %d i16 %d t8 %d cbp %03x d16 %d nnz0 %d %d %d %d\n", addr, w.cur->skip, w.cur->intra,
              w.cur->i16, w.cur->t8x8, w.cur->cbp, w.cur->direct16, w.cur->nnz[0][0], w.cur->nnz[0][1], w.cur->nnz[1][0], w.cur->nnz[2][0]);
    if (w.err) { ret = w.err; break; }
    w.cur->decoded = 1;
    avr_walk_mbs_done++;
    avr_walk_last_mb = addr + 1 >= w.W * w.H;
    if (term(&w, SE_EOS)) break;
    if (stop_after && avr_walk_mbs_done == stop_after) { ret = 1; break; }   /* the piece's end */
    addr++;
  }
  free(w.mbs);
  return ret;
}

int avr_walk_slice(const avr_slice_hdr_t *h, const avr_hooks_t *hooks, int picture_id) {
  return walk(h, hooks, picture_id, NULL);
}
int avr_walk_piece(const avr_slice_hdr_t *h, const avr_hooks_t *hooks, int picture_id, const avr_piece_start_t *ps) {
  return walk(h, hooks, picture_id, ps);
}
