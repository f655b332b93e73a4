/*
 * Oracle-internal: the h264_model predictor (recode.cpp:615-1059).  TEST INFRASTRUCTURE ONLY.
 */
#ifndef AVR_ORACLE_MODEL_H
#define AVR_ORACLE_MODEL_H

#include "avr_oracle.h"

/* model_key = tuple<const void*, int, int> (recode.cpp:318).  The pointer identity is replaced by
 * a kind id: FFmpeg cabac_state[] slot 0..1023, or one of the model's own objects. */
enum {
  K_BYPASS = 1024,      /* &bypass_context       (recode.cpp:1049) */
  K_TERMINATE = 1025,   /* &terminate_context    */
  K_SIGNIF = 1026,      /* &significance_context */
  K_FAKE_EOB = 1027,    /* static fake_context   (recode.cpp:805) */
  K_NZBIT = 1028,       /* &STATE_FOR_NUM_NONZERO_BIT[i], i = 0..5 (recode.cpp:625) */
};
typedef uint64_t model_key_t;
static inline model_key_t mk_key(int kind, int a, int b) {
  return (uint64_t)kind << 48 | (uint64_t)(uint32_t)a << 24 | (uint64_t)(uint32_t)b;
}

typedef struct { uint8_t num_nonzeros[51]; uint8_t coded, is_8x8; } blockmeta_t; /* block.h:9-23 */
typedef struct { uint16_t residual[816]; } mbblock_t;                            /* block.h:4-8 */
typedef struct {
  uint32_t width, height;
  int frame_num;
  blockmeta_t *meta;
  mbblock_t *image;
} framebuf_t; /* framebuffer.h */

typedef struct { int pos, neg; } estimator_t;

struct avr_model {
  int coding_type;
  framebuf_t frames[2];
  int cur_frame;
  int mb_x, mb_y, scan8_index, zigzag_index; /* mb_coord */
  int nonzeros_observed, sub_mb_cat, sub_mb_size, sub_mb_is_dc, sub_mb_chroma422;
  /* std::map<model_key, estimator> (recode.cpp:1058) as an open-addressing hash */
  model_key_t *keys;
  estimator_t *vals;
  uint8_t *used;
  size_t cap, count;
  int decompress_side; /* set by the decompressor driver: see finished_queueing */
  int p32;             /* the parallel model's container: P-format coder (pc_p1), not rc_p1 */
  size_t bill[8], cabac_bill[8];
};

model_key_t model_get_key(avr_model_t *m, int ctx_kind);
uint64_t model_p1(avr_model_t *m, uint64_t range, model_key_t key);
void model_update_key(avr_model_t *m, int symbol, model_key_t key);
void model_update_state(avr_model_t *m, int symbol, int ctx_kind);
void model_update_tracking(avr_model_t *m, int symbol);
void model_update_frame_spec(avr_model_t *m, int frame_num, int mb_width, int mb_height);
int model_begin_coding_type(avr_model_t *m, int ct);
void model_end_coding_type(avr_model_t *m, int ct);
void model_reset_sig_tracking(avr_model_t *m);
typedef void (*nz_cb_t)(void *ctx, avr_model_t *m, model_key_t key, int *symbol);
void model_finished_queueing(avr_model_t *m, int ct, nz_cb_t cb, void *ctx);
blockmeta_t *model_meta(avr_model_t *m, int which, int x, int y);

#endif
