/*
 * avrecode oracle — CPU restatement of the reference's recode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (avrecode_amd/, include/) links,
 * imports or executes this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and there only as the checker / CPU baseline.
 *
 * What it restates (reference = /root/reference, read-only, ddkang/avrecode):
 *   - arithmetic_code.h:31-320        generic binary arithmetic coder (encoder, decoder, finish)
 *   - cabac_code.h:16-86              CABAC re-encoder on top of the generic coder
 *   - recode.cpp:233-471, 615-1100    h264_model predictor, scan geometry, h264_symbol::execute
 *   - recode.cpp:1102-1624            compressor / decompressor drivers, surrogates, roundtrip
 *   - recode.proto                    Recoded container (hand-written proto2 wire codec)
 * and, because the libavcodec-hooks FFmpeg fork (submodule ffmpeg/, pinned commit unknowable,
 * FFmpeg 2.8-3.0 API era) is absent from the reference, the parts of it the hot path calls:
 *   - ITU-T H.264 9.3 CABAC decoding engine (ff_get_cabac / _bypass / _terminate)
 *   - ITU-T H.264 7.3.4/7.3.5 CABAC slice_data()/macroblock_layer() parse that drives the hooks
 *   - H.264 NAL / SPS / PPS / slice header parsing, MP4 (avcC) and Annex-B demux.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - the generic coder is pinned bit-exactly against arithmetic_code.h compiled as-is
 *     (oracle/ref_arith_driver.cpp -> oracle/_ref/ref_arith, goldens in tests/golden/);
 *   - the CABAC engine + parser are pinned by real x264 streams (tests/fixtures): every slice must
 *     parse to end_of_slice at the last MB with the CABAC decoder ending exactly on the
 *     rbsp_stop_one_bit, and re-encoding the parsed bins must regenerate the original bytes;
 *   - the predictor (h264_model) is unpinned against a reference build (recode.cpp needs the
 *     fork's headers, protoc and libprotobuf: unbuildable here) and is a line-by-line restatement.
 */
#ifndef AVR_ORACLE_H
#define AVR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------ */
/* growable byte buffer                                                                        */
typedef struct {
  uint8_t *data;
  size_t len, cap;
} obuf_t;
void ob_init(obuf_t *b);
void ob_free(obuf_t *b);
void ob_put(obuf_t *b, uint8_t v);
void ob_append(obuf_t *b, const uint8_t *p, size_t n);

/* ------------------------------------------------------------------------------------------ */
/* Generic arithmetic coder, arithmetic_code.h:31-299.                                          */
/* One struct serves both instantiations used by the reference:                                */
/*   recoded:  <uint64_t, uint8_t, 0>        (recode.cpp:315-316)                               */
/*   cabac:    <uint32_t, uint16_t, 0x200> with uint8_t output digits (cabac_code.h:24,83)      */
typedef struct {
  uint64_t fixed_one;     /* 2^(bits-1) */
  int digit_bits;         /* CompressedDigit width in bits (8 or 16) */
  int out_bits;           /* OutputDigit width in bits (8) */
  uint64_t min_range;
  uint64_t low, range;
  uint16_t *overflow;     /* deferred CompressedDigits (arith:200) */
  size_t novf, capovf;
  size_t bytes_emitted;
  obuf_t *out;
} ac_enc_t;

void ac_enc_init(ac_enc_t *e, obuf_t *out, int fixed_bits, int digit_bits, uint64_t min_range,
                 uint64_t initial_range);
/* put(symbol, range_of_1) — range_of_1 must be computed by the caller from e->range. */
size_t ac_enc_put(ac_enc_t *e, int symbol, uint64_t range_of_1);
void ac_enc_finish(ac_enc_t *e);
void ac_enc_free(ac_enc_t *e);

typedef struct {
  uint64_t fixed_one, min_range, digit_base, digit_alignment;
  int digit_bytes;
  uint64_t low, range, next_digit;
  const uint8_t *in, *end;
} ac_dec_t;
void ac_dec_init(ac_dec_t *d, const uint8_t *in, const uint8_t *end, int fixed_bits, int digit_bits,
                 uint64_t min_range);
int ac_dec_get(ac_dec_t *d, uint64_t range_of_1);

/* recoded coder helpers: recode.cpp:816-820 probability (range/total)*pos */
static inline uint64_t rc_p1(uint64_t range, int pos, int neg) {
  return (range / (uint64_t)(pos + neg)) * (uint64_t)pos;
}
void rc_enc_init(ac_enc_t *e, obuf_t *out);
void rc_dec_init(ac_dec_t *d, const uint8_t *in, size_t n);

/* P-format coder: NOT part of the reference.  The parallel model's optional container (tag
 * "avrecode-amd:P32") is this library's own format and codes the model's decisions with a 32-bit
 * range coder with byte digits (avrecode_amd/csrc/avr_engine.h, PEncoder / PDecoder), restated
 * here: range in [2^24, 2^32) between decisions (0xFFFFFFFF at the start), bin 1 takes the top
 * r1 = floor(range * floor(2^32 / tot) / 2^32) * pos of the range (tot = pos + neg), one 8-bit
 * renormalisation step when range < 2^24. */
typedef struct {
  uint64_t low;           /* window bits 0-31, carry bit 32 */
  uint32_t range, pending, cache;
  int have_cache, err;
  uint32_t bill_pend;     /* digits the billing rule still defers */
  obuf_t *out;
} pc_enc_t;
typedef struct {
  uint32_t low, range;
  const uint8_t *in, *end;
} pc_dec_t;
static inline uint32_t pc_p1(uint32_t range, int pos, int neg) {
  const uint32_t rcp = (uint32_t)((1ull << 32) / (uint64_t)(pos + neg));
  return (uint32_t)(((uint64_t)range * rcp) >> 32) * (uint32_t)pos;
}
void pc_enc_init(pc_enc_t *e, obuf_t *out);
/* returns the bytes billed to this put: at a renormalisation, the digit and every digit deferred
 * before it once its value is final (as arithmetic_code::encoder::put reports, arith:146-175) */
size_t pc_enc_put(pc_enc_t *e, int symbol, uint32_t r1);
void pc_enc_finish(pc_enc_t *e);
void pc_dec_init(pc_dec_t *d, const uint8_t *in, size_t n);
int pc_dec_get(pc_dec_t *d, uint32_t r1);

/* ------------------------------------------------------------------------------------------ */
/* CABAC tables (ITU-T H.264 Tables 9-12..9-33, 9-44, 9-45) in FFmpeg layout                   */
extern uint8_t avr_lps_range[4 * 128];    /* [q*128 + state], state=(pStateIdx<<1)|valMPS  */
extern uint8_t avr_mlps_state[256];         /* [128+s] after MPS, [127-s] after LPS          */
/* init state bytes for 1024 contexts; init_idc = -1 for I/SI slices, 0..2 otherwise           */
void avr_cabac_init_states(uint8_t state[1024], int init_idc, int slice_qp);

/* CABAC re-encoder, cabac_code.h:27-80 */
typedef struct {
  ac_enc_t e;
} cabac_enc_t;
void cabac_enc_init(cabac_enc_t *c, obuf_t *out);
size_t cabac_enc_put(cabac_enc_t *c, int symbol, uint8_t *state);
size_t cabac_enc_put_bypass(cabac_enc_t *c, int symbol);
size_t cabac_enc_put_terminate(cabac_enc_t *c, int symbol);
void cabac_enc_free(cabac_enc_t *c);

/* CABAC decoding engine, ITU-T H.264 9.3.1.2 / 9.3.3.2 (ff_get_cabac & co, fork) */
typedef struct {
  const uint8_t *buf;
  size_t nbits;     /* payload size in bits */
  size_t pos;       /* next bit to read */
  uint32_t range, offset;
  int overrun;      /* bits read past the end */
} cabac_dec_t;
void cabac_dec_init(cabac_dec_t *d, const uint8_t *buf, size_t n);
int cabac_dec_decision(cabac_dec_t *d, uint8_t *state);
int cabac_dec_bypass(cabac_dec_t *d);
int cabac_dec_terminate(cabac_dec_t *d);

/* ------------------------------------------------------------------------------------------ */
/* H.264 front end                                                                             */
typedef struct {
  int valid;
  int profile_idc, chroma_format_idc, separate_colour_plane, bit_depth_luma, bit_depth_chroma;
  int log2_max_frame_num, poc_type, log2_max_poc_lsb, delta_pic_order_always_zero;
  int frame_mbs_only, mb_aff, direct_8x8_inference;
  int mb_width, mb_height; /* in MBs (frame) */
} avr_sps_t;

typedef struct {
  int valid;
  int sps_id, entropy_coding_mode, bottom_field_pic_order_present, num_slice_groups;
  int num_ref_idx_default[2], weighted_pred, weighted_bipred_idc, pic_init_qp;
  int deblocking_filter_control_present, constrained_intra_pred, redundant_pic_cnt_present;
  int transform_8x8_mode;
} avr_pps_t;

enum { AVR_SLICE_P = 0, AVR_SLICE_B = 1, AVR_SLICE_I = 2, AVR_SLICE_SP = 3, AVR_SLICE_SI = 4 };

typedef struct {
  int nal_unit_type, nal_ref_idc;
  int first_mb, slice_type, pps_id, frame_num, field_pic, bottom_field, idr_pic_id, poc_lsb;
  int direct_spatial, num_ref_idx_active[2], cabac_init_idc, slice_qp;
  int mbaff;
  /* derived */
  int chroma_array_type, transform_8x8_mode, direct_8x8_inference, mb_width, mb_height;
  int constrained_intra_pred;
  int x264_build;      /* from the x264 SEI user data, -1 if absent (FFmpeg h->x264_build) */
  size_t cabac_start;  /* byte offset of slice_data() in the unescaped RBSP */
  int supported;       /* 0 = the walker cannot parse this slice (MBAFF, field, FMO, ...) */
} avr_slice_hdr_t;

/* unescape an H.264 NAL payload (emulation prevention), FFmpeg 2.8 ff_h264_decode_nal rules */
size_t avr_nal_unescape(const uint8_t *src, size_t n, uint8_t *dst);
/* FFmpeg RBSP bit length rule: trailing zero bytes stripped, stop bit excluded */
size_t avr_rbsp_bit_length(const uint8_t *rbsp, size_t n);

typedef struct {
  avr_sps_t sps[32];
  avr_pps_t pps[256];
} avr_param_sets_t;
int avr_parse_sps(avr_param_sets_t *ps, const uint8_t *rbsp, size_t n);
int avr_parse_pps(avr_param_sets_t *ps, const uint8_t *rbsp, size_t n);
/* FFmpeg decode_unregistered_user_data: "x264 - core %d" in an SEI user_data_unregistered */
int avr_parse_sei_x264_build(const uint8_t *rbsp, size_t n);
int avr_parse_slice_header(const avr_param_sets_t *ps, const uint8_t *rbsp, size_t n,
                           int nal_unit_type, int nal_ref_idc, avr_slice_hdr_t *h);

/* a NAL unit located in the file */
typedef struct {
  size_t offset;   /* file offset of the NAL header byte */
  size_t size;     /* escaped size incl. header byte */
} avr_nal_t;
/* Enumerate the video NAL units of an MP4 (avcC) or Annex-B file in decode order.
 * Returns count, *out malloc'd.  avcC parameter sets are returned first with offset into file. */
int avr_demux(const uint8_t *file, size_t n, avr_nal_t **out);

/* ------------------------------------------------------------------------------------------ */
/* The hook surface the parser drives — AVCodecHooks (recode.cpp:137-228, signatures of the   */
/* libavcodec-hooks fork).  CodingType identity follows EACH_PIP_CODING_TYPE usage.            */
typedef enum {
  PIP_UNKNOWN = 0,
  PIP_UNREACHABLE,
  PIP_SIGNIFICANCE_MAP,
  PIP_SIGNIFICANCE_EOB,
  PIP_SIGNIFICANCE_NZ,
  PIP_RESIDUALS,
} avr_coding_type;

typedef struct {
  void *opaque;
  /* cabac hooks: return the bin; ctx_idx names FFmpeg's cabac_state[] slot */
  int (*get)(void *opaque, uint8_t *state, int ctx_idx);
  int (*get_bypass)(void *opaque);
  int (*get_terminate)(void *opaque);
  /* model hooks */
  void (*frame_spec)(void *opaque, int frame_num, int mb_width, int mb_height);
  void (*mb_xy)(void *opaque, int x, int y);
  void (*begin_sub_mb)(void *opaque, int cat, int scan8index, int max_coeff, int is_dc, int chroma422);
  void (*end_sub_mb)(void *opaque, int cat, int scan8index, int max_coeff, int is_dc, int chroma422);
  void (*begin_coding_type)(void *opaque, avr_coding_type ct, int zigzag_index, int param0, int param1);
  void (*end_coding_type)(void *opaque, avr_coding_type ct);
  /* NOT a reference hook (optional, NULL: not called): the start of a macroblock row of a progressive
   * frame slice other than its first macroblock, before that row's mb_xy -- where the parallel
   * model's long-slice split may begin a piece (avr_seam_t below).  state: the 1024 CABAC context
   * bytes; edge_row: AVR_EDGE_BYTES per column, the upper row's bottom edges (avr_edge_row);
   * last_dqp_nz: the previous macroblock's mb_qp_delta != 0. */
  void (*row_start)(void *opaque, int mb_addr, const uint8_t *state, const uint8_t *edge_row, int last_dqp_nz);
} avr_hooks_t;

/* Parse slice_data() of one slice, pulling every bin through hooks.  The parser owns the     */
/* 1024 CABAC context bytes (FFmpeg's sl->cabac_state).  Returns 0 on success (end_of_slice   */
/* reached at a legal MB), <0 on a syntax error / unsupported syntax / overrun.               */
int avr_walk_slice(const avr_slice_hdr_t *h, const avr_hooks_t *hooks, int picture_id);
/* One piece of a split slice (avr_seam_t): the walk from start_mb (a row start) for n_mbs
 * macroblocks (0: to end_of_slice), the CABAC contexts, the upper row and last_dqp_nz from the
 * seam (edge == NULL: the slice's own start).  Returns 1 when it stopped after n_mbs. */
typedef struct {
  int start_mb, n_mbs, last_dqp_nz;
  const uint8_t *state, *edge;
} avr_piece_start_t;
int avr_walk_piece(const avr_slice_hdr_t *h, const avr_hooks_t *hooks, int picture_id, const avr_piece_start_t *ps);

/* ------------------------------------------------------------------------------------------ */
/* The predictor (recode.cpp:615-1059) and the two drivers                                   */
/* R: the reference model.  P: the parallel model (fresh model per slice) on the reference's
 * arithmetic_code<uint64_t, uint8_t> (tag "avrecode-amd:P64").  P32: the parallel model on the P-format
 * coder below (tag "avrecode-amd:P32"). */
enum { AVR_MODE_R = 0, AVR_MODE_P = 1, AVR_MODE_P32 = 2, AVR_MODE_C = 3 };
/* C: the reference model in chains -- a fresh model (estimators and frames, as a new file) before
 * every AVR_CHAIN_SLICES-th coded slice (tag "avrecode-amd:R16"): each chain is sequential, the chains
 * are independent, so a file decodes with (coded slices / 16) walkers at once while the model still
 * learns across a chain's slices. */
#define AVR_CHAIN_SLICES 16

typedef struct avr_model avr_model_t;
avr_model_t *avr_model_new(void);
void avr_model_free(avr_model_t *m);

/* Whole-file drivers.  out is malloc'd.  Return 0 on success. */
int avr_compress(const uint8_t *file, size_t n, int mode, uint8_t **out, size_t *out_len);
int avr_decompress(const uint8_t *in, size_t n, uint8_t **out, size_t *out_len);

/* Per-slice statistics for tests and the CPU baseline */
typedef struct {
  size_t file_bytes, slices, coded_slices, skipped_slices, payload_bytes, recoded_bytes, bins;
} avr_stats_t;
extern avr_stats_t avr_last_stats;
/* h264_model::bill / cabac_bill (recode.cpp:615-661) of the last avr_compress / avr_decompress,
 * summed over its model(s), indexed by avr_coding_type: bytes the re-coded encoder emitted per
 * put (compress, recode.cpp:1074-1078, 1213-1220) and bytes the CABAC encoder emitted per put
 * (decompress, 1443-1446, 1455-1457, 1466-1468). */
extern size_t avr_last_bill[8], avr_last_cabac_bill[8];
void avr_model_bills(const avr_model_t *m, size_t bill[8], size_t cabac_bill[8]);

/* ------------------------------------------------------------------------------------------ */
/* Slice-level API used by the tests to cross-check the GPU kernels slice by slice.          */
/* Compress one CABAC slice payload with a FRESH model (P-mode semantics).                   */
int avr_compress_slice_p(const avr_slice_hdr_t *h, const uint8_t *payload, size_t n, obuf_t *recoded,
                         size_t *bins);
/* Decompress one slice (P-mode): regenerate the CABAC bytes (before the last-byte patch).   */
int avr_decompress_slice_p(const avr_slice_hdr_t *h, const uint8_t *recoded, size_t n, obuf_t *cabac);
/* Regenerate CABAC bytes by decode+re-encode (no model): the parser/engine self-check.      */
int avr_cabac_regenerate(const avr_slice_hdr_t *h, const uint8_t *payload, size_t n, obuf_t *cabac,
                         size_t *bins, size_t *end_bitpos);

/* Per-slice fresh-model compress -> decompress records for CABAC slices [lo, hi) of a file      */
/* (layout in oracle_recode.c), on the u64 coder (p32 = 0) or the P32 coder (p32 = 1).          */
/* Returns the file's CABAC slice count, or -1.                                                  */
long avr_oracle_slices_p(const uint8_t *file, size_t n, long lo, long hi, int check_recodable, int p32, uint8_t **out,
                         size_t *out_len);

/* ------------------------------------------------------------------------------------------ */
/* Long-slice split of the parallel model (NOT part of the reference: this library's own format,  */
/* restated here as the checker; avrecode_amd/csrc/avr_api.cpp "seams").  A progressive-frame     */
/* slice is cut at macroblock-row starts into pieces, each re-coded with a fresh parallel model  */
/* (its estimators reset, its upper row's model bytes zero, as at a slice start), so that the     */
/* pieces decompress side by side.  A cut (a "seam") comes at the first row start with at least   */
/* 8 * split_bytes CABAC bits decoded since the previous seam (or the slice start) and at least   */
/* 4 * split_bytes bits of the payload still ahead.  Block field 16 ("seams", zlib) carries what   */
/* a piece's decompressor needs from before it (avr_seams_encode); Block.cabac holds the pieces'   */
/* re-coded streams one after the other.                                                         */
#define AVR_EDGE_BYTES 40          /* one column of the upper row: flags | cbp << 16, nnz[3][4] (bottom
                                    * rows), mvd[2][4][2], ref[2][2], direct8[2], 2 zero bytes */
#define AVR_SPLIT_BYTES_DEFAULT 98304
typedef struct {
  uint32_t first_mb;               /* the piece's first macroblock (a row start) */
  uint32_t q;                      /* where its regenerated bytes begin in the slice's CABAC bytes */
  uint32_t last_dqp_nz;
  /* the CABAC re-encoder at the cut (avr_engine.h CabacEncoder: cache byte, outstanding 0xFF bytes,
   * low = pending bits + 10-bit window, queue = pending bits - 8, range) */
  uint32_t ce_low, ce_outstanding, ce_cache, ce_range;
  int32_t ce_queue;
  uint8_t state[1024];             /* CABAC context bytes */
  uint8_t *edge;                   /* AVR_EDGE_BYTES * mb_width (malloc'd) */
} avr_seam_t;
/* split_bytes of the whole-file compress (0: no split): AVR_SPLIT_BYTES from the environment, else
 * AVR_SPLIT_BYTES_DEFAULT; avr_oracle_set_split_bytes overrides both */
size_t avr_oracle_split_bytes(void);
void avr_oracle_set_split_bytes(size_t bytes);
/* The re-encoder's state where the CABAC decoder stands after `bitpos` bits (9 + renormalisation
 * shifts) with codIOffset `offset` and codIRange `range` on this payload: 0, or -1 when the cut
 * cannot be placed there (the arithmetic's pending digits reach too far back). */
int avr_seam_encoder(const uint8_t *payload, size_t n, size_t bitpos, uint32_t offset, uint32_t range,
                     avr_seam_t *s);
/* the seams blob: u32 raw length, then zlib (level 9) of { u32 2, u32 seams, u32 mb_width,
 * u32 piece_len[seams + 1], per seam { u32 first_mb, q, last_dqp_nz, ce_low, ce_queue, ce_outstanding,
 * ce_cache, ce_range, u8 state[1024] XOR the slice's initial context states (9.3.1.1), u8 edges
 * byte-major (byte j of every column, j = 0..39), nnz as nonzero and |mvd| up to 33 } }, little-endian */
int avr_seams_encode(const avr_seam_t *s, int n_seams, int mb_width, const uint32_t *piece_len,
                     const uint8_t init_state[1024], obuf_t *out);
/* parses a seams blob: 0 and *s (malloc'd, n_seams entries), *piece_len (malloc'd, n_seams + 1); -1 */
int avr_seams_decode(const uint8_t *p, size_t n, int mb_width, const uint8_t init_state[1024], avr_seam_t **s,
                     int *n_seams, uint32_t **piece_len);
void avr_seams_free(avr_seam_t *s, int n_seams);
/* the device's CABAC re-encoder in byte form (avr_engine.h CabacEncoder), which a piece starts from a
 * seam's state (s == NULL: a slice start) and ends with avr_ce_seam_flush */
typedef struct {
  uint32_t low, range, outstanding, cache;
  int queue, have_cache, err;
  obuf_t *out;
} avr_ce_t;
void avr_ce_init(avr_ce_t *e, obuf_t *out, const avr_seam_t *s);
void avr_ce_decision(avr_ce_t *e, int bin, uint8_t *state);
void avr_ce_bypass(avr_ce_t *e, int bin);
void avr_ce_terminate(avr_ce_t *e, int bin);
void avr_ce_seam_flush(avr_ce_t *e);
/* One piece of a split P-mode slice decompressed on its own, as the device does it: a fresh model on
 * the piece's stream rc[0..n), the walk from the seam (NULL: the slice start) for n_mbs macroblocks (0:
 * to the slice's end), the byte-form re-encoder from the seam's state.  *out: the regenerated bytes
 * from the seam's q (a last piece without its trailing 0x80, recode.cpp:1503-1505). */
int avr_decompress_piece(const avr_slice_hdr_t *h, int picture_id, const uint8_t *rc, size_t n, const avr_seam_t *seam,
                         int n_mbs, obuf_t *out);
/* every split slice of a file (split_bytes) decompressed piece by piece and compared (oracle_recode.c) */
int avr_check_pieces(const uint8_t *file, size_t n, size_t split_bytes, int *n_split, int *n_pieces);

/* protobuf wire codec for recode.proto */
typedef struct {
  int64_t size;
  int has_size, has_literal, has_skip, has_cabac, has_parity, has_last_byte, has_seams;
  int skip_coded, length_parity;
  const uint8_t *literal;
  size_t literal_len;
  const uint8_t *cabac;
  size_t cabac_len;
  uint8_t last_byte;
  int last_byte_len;
  const uint8_t *seams;   /* field 16 (this library's parallel-model long-slice split), zlib */
  size_t seams_len;
} avr_pb_block_t;
void avr_pb_put_block(obuf_t *o, const avr_pb_block_t *b);
/* model mode recorded in Recoded.metadata.version (R-mode: absent, as the reference writes):
 * AVR_MODE_R / _P / _P32 / _C, or -1 for another "avrecode-amd:" format */
int avr_pb_mode(const uint8_t *in, size_t n);
/* parses a Recoded message; returns block count, *blocks malloc'd (pointers into in) */
int avr_pb_parse(const uint8_t *in, size_t n, avr_pb_block_t **blocks);

#ifdef __cplusplus
}
#endif
#endif
