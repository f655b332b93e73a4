/*
 * avrecode-amd: MI355X-native implementation of avrecode's CABAC decode -> predict ->
 * arithmetic re-encode path (ddkang/avrecode, reference mounted at /root/reference).
 *
 * C ABI: extern "C", plain pointers and sizes, integer status codes, no exceptions across the
 * boundary, caller-owned buffers unless stated, one avr_ctx per host thread (not thread-safe).
 *
 * Reference interfaces each group replaces (file:line in /root/reference):
 *   avr_compress_file    compressor(...).run()           recode.cpp:1102-1125, 1275-1297
 *   avr_decompress_file  decompressor(...).run()         recode.cpp:1312-1357, 1359-1409, 1527-1573
 *   avr_roundtrip_file   roundtrip(input, out)           recode.cpp:1594-1624
 *   avr_compress_files / avr_decompress_files  the two runs above over a corpus of files at once
 *   avr_roundtrip_files  roundtrip() over a corpus of files at once
 *   avr_compress_slices  compressor::cabac_decoder x N    recode.cpp:1134-1268 (+ h264_model 615-1059,
 *                        (one CABAC slice per wavefront)  h264_symbol::execute 1061-1100,
 *                                                         arithmetic_code.h encoder 89-203)
 *   avr_decompress_slices decompressor::cabac_decoder x N recode.cpp:1411-1520 (+ cabac_code.h 27-80,
 *                                                         arithmetic_code.h decoder 211-298)
 *   avr_hook_*           the libavcodec-hooks callback surface, AVCodecHooks    recode.cpp:137-228
 *                        (cabac.init_decoder/get/get_bypass/get_terminate/skip_bytes, model.frame_spec/
 *                        mb_xy/begin_sub_mb/end_sub_mb/begin_coding_type/end_coding_type)
 * The device kernels own the CABAC parse; the hooks layer serves the bins the device decoded to a
 * libavcodec-hooks caller, call by call, and checks the caller's parse against the device's.
 */
#ifndef AVRECODE_AMD_H
#define AVRECODE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVRECODE_ABI_VERSION 6  /* 6: the parallel model's long-slice split (avr_set_split_bytes, Block field 16);
                                 * 5: avr_slice_desc.file_offset (96 B), dec-plan handle, ranged parse */

typedef enum {
  AVR_OK = 0,
  AVR_ERR_INVALID_ARGUMENT = -1,
  AVR_ERR_DEVICE = -2,          /* HIP error; see avr_last_error */
  AVR_ERR_FORMAT = -3,          /* malformed input file / container */
  AVR_ERR_OUT_OF_MEMORY = -4,
  AVR_ERR_ROUNDTRIP = -5,       /* decompress(compress(x)) != x */
  AVR_ERR_UNSUPPORTED = -6,
} avr_status;

/* Model modes.  REFERENCE = recode.cpp's h264_model exactly (estimators persist across slices,
 * previous-frame and cross-slice contexts); output bytes equal the reference compressor's.
 * Sequential over slices (one wavefront for the whole file).
 * PARALLEL = the same model applied to every slice from a fresh state; slices are
 * independent, one wavefront per slice, shardable across GPUs.  Its decisions go through the
 * reference's own coder, arithmetic_code<uint64_t, uint8_t> with p1 = (range / (pos + neg)) * pos
 * (arithmetic_code.h:106-126, 232-248; recode.cpp:315-316, 816-820).  Tagged in
 * Recoded.Metadata.version as "avrecode-amd:P64".
 * PARALLEL32 = the parallel model with this library's optional 32-bit range coder (byte digits,
 * r1 = floor(range * floor(2^32 / tot) / 2^32) * pos; avr_engine.h PEncoder): fewer instructions per
 * decision, not the reference's arithmetic.  Tagged "avrecode-amd:P32".  Containers of every mode
 * decompress with avr_decompress_file, which reads the tag. */
/* AVR_MODEL_CHAINED: the reference model in chains -- a fresh model (estimators and frame metadata,
 * as at the start of a file) before every AVR_CHAIN_SLICES-th coded slice of a file, tagged
 * "avrecode-amd:R16".  It compresses like the reference model (the estimators learn across a chain's
 * 16 slices: realshort.mp4 0.998, cockatoo.mp4 0.994 of the input, against 0.990 / 0.991 for the
 * reference model and 1.041 / 1.010 for the parallel one), and a file's chains decode on as many
 * workgroups at once.  Whole-file calls only (avr_compress_file(s), avr_decompress_file(s),
 * avr_roundtrip_file(s), the hooks sessions -- the streaming one makes its container at
 * avr_hooks_end from the complete file, as for the reference model -- and the per-rank chain
 * ranges of one file, avr_compress_chain_range / avr_decompress_chain_range); the device
 * slice-batch calls refuse it with AVR_ERR_INVALID_ARGUMENT. */
typedef enum { AVR_MODEL_REFERENCE = 0, AVR_MODEL_PARALLEL = 1, AVR_MODEL_PARALLEL32 = 2, AVR_MODEL_CHAINED = 3 } avr_model;
#define AVR_CHAIN_SLICES 16

typedef struct avr_ctx avr_ctx;

/* device = HIP device ordinal.  Fails with AVR_ERR_DEVICE when no usable GPU is present: the
 * library has no CPU implementation of the hot path. */
int avr_create(int device, avr_ctx** out);
void avr_destroy(avr_ctx* ctx);
const char* avr_last_error(const avr_ctx* ctx);
/* free a buffer returned by the library */
void avr_free(void* p);

/* The parallel model's long-slice split (this library's own format; not in the reference, which
 * decodes a slice as one chain, recode.cpp:1411-1520).  The whole-file compress of AVR_MODEL_PARALLEL
 * cuts a progressive-frame slice at macroblock-row starts into pieces -- a cut candidate every
 * 8 * split_bytes decoded CABAC bits with half a piece still ahead -- each re-coded with a fresh
 * model, so the slice decompresses one workgroup per piece.  Block.cabac holds the pieces' streams
 * one after the other; Block field 16 ("seams", zlib) what each piece's decompress needs from before
 * it (its first macroblock and output byte, the CABAC re-encoder's state, the context states, the
 * upper row's neighbour fields).  Such containers decompress through the whole-file calls
 * (avr_decompress_file(s), avr_roundtrip_file(s)) and the hooks sessions (which regenerate one
 * whole at begin, as a reference-model container); the per-slice plans (avr_plan_decompress,
 * avr_dec_plan_load) refuse them with AVR_ERR_UNSUPPORTED.  split_bytes = 0: no split.  Default: the environment's AVR_SPLIT_BYTES, else 98304.  Checked by the oracle's
 * restatement (oracle/oracle_seams.c). */
int avr_set_split_bytes(avr_ctx* ctx, size_t split_bytes);
size_t avr_get_split_bytes(const avr_ctx* ctx);

/* ------------------------------------------------------------------ whole files (host memory) */
/* in: an MP4 (avcC) or Annex-B H.264 file.  *out: serialized Recoded protobuf (recode.proto). */
int avr_compress_file(avr_ctx* ctx, const uint8_t* in, size_t n, int model, uint8_t** out, size_t* out_len);
/* in: a Recoded protobuf.  *out: the original file bytes. */
int avr_decompress_file(avr_ctx* ctx, const uint8_t* in, size_t n, uint8_t** out, size_t* out_len);

/* Several files at once (a corpus): compressor::run / decompressor::run (recode.cpp:1102-1357) for
 * each of in[0 .. n_files), with the device work of all files batched.  A file is the reference
 * model's unit of sequential work (its estimators persist across ITS slices, recode.cpp:662-665, and
 * nothing crosses files), so reference-model files run side by side: the compress side in one
 * parallel pass over every slice of every file with per-file estimators, the decompress side one
 * workgroup (wavefront) per file; parallel-model slices of all files run one wavefront each.
 * out[f] / out_len[f]: file f's result (malloc'd, avr_free; NULL on failure).  status (optional,
 * n_files entries) receives each file's status and the call returns AVR_OK unless the batch as a
 * whole failed; without it the call returns the first file failure -- and out[f] is still set for
 * every file that succeeded, so the caller frees every non-NULL out[f] whatever the call returns.
 * avr_last_error holds one message: the last failing file's.  Output bytes equal
 * avr_compress_file / avr_decompress_file on each file alone. */
int avr_compress_files(avr_ctx* ctx, int n_files, const uint8_t* const* in, const size_t* in_len, int model,
                       uint8_t** out, size_t* out_len, int32_t* status);
int avr_decompress_files(avr_ctx* ctx, int n_files, const uint8_t* const* in, const size_t* in_len, uint8_t** out,
                         size_t* out_len, int32_t* status);

/* Where the wall time of a whole-file call goes (seconds).  Host phases by wall clock, device
 * phases by HIP events on the context's stream (summed over the call's device passes):
 *   demux_s      compress: demux, NAL unescape, parameter-set / slice-header parse, plan building;
 *                decompress: container parse, surrogate stream, header parse, plan building
 *   upload_s     host -> device copies of payloads / re-coded streams and descriptors
 *   kernel_s     the device passes (slice kernels, schedule, R-mode scan / sort / coder, verify)
 *   download_s   device -> host copies of results and outputs
 *   container_s  compress: segmentation + Recoded protobuf (and the reference model's re-plans);
 *                decompress: splicing literals + regenerated slices, last-byte patch
 *   other_s      the rest of the call's wall time (allocation, launch and synchronisation
 *                overhead) */
typedef struct {
  double demux_s, upload_s, kernel_s, download_s, container_s, other_s;
} avr_phase_times;

typedef struct {
  uint64_t file_bytes, slices, coded_slices, skipped_slices, payload_bytes, recoded_bytes, bins;
  double compress_s, decompress_s;  /* wall time of the two halves (host + device), summed over attempts */
  /* h264_model::bill / cabac_bill (recode.cpp:615-661), indexed by avr_pip_coding_type: bytes the
   * re-coded encoder emitted per put during compress (recode.cpp:1074-1078, 1213-1220) and bytes
   * the CABAC encoder emitted per put during decompress (1443-1446, 1455-1457, 1466-1468), summed
   * over the file's coded slices (the parallel model's per-slice models included). */
  uint64_t bill[6], cabac_bill[6];
  /* compress + decompress passes the roundtrip took: 1, or 2 when the parallel model's unverified
   * first pass did not come back and the file was compressed again with the per-slice check */
  uint32_t attempts, reserved;
  avr_phase_times compress_phases, decompress_phases;   /* summed over attempts */
} avr_file_stats;
/* The phase breakdown of the last whole-file call on ctx (avr_compress_file(s),
 * avr_decompress_file(s), avr_roundtrip_file: its last decompress). */
int avr_last_phase_times(const avr_ctx* ctx, avr_phase_times* out);
/* compress, decompress, compare (recode.cpp:1594-1624).  Returns AVR_ERR_ROUNDTRIP on mismatch. */
int avr_roundtrip_file(avr_ctx* ctx, const uint8_t* in, size_t n, int model, uint8_t** compressed,
                       size_t* compressed_len, avr_file_stats* stats);
/* avr_roundtrip_file (roundtrip(), recode.cpp:1594-1624) over a corpus, with the device work of
 * all files batched as in avr_compress_files / avr_decompress_files: every file compressed (the parallel model without its
 * per-slice device check), every container decompressed and compared with its input; the files
 * that do not come back are compressed again with the check, decompressed and compared again.
 * out[f] / out_len[f]: file f's container (malloc'd, avr_free; NULL when it failed), status[f]: its
 * result (AVR_ERR_ROUNDTRIP when even the checked container does not restore it).  times (optional,
 * 2 entries): wall seconds of the compress and the decompress calls, summed over attempts.  Returns
 * AVR_OK unless the batch as a whole failed. */
int avr_roundtrip_files(avr_ctx* ctx, int n_files, const uint8_t* const* in, const size_t* in_len, int model,
                        uint8_t** out, size_t* out_len, int32_t* status, double* times);

/* ------------------------------------------------------- slice batches (device-resident data) */
/* One CABAC slice: the (buf, size) FFmpeg hands to AVCodecHooks.cabac.init_decoder
 * (recode.cpp:143), plus the slice-header fields the slice_data() parse needs. */
typedef struct {
  uint64_t payload_offset;   /* byte offset of the CABAC payload in the input buffer */
  uint32_t payload_size;     /* init_decoder's size */
  uint32_t read_limit;       /* bytes readable from payload_offset (>= payload_size) */
  uint64_t out_offset;       /* where this slice's output goes in the output buffer */
  uint32_t out_capacity;     /* bytes reserved there */
  int32_t slice_type;        /* 0 P, 1 B, 2 I */
  int32_t slice_qp, cabac_init_idc, first_mb, mb_width, mb_height;
  int32_t num_ref_idx_l0, num_ref_idx_l1;
  int32_t chroma_array_type, transform_8x8_mode, direct_8x8_inference, x264_build;
  int32_t picture_id;        /* decode-order picture counter (frame_spec, recode.cpp:824-843) */
  int32_t coded;             /* 0: skip_coded slice (reference mode only calls frame_spec) */
  int32_t structure;         /* AVR_STRUCT_*: frame, top / bottom field picture (PAFF), MBAFF frame;
                              * mb_height is the FRAME height in macroblocks in every case */
  uint64_t file_offset;      /* host only (avr_parse_stream): where the payload's bytes stand verbatim in
                              * the parsed file (its NAL has no emulation-prevention bytes), else
                              * UINT64_MAX; the container assembly's segmentation starts there
                              * (recode.cpp:1275-1297).  The kernels ignore it. */
} avr_slice_desc;
enum { AVR_STRUCT_FRAME = 0, AVR_STRUCT_TOP_FIELD = 1, AVR_STRUCT_BOTTOM_FIELD = 2, AVR_STRUCT_MBAFF = 3 };

/* avr_slice_result.status: 0, or why the slice cannot be coded (the container stores it skip_coded) */
enum {
  AVR_SLICE_OK = 0,
  AVR_SLICE_PCM = -2,             /* I_PCM macroblock (skip_bytes; the reference throws, recode.cpp:161-163) */
  AVR_SLICE_BAD_REF_IDX = -3,     /* ref_idx unary prefix past 32 */
  AVR_SLICE_BAD_MVD = -4,         /* mvd suffix exponent past 24 */
  AVR_SLICE_BAD_LEVEL = -5,       /* coeff_abs_level_minus1 suffix exponent past 30 */
  AVR_SLICE_BAD_QP_DELTA = -6,    /* mb_qp_delta past 102 */
  AVR_SLICE_BAD_MB_ADDR = -7,     /* macroblock address past the picture */
  AVR_SLICE_OVERREAD = -8,        /* the parse ran past the payload */
  AVR_SLICE_NO_END = -9,          /* the walk ended without end_of_slice_flag = 1 */
  AVR_SLICE_CODER = -10,          /* coder invariant violated (carry into an emitted byte: corrupt input) */
  AVR_SLICE_NO_STOP = -11,        /* compress: a CABAC re-encode would not restore the payload (last-byte rule) */
  AVR_SLICE_OVERFLOW = -12,       /* output past out_capacity */
  AVR_SLICE_MBAFF_RING = -20,     /* MBAFF slice launched with max_mb_width < 3 * mb_width + 7 */
  AVR_SLICE_NO_ROUNDTRIP = -21    /* file calls: the device roundtrip check did not regenerate the payload */
};

typedef struct {
  uint32_t out_len;          /* bytes written at out_offset */
  int32_t status;            /* AVR_SLICE_*: 0 ok, < 0 the slice must be stored skip_coded */
  uint32_t bins;             /* CABAC bins processed */
  uint32_t mbs;              /* macroblocks parsed */
  /* h264_model billing of this slice by avr_pip_coding_type (recode.cpp:615-661), filled only
   * by the whole-file calls (zero from the batch entry points): compress = re-coded bytes emitted
   * per put (h264_model::bill), decompress = CABAC bytes emitted per put (cabac_bill). */
  uint32_t bill[6];
} avr_slice_result;

/* All pointers are device pointers; stream is a hipStream_t (NULL = default stream).
 * Compress: payload bytes -> re-coded bytes.  For each slice the kernel also checks that a
 * CABAC re-encode plus the decompressor's last-byte rule (recode.cpp:1345-1356, 1503-1505)
 * restores the payload, and reports status < 0 otherwise. */
/* max_mb_width / max_mb_height bound every slice's picture size (LDS ring and frame sizing).
 * max_mb_width is the LDS ring's width in macroblock records: mb_width, or 3 * mb_width + 7 for an
 * AVR_STRUCT_MBAFF slice (its pair records live there too) -- the value avr_parse_stream reports.
 * An MBAFF slice launched with less fails alone (status < 0). */
int avr_compress_slices(avr_ctx* ctx, const avr_slice_desc* d_desc, int n, int max_mb_width, int max_mb_height,
                        const uint8_t* d_in, uint8_t* d_out, avr_slice_result* d_res, int model, void* stream);
/* Decompress: re-coded bytes (at payload_offset/payload_size = recoded stream) -> regenerated
 * CABAC bytes at out_offset (before the last-byte patch; trailing 0x80 already dropped). */
int avr_decompress_slices(avr_ctx* ctx, const avr_slice_desc* d_desc, int n, int max_mb_width, int max_mb_height,
                          const uint8_t* d_in, uint8_t* d_out, avr_slice_result* d_res, int model, void* stream);
/* Pack variable-length per-slice outputs contiguously: d_packed[k] gets slice k's bytes at
 * d_offsets[k] (exclusive prefix sum of out_len, computed on the device). */
int avr_pack_outputs(avr_ctx* ctx, const avr_slice_desc* d_desc, const avr_slice_result* d_res, int n,
                     const uint8_t* d_out, uint8_t* d_packed, uint64_t* d_offsets, void* stream);

/* Device-resident roundtrip of a slice batch: recode.cpp:1594-1624 applied per slice, without the
 * container.  Compress d_in -> d_work (at each desc's out_offset), derive the decompress
 * descriptors on the device (d_dec_desc, n entries of scratch), decompress d_work -> d_regen
 * (slice k at d_desc[k].payload_offset, i.e. d_regen has d_in's layout), then apply the last-byte
 * rule (recode.cpp:1345-1356) and compare with the payload.  d_verdict[k]: 1 bit-exact,
 * 0 mismatch, 2 not coded (compress status != 0: the container stores it skip_coded).
 * Everything is enqueued on `stream`; nothing is synchronised. */
int avr_roundtrip_slices(avr_ctx* ctx, const avr_slice_desc* d_desc, int n, int max_mb_width, int max_mb_height,
                         const uint8_t* d_in, uint8_t* d_work, uint8_t* d_regen, avr_slice_desc* d_dec_desc,
                         avr_slice_result* d_res_c, avr_slice_result* d_res_d, int32_t* d_verdict, int model,
                         void* stream);

/* The two device steps avr_roundtrip_slices runs between its compress and decompress launches,
 * for callers that time or overlap the halves themselves (same semantics as above). */
int avr_derive_decompress_descs(avr_ctx* ctx, const avr_slice_desc* d_desc, const avr_slice_result* d_res_c, int n,
                                avr_slice_desc* d_dec_desc, void* stream);
int avr_verify_slices(avr_ctx* ctx, const avr_slice_desc* d_desc, const avr_slice_result* d_res_c,
                      const avr_slice_result* d_res_d, int n, const uint8_t* d_in, const uint8_t* d_regen,
                      int32_t* d_verdict, void* stream);

/* The chained model (AVR_MODEL_CHAINED) across GPUs, within one file.  Its chains are independent
 * (a fresh reference model before every AVR_CHAIN_SLICES-th coded slice), so a file's chains are cut
 * into `world` contiguous ranges balanced by payload bytes (the rule of the Python shard.partition)
 * and rank `rank` runs its range on this context's GPU:
 *   avr_compress_chain_range: the file parsed and segmented as avr_compress_file does it, then the
 *     reference-model pass over this rank's chains (compressor::run, recode.cpp:1102-1132, with the
 *     model restarted per chain, 662-665).  Outputs for the file's slices [*lo, *hi): status 0 =
 *     coded (its re-coded bytes at recoded + offsets[k], lens[k]), -1 = not coded, -2 = a coded
 *     slice the pass failed (avr_compress_file would demote it and re-segment, which moves every
 *     later chain: compress the file whole instead).  The ranks' outputs, concatenated in rank order,
 *     are avr_assemble_container's status / recoded / offsets / lens for model AVR_MODEL_CHAINED:
 *     byte-identical to avr_compress_file(file, AVR_MODEL_CHAINED).
 *   avr_decompress_chain_range: the container planned as avr_decompress_file plans it (every slice,
 *     coded or not), this rank's chains regenerated (decompressor::cabac_decoder, recode.cpp:
 *     1411-1520, one chain per workgroup).  Outputs for the plan's slices [*lo, *hi): status 0 =
 *     regenerated (bytes at regen + offsets[k], lens[k]), 1 = not coded, < 0 failed.  Concatenated in
 *     rank order they are avr_dec_plan_splice's inputs on a plan of the same container.  A
 *     reference-model container is one unit (rank 0 takes it whole).
 * Buffers are allocated here (avr_free).  No reference counterpart: the reference is one CPU thread. */
int avr_compress_chain_range(avr_ctx* ctx, const uint8_t* file, size_t n, int world, int rank, int* lo, int* hi,
                             int32_t** status, uint8_t** recoded, size_t* recoded_len, uint64_t** offsets,
                             uint32_t** lens);
int avr_decompress_chain_range(avr_ctx* ctx, const uint8_t* avrc, size_t n, int world, int rank, int* lo, int* hi,
                               int32_t** status, uint8_t** regen, size_t* regen_len, uint64_t** offsets,
                               uint32_t** lens);

/* Which device kernel a parallel-model batch of n slices (widest picture max_mb_width macroblocks)
 * runs on this context's GPU, by the rule avr_compress_slices / avr_decompress_slices apply:
 * *kind = 0 the resident kernel (slices_parallel_kernel: one workgroup per slice, the whole batch
 * resident at once), 1 the persistent queue kernel (slices_queue_kernel: more slices than the chip
 * holds at once, or pictures wide enough that their model row lives in global scratch).  For
 * naming the measured kernel in profiles; no reference counterpart (the reference is one CPU
 * thread). */
int avr_slice_kernel(avr_ctx* ctx, int decompress, int n, int max_mb_width, int* kind);

/* ------------------------------------------------------------ host-side slice extraction */
/* What FFmpeg hands AVCodecHooks.cabac.init_decoder for every CABAC slice of a file
 * (av_decoder::decode_video, recode.cpp:73-135): demux (MP4/avcC or Annex-B), unescape, parse
 * SPS/PPS/SEI/slice headers.  Host only, no device needed.  Returns malloc'd arrays (free with
 * avr_free): *descs (n entries; payload_offset/read_limit index *arena, out_offset/out_capacity
 * index a work buffer of *work_len bytes sized for compress output) and *arena (payloads, each
 * 16-byte aligned, followed by >= 16 zero bytes).  desc.coded = 0 for slices the recoder does not
 * take (unsupported syntax, or shorter than a surrogate marker, recode.cpp:1285). */
int avr_parse_stream(const uint8_t* file, size_t n, avr_slice_desc** descs, int* n_slices, uint8_t** arena,
                     size_t* arena_len, size_t* work_len, int* max_mb_width, int* max_mb_height);
/* avr_parse_stream for the slices [lo, hi) only (hi < 0: to the end), descs and arena rebased to
 * them: a rank of a sharded compress takes its own range of a stream without copying the rest
 * (the whole stream's headers are still parsed: slice indices and picture ids are the file's). */
int avr_parse_stream_range(const uint8_t* file, size_t n, int lo, int hi, avr_slice_desc** descs, int* n_slices,
                           uint8_t** arena, size_t* arena_len, size_t* work_len, int* max_mb_width,
                           int* max_mb_height);
/* The payload_size of every CABAC slice of a file (what avr_parse_stream reports), without copying a
 * payload: the input of a sharded run's partition on every rank.  *sizes malloc'd (avr_free). */
int avr_slice_payload_sizes(const uint8_t* file, size_t n, uint32_t** sizes, int* n_slices);

/* Rank 0 of a sharded PARALLEL-model compress: build the Recoded container from per-slice outputs
 * gathered from every rank (compressor::run + find_next_coded_block_and_emit_literal,
 * recode.cpp:1115-1132, 1275-1297).  Host only.  model = the model the outputs were made with (the
 * container's tag): AVR_MODEL_PARALLEL / _PARALLEL32 (avr_compress_slices on each rank's slice
 * range), or AVR_MODEL_CHAINED (avr_compress_chain_range on each rank's chains).  Slice k (avr_parse_stream order) is
 * coded when it is a candidate and status[k] == 0; its re-coded bytes are recoded[offsets[k] ..
 * + lens[k]), inside recoded_len (AVR_ERR_INVALID_ARGUMENT otherwise).  The result is
 * byte-identical to avr_compress_file(..., model).  avr_assemble_container parses `file` again;
 * avr_assemble_container_parsed takes avr_parse_stream's descs and arena for it instead (the parse
 * a sharded caller already holds: no second pass over a multi-GB stream).  Only that call's output,
 * unmodified, for this file is accepted: a coded desc must be a recodable candidate and a verbatim
 * payload must stand at its file_offset (checked on its first and last bytes; otherwise
 * AVR_ERR_INVALID_ARGUMENT).  The segmentation searches only each slice's literal gap when the parse
 * found its payload verbatim, and the container is written once, its bytes copied by host threads. */
int avr_assemble_container(const uint8_t* file, size_t n, int model, int n_slices, const int32_t* status,
                           const uint8_t* recoded, size_t recoded_len, const uint64_t* offsets, const uint32_t* lens,
                           uint8_t** out, size_t* out_len);
int avr_assemble_container_parsed(const uint8_t* file, size_t n, int model, const avr_slice_desc* descs, int n_slices,
                                  const uint8_t* arena, size_t arena_len, const int32_t* status,
                                  const uint8_t* recoded, size_t recoded_len, const uint64_t* offsets,
                                  const uint32_t* lens, uint8_t** out, size_t* out_len);
/* avr_assemble_container_parsed into the caller's buffer out (out_cap bytes): a step that assembles
 * every time reuses one buffer, already mapped, instead of a fresh multi-GB allocation.  *out_len =
 * the container's size; when it exceeds out_cap nothing is written and AVR_ERR_INVALID_ARGUMENT is
 * returned with *out_len set.  A bound: n + sum(lens of coded slices) + 64 (n_slices + 2). */
int avr_assemble_container_into(const uint8_t* file, size_t n, int model, const avr_slice_desc* descs, int n_slices,
                                const uint8_t* arena, size_t arena_len, const int32_t* status, const uint8_t* recoded,
                                size_t recoded_len, const uint64_t* offsets, const uint32_t* lens, uint8_t* out,
                                size_t out_cap, size_t* out_len);
/* The model mode a Recoded container was written with (its Metadata.version): AVR_MODEL_*.
 * AVR_ERR_FORMAT for bytes that are not a Recoded message or name another avrecode-amd format. */
int avr_container_model(const uint8_t* avrc, size_t n, int* model);

/* Sharded PARALLEL-model decompress (decompressor::run, recode.cpp:1312-1357, split over ranks).
 * avr_plan_decompress: the container's coded slices as a decompress batch, host only -- *descs
 * (n entries, in container order; payload_offset / read_limit / payload_size index *arena = the
 * re-coded streams, out_offset / out_capacity index a work buffer of *work_len bytes for the
 * regenerated CABAC bytes) for avr_decompress_slices on any rank's slice range.  Returns
 * AVR_ERR_UNSUPPORTED for a reference-model container (its slices chain: replicas only).
 * avr_splice_container (rank 0): the original file from the container's literals and slice k's
 * regenerated bytes regen[offsets[k] .. + lens[k]) (avr_decompress_slices output before the
 * last-byte patch, which this applies, recode.cpp:1345-1356); status[k] != 0 fails the file with
 * AVR_ERR_FORMAT; a slice whose bytes lie outside regen_len or exceed its descriptor's out_capacity
 * gives AVR_ERR_INVALID_ARGUMENT.  Byte-identical to avr_decompress_file.  A sharded caller
 * decompresses the batch with the container's model (avr_container_model). */
int avr_plan_decompress(const uint8_t* avrc, size_t n, avr_slice_desc** descs, int* n_slices, uint8_t** arena,
                        size_t* arena_len, size_t* work_len, int* max_mb_width, int* max_mb_height);
int avr_splice_container(const uint8_t* avrc, size_t n, int n_slices, const int32_t* status, const uint8_t* regen,
                         size_t regen_len, const uint64_t* offsets, const uint32_t* lens, uint8_t** out,
                         size_t* out_len);

/* The sharded decompress's host halves on one parse (decompressor::run, recode.cpp:1338-1409):
 * a plan handle loads a container -- read_packet's surrogate stream parsed and
 * matched to the coded blocks, as avr_plan_decompress, but without copying any bytes yet -- then
 * writes the descriptors and the re-coded streams' arena where the caller wants them (the arena
 * with host threads), and splices the regenerated slices with the literals and the last-byte patch
 * (recode.cpp:1345-1356) into the caller's buffer, as avr_splice_container.  The container must stay
 * alive and unchanged from avr_dec_plan_load to the last call on it; a handle keeps its scratch
 * (the surrogate stream's buffer) for the next load.  arena_len / work_len / max_mb_* as
 * avr_plan_decompress.  avr_dec_plan_splice: *out_len = the file's size; AVR_ERR_INVALID_ARGUMENT
 * when out_cap is smaller (nothing written) or a slice's bytes lie outside regen or past its
 * capacity, AVR_ERR_FORMAT when a coded block has no slice or a slice's status is not 0.  A
 * parallel-model plan lists the coded slices (one device batch); a reference- or chained-model plan
 * lists every slice, coded or not (the reference model turns frames over on uncoded ones), which is
 * the indexing avr_decompress_chain_range's outputs use. */
typedef struct avr_dec_plan avr_dec_plan;
int avr_dec_plan_new(avr_dec_plan** out);
void avr_dec_plan_free(avr_dec_plan* plan);
int avr_dec_plan_load(avr_dec_plan* plan, const uint8_t* avrc, size_t n, int* n_slices, size_t* arena_len,
                      size_t* work_len, int* max_mb_width, int* max_mb_height);
int avr_dec_plan_descs(const avr_dec_plan* plan, avr_slice_desc* out);
int avr_dec_plan_arena(const avr_dec_plan* plan, uint8_t* out, size_t cap);
int avr_dec_plan_splice(const avr_dec_plan* plan, const int32_t* status, const uint8_t* regen, size_t regen_len,
                        const uint64_t* offsets, const uint32_t* lens, uint8_t* out, size_t out_cap, size_t* out_len);

/* Container codec check (host only): parse a Recoded protobuf (recode.proto:1-19) with the
 * library's own wire codec -- the one avr_decompress_file uses -- and return (a) its fields as JSON,
 * {"version": null | hex, "blocks": [{"size": int, "literal": hex, "skip_coded": bool, "cabac": hex,
 * "length_parity": bool, "last_byte": hex}, ...]} with only the fields present, and (b) the message
 * re-serialised by the library's writer (the one avr_compress_file uses; Metadata.version only).
 * Both buffers are malloc'd (avr_free).  AVR_ERR_FORMAT when the bytes are not a Recoded message. */
int avr_container_describe(const uint8_t* in, size_t n, char** json, uint8_t** reserialized, size_t* len);

/* Model neighbour geometry (get_neighbor_sub_mb + reverse_scan_8, recode.cpp:279-312, 419-471) as the
 * kernels use it (HotTables::nb_left / nb_up, loaded into every workgroup's LDS): out[n] (n < 48) =
 * the 4x4 block left of block n, out[48 + n] = the block above it, | 128 when that block lies in
 * the left / upper macroblock.  ctx NULL: the table the library builds on the host (no device
 * needed); a context: read back from that device's copy.  Pinned against the reference compiled
 * here by tests/test_oracle_geometry.py and tests/test_gpu_parity.py. */
int avr_neighbor_tables(avr_ctx* ctx, uint8_t out[96]);

/* ------------------------------------------------ libavcodec-hooks callback surface (AVCodecHooks) */
/* For a caller that drives the recode path from its own H.264 decoder exactly as the reference's
 * libavcodec-hooks fork does (recode.cpp:137-228).  A session runs the whole file on the device up
 * front (compress: recoded container + the decode-order bin trace of every coded slice;
 * decompress: the original file + the same traces), then serves the per-bin callbacks from the
 * traces: get() returns the bin and advances *state the way ff_get_cabac / cabac::encoder::put
 * would (recode.cpp:1176, 1443).  Every callback checks the caller's parse against the device's
 * (state byte before each decision, bin kinds, sub-MB / coding-type pairing, recode.cpp:185-189,
 * 933-947); a mismatch makes avr_hooks_end fail with AVR_ERR_FORMAT.  Not thread-safe.
 * LIMITATION (by design): the caller's parse never drives the model.  In the reference the
 * decoder's own calls decide the model keys bin by bin (recode.cpp:1435-1449); here the device's
 * parse (avr_walker.h) has decided every bin, key and coding-type event before the first callback,
 * and the callbacks only replay and verify it.  A caller whose decoder parses a slice differently
 * (another FFmpeg revision's syntax handling, a damaged stream it conceals) is refused with
 * AVR_ERR_FORMAT instead of being followed. */
typedef struct avr_hooks_session avr_hooks_session;

/* CodingType (EACH_PIP_CODING_TYPE, recode.cpp:616) */
typedef enum {
  AVR_PIP_UNKNOWN = 0, AVR_PIP_UNREACHABLE, AVR_PIP_SIGNIFICANCE_MAP, AVR_PIP_SIGNIFICANCE_EOB,
  AVR_PIP_SIGNIFICANCE_NZ, AVR_PIP_RESIDUALS
} avr_pip_coding_type;

/* compressor(input, out) (recode.cpp:1102-1113): file = the H.264 file the caller decodes. */
int avr_hooks_compress_begin(avr_ctx* ctx, const uint8_t* file, size_t n, int model, avr_hooks_session** out);
/* decompressor(input, out) (recode.cpp:1312-1336): avrc = a Recoded container.  *stream is what
 * read_packet feeds the decoder (literals + surrogate blocks, recode.cpp:1359-1409), valid until
 * avr_hooks_destroy.  A parallel-model container (avrecode-amd:P64 / P32) is decoded on demand, as
 * the reference decodes each slice when the decoder reaches it (recode.cpp:1411-1520): begin only
 * plans it; an avr_hook_init_decoder that reaches a slice not yet regenerated regenerates it on
 * the device together with at most 31 coded slices after it, and avr_hooks_end regenerates the
 * rest for the output file.  A reference-model container is regenerated whole at begin (its
 * estimators chain across slices).  AVR_HOOKS_EAGER=1 in the environment: always whole. */
int avr_hooks_decompress_begin(avr_ctx* ctx, const uint8_t* avrc, size_t n, avr_hooks_session** out,
                               const uint8_t** stream, size_t* stream_len);
/* Streaming compress: the caller's demuxer hands the file's bytes to the session as it reads them
 * (avr_hooks_feed: the fork's read_packet, recode.cpp:1127-1131) instead of the whole file up front.
 * Each init_decoder finds its slice in the bytes fed so far and traces that slice alone on the device
 * (the hooks answer with the CABAC parse, whichever model the container uses); a slice not yet fed
 * completely fails the session.  avr_hooks_end compresses the complete file with `model` -- the
 * container needs every slice's model state, as the reference writes it after the last slice
 * (recode.cpp:1102-1125) -- and returns it as avr_hooks_compress_begin's session would.  The
 * callbacks and their checks are the same. */
int avr_hooks_compress_stream_begin(avr_ctx* ctx, int model, avr_hooks_session** out);
int avr_hooks_feed(avr_hooks_session* s, const uint8_t* bytes, size_t n);
/* AVCodecHooks.cabac: opaque = the session.  init_decoder returns the per-slice opaque, or NULL
 * when the slice is not re-coded (the caller then decodes it natively, recode.cpp:1139-1145). */
void* avr_hook_init_decoder(void* opaque, void* cabac_context, const uint8_t* buf, int size);
int avr_hook_get(void* slice, uint8_t* state);
int avr_hook_get_bypass(void* slice);
int avr_hook_get_terminate(void* slice);
/* I_PCM is unsupported, as in the reference (recode.cpp:161-163): records an error, returns NULL. */
const uint8_t* avr_hook_skip_bytes(void* slice, int n);
/* AVCodecHooks.model: opaque = the session */
void avr_hook_frame_spec(void* opaque, int frame_num, int mb_width, int mb_height);
void avr_hook_mb_xy(void* opaque, int x, int y);
void avr_hook_begin_sub_mb(void* opaque, int cat, int scan8index, int max_coeff, int is_dc, int chroma422);
void avr_hook_end_sub_mb(void* opaque, int cat, int scan8index, int max_coeff, int is_dc, int chroma422);
void avr_hook_begin_coding_type(void* opaque, int coding_type, int zigzag_index, int param0, int param1);
void avr_hook_end_coding_type(void* opaque, int coding_type);
/* compress: *out = the Recoded container; decompress: *out = the original file (avr_free). */
int avr_hooks_end(avr_hooks_session* s, uint8_t** out, size_t* out_len);
void avr_hooks_destroy(avr_hooks_session* s);

/* --------------------------------------------------------------- synthetic H.264 (benchmarks) */
typedef struct {
  int32_t mb_width, mb_height;   /* e.g. 120 x 68 for 1080p */
  int32_t slice_type;            /* 0 P, 1 B, 2 I */
  int32_t slice_qp;
  int32_t chroma_format_idc;     /* 1 (4:2:0) .. 3 */
  int32_t transform_8x8_mode;
  int32_t num_ref_idx_l0, num_ref_idx_l1;
  uint64_t seed;
  int32_t slices_per_picture;    /* 0 or 1: one slice per picture; k: k slices (equal MB runs) */
  int32_t gop_length;            /* 0: every picture has slice_type; g > 0: picture i is an IDR
                                  * I picture when i % g == 0, else slice_type (e.g. I + 31 P);
                                  * with slice_type B: I B B P B B P ... (P when (i % g) % 3 == 0) */
  int32_t repeat;                /* 0 or 1: once; r > 1: the n generated pictures are written r
                                  * times, copy t with frame_num / idr_pic_id advanced by t n (a
                                  * long stream tiled from one GOP; the payloads repeat) */
  int32_t structure;             /* 0 progressive frames; 1 field pictures (PAFF: each picture a
                                  * top then a bottom field, mb_height even); 2 MBAFF frames (every
                                  * macroblock pair field or frame coded at random, mb_height even);
                                  * 3 field pictures, bottom field first */
} avr_synth_params;
/* Generate n pictures on the device (each slices_per_picture slices, in decode order) and return
 * them as one Annex-B stream (SPS/PPS + the slice NAL units) in host memory.  Pictures are
 * consecutive frames (frame_num / idr_pic_id = picture index), so the reference model's
 * previous-frame contexts (recode.cpp:824-843, 884) see each P picture's predecessor. */
int avr_synthesize_stream(avr_ctx* ctx, const avr_synth_params* params, int n, uint8_t** out, size_t* out_len);

#ifdef __cplusplus
}
#endif
#endif
