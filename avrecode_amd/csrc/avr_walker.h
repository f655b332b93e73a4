// The per-slice walker shared by the slice kernels (included by the avr_k_*.hip translation
// units only; each instantiates one kernel so the kernels compile in parallel).
//
// One wavefront (64 lanes) owns one CABAC slice and runs the whole hot path for it:
//   compress:    CABAC decode (fork ff_get_cabac*) -> H.264 slice_data() parse (the fork's
//                caller of the hooks) -> h264_model keys/estimators (recode.cpp:615-1059)
//                -> recoded arithmetic encode (arithmetic_code.h, recode.cpp:1061-1100, 1134-1268)
//   decompress:  recoded decode -> parse -> model -> CABAC re-encode (recode.cpp:1411-1520,
//                cabac_code.h)
//   generate:    seeded bins -> parse -> CABAC encode (synthetic benchmark slices)
// The serial part runs redundantly on all lanes (wave-uniform values); the lanes cooperate on
// staging the byte streams through LDS and on clearing the model tables.  Everything is inlined
// into the kernel (no calls, no private arrays) so the walker state lives in registers: a
// non-inlined member call would put the whole Walker in scratch memory.
//
// Model modes: RM = true reproduces recode.cpp exactly (estimators and frame metadata persist
// across slices; one wavefront walks all slices in file order).  RM = false applies the same
// model to each slice from a fresh state (independent slices, one wavefront per slice).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#include "../../include/avrecode.h"
#include "avr_engine.h"
#include "avr_kernels.h"

#define AVR_FI __device__ __forceinline__

// Cycle accounting per walker section, compiled in with -DAVR_PROFILE only (scripts/prof_sections):
// 0 slice, 1 macroblock syntax, 2 residual, 3 map decode, 4 nnz bins, 5 map re-code, 6 levels,
// 7 per-macroblock bookkeeping; [8 + i] bins coded in section i.  Summed over slices into avr_prof (one copy per TU).
#ifdef AVR_PROFILE
#define PROF_T() ((uint64_t)__builtin_readcyclecounter())
#define PROF_BEGIN(v) const uint64_t v = PROF_T(); const uint32_t v##_b = bins
#define PROF_BEGINW(v) const uint64_t v = PROF_T(); const uint32_t v##_b = w.bins
#define PROF_END(i, v) prof[i] += PROF_T() - (v), profb[i] += bins - v##_b
#define PROF_ENDW(i, v) w.prof[i] += PROF_T() - (v), w.profb[i] += w.bins - v##_b
// macroblock-layer sub-sections (avr_prof[32 + i] cycles, [40 + i] bins): 0 macroblock start,
// 1 mb_skip_flag, 2 mb_type + sub_mb_type, 3 intra prediction modes, 4 ref_idx, 5 mvd,
// 6 coded_block_pattern + transform_size_8x8_flag + mb_qp_delta, 7 end_of_slice + publish
#define SPROF_END(i, v) sprof[i] += PROF_T() - (v), sprofb[i] += bins - v##_b
#define SPROF_ENDW(i, v) w.sprof[i] += PROF_T() - (v), w.sprofb[i] += w.bins - v##_b
#else
#define SPROF_END(i, v)
#define SPROF_ENDW(i, v)
#define PROF_BEGINW(v)
#define PROF_ENDW(i, v)
#define PROF_BEGIN(v)
#define PROF_END(i, v)
#endif

namespace avr {

#if defined(AVR_PROFILE) && defined(AVR_WATCHDOG)
#error "AVR_WATCHDOG records share avr_prof with the AVR_PROFILE section counters: build one at a time"
#endif
#if defined(AVR_PROFILE) || defined(AVR_WATCHDOG)
static __device__ unsigned long long avr_prof[64];
#endif
#ifdef AVR_PROFILE
// wave placement per slice (AVR_PROFILE builds): HW_ID of waves 0..2, XCC_ID, walker start / end
// (s_memtime low 32 bits), walker start / end (s_memrealtime, 100 MHz) -- scripts/placement.py
constexpr int kPlaceSlices = 4096;
static __device__ uint32_t avr_place[kPlaceSlices][8];
AVR_FI void record_placement(int s, int wave) {
  if (s < kPlaceSlices && __lane_id() == 0) {
    avr_place[s][wave] = __builtin_amdgcn_s_getreg(4 | (31 << 11));        // HW_REG_HW_ID
    if (wave == 0) avr_place[s][3] = __builtin_amdgcn_s_getreg(20 | (15 << 11));  // HW_REG_XCC_ID
  }
}
#define AVR_PLACE(s, wave) record_placement(s, wave)
#define AVR_PLACE_T(s, k) if ((s) < kPlaceSlices && __lane_id() == 0) { \
    avr_place[s][4 + (k)] = (uint32_t)__builtin_readcyclecounter(); \
    avr_place[s][6 + (k)] = (uint32_t)__builtin_amdgcn_s_memrealtime(); }
#else
#define AVR_PLACE(s, wave)
#define AVR_PLACE_T(s, k)
#endif

// MODE_TRACE: the compress-side CABAC decode + parse alone, recording every bin in decode order
// (2 bytes: bin | kind << 1, the context's state byte before the bin) -- the bin sequence the
// libavcodec-hooks layer (avr_hook_*) serves to its caller -- and, between the bins, the model
// events that decide the model keys (kind 3 records, TRACE_EV_*): where each significance map
// begins and ends, with the model coordinates (mb_xy) and sub-macroblock (begin_sub_mb) it runs
// under; the hooks layer checks the caller's begin/end_coding_type(SIG_MAP), mb_xy and
// begin_sub_mb against them (recode.cpp:166-207, 951-974).
enum { MODE_COMPRESS = 0, MODE_DECOMPRESS = 1, MODE_GENERATE = 2, MODE_TRACE = 3 };
enum { F_DEC = 1, F_SKIP = 2, F_INTRA = 4, F_I16 = 8, F_D16 = 16, F_T8 = 32, F_CPRED = 64 };
enum { SE_OTHER = 0, SE_REF, SE_QPDELTA, SE_MVD_SUFFIX, SE_LEVEL_SUFFIX, SE_EOS, SE_PCM };
// MODE_TRACE event records: 0x06 (kind 3), type, payload.  MAP_BEGIN: mb_x, model row (u16 LE
// each), cat, scan8 index, max_coeff, is_dc | chroma422 << 1 (10 bytes); MAP_END: 2 bytes.
enum { TRACE_EV_MAP_BEGIN = 1, TRACE_EV_MAP_END = 2 };

static __constant__ uint8_t c_scan8[51] = {
  4 + 1 * 8,  5 + 1 * 8,  4 + 2 * 8,  5 + 2 * 8,  6 + 1 * 8,  7 + 1 * 8,  6 + 2 * 8,  7 + 2 * 8,
  4 + 3 * 8,  5 + 3 * 8,  4 + 4 * 8,  5 + 4 * 8,  6 + 3 * 8,  7 + 3 * 8,  6 + 4 * 8,  7 + 4 * 8,
  4 + 6 * 8,  5 + 6 * 8,  4 + 7 * 8,  5 + 7 * 8,  6 + 6 * 8,  7 + 6 * 8,  6 + 7 * 8,  7 + 7 * 8,
  4 + 8 * 8,  5 + 8 * 8,  4 + 9 * 8,  5 + 9 * 8,  6 + 8 * 8,  7 + 8 * 8,  6 + 9 * 8,  7 + 9 * 8,
  4 + 11 * 8, 5 + 11 * 8, 4 + 12 * 8, 5 + 12 * 8, 6 + 11 * 8, 7 + 11 * 8, 6 + 12 * 8, 7 + 12 * 8,
  4 + 13 * 8, 5 + 13 * 8, 4 + 14 * 8, 5 + 14 * 8, 6 + 13 * 8, 7 + 13 * 8, 6 + 14 * 8, 7 + 14 * 8,
  0 + 0 * 8,  0 + 5 * 8,  0 + 10 * 8,
};
static __constant__ uint8_t c_b_pairs[9][2] = {{1, 1}, {2, 2}, {1, 2}, {2, 1}, {1, 3}, {2, 3}, {3, 1}, {3, 2}, {3, 3}};
constexpr int kSigEst = 229376;
constexpr int kNzEst = 63 * 2 * 3 * 3 * 57;
constexpr int kEstDefault = 1026;
static_assert(kEstTable >= kSigEst + kNzEst, "estimator table size");

struct MbRec {
  uint8_t flags, is8x8;
  uint16_t cbp;         // FFmpeg cbp_table layout: luma b0-3, chroma b4-5, chroma DC b6-7, luma DC b8-10
  uint8_t nnz[3][16];   // coefficient count per 4x4, raster per plane
  uint8_t mvd[2][16][2];
  int8_t ref[2][4];
  uint8_t direct8[4];
  uint8_t mnnz[52];     // model BlockMeta.num_nonzeros[51]
};
// bottom edge of the macroblock above, dword j gathered from MbRec dword Walker::edge_src (lane j)
// at the publish; 92 B keeps four 1080p workgroups within a CU's LDS
struct EdgeRec {
  uint8_t flags, pad;
  uint16_t cbp;
  uint8_t nnz[3][4];    // bottom row of each plane
  uint8_t mvd[2][4][2]; // bottom row
  int8_t ref[2][2];     // bottom two 8x8 of each list
  uint8_t direct8[2], pad2[2];
  uint8_t mnnz[52];
};
static_assert(sizeof(EdgeRec) == 92, "EdgeRec layout");
// The progressive walkers' ring holds EdgeRec's first ten dwords only (the parse's neighbour
// fields); the model bytes of each column (EdgeRec::mnnz, read by the NZ-tree keys of the parallel
// model) live in a row of their own, `mring`: in LDS after the ring, or -- when that is what lets
// four wide workgroups share a CU's LDS (4K: 240 columns x 92 B would leave room for three) -- in
// the workgroup's global scratch (kFlagMringGlobal).  Only the upper macroblock's bottom-row
// blocks and DC entries are ever read there (get_neighbor_sub_mb's upper neighbours: mnnz bytes
// 8-15, 24-31, 40-50, i.e. dwords 2, 3, 6, 7, 10, 11, 12 -- tests/test_oracle_geometry.py checks
// the table), so a column keeps those 7 dwords, dword d at ((d >> 2) << 1) | (d & 1): 28 B instead
// of 52 (round 6: the 4K stream's model-row write-backs were most of its HBM writes).
struct EdgeCore {
  uint8_t flags, pad;
  uint16_t cbp;
  uint8_t nnz[3][4];
  uint8_t mvd[2][4][2];
  int8_t ref[2][2];
  uint8_t direct8[2], pad2[2];
};
static_assert(sizeof(EdgeCore) == 40 && offsetof(EdgeRec, mnnz) == 40, "EdgeCore = EdgeRec's first ten dwords");
constexpr int kMringDwords = 7;      // per column: the read dwords of EdgeRec::mnnz
constexpr uint32_t kEdgeMringNz = 0x200u;   // EdgeCore dword 0: the column's model row was stored (global row)
constexpr uint32_t kMringUsed = 0x1CCCu;   // those dwords (2, 3, 6, 7, 10, 11, 12) of the 13
AVR_FI uint32_t mring_dword(uint32_t d) { return (d >> 2) << 1 | (d & 1); }
static_assert(sizeof(MbRec) == 180, "MbRec layout (dword map in Walker::edge_src)");

// LDS layout (per workgroup = one slice); the ring is sized by mb_width at launch.
// SIG + NZ estimators: an LDS hash table (4096 slots, 16 KB) in front of the dense per-model
// table in HBM (kEstTable u16 entries).  A slice touches ~3.5-5.5 K distinct SIG/NZ keys out of
// 294 K, so the first ones seen get an LDS slot for the rest of the model's life and only the
// keys that find their probe window full live in HBM (0.4 % of lookups at QP 22, none at QP 30,
// vs ~11 % misses for the direct-mapped write-back cache this replaces).  Keys never leave the
// table, so "not in the window and the window has a free slot" means "never seen": a new key
// starts at the default estimator without any HBM access.
//   key p = idx * kEstKeyMul mod 2^19 (a bijection), home slot p >> 7, tag p & 127; one probe is
//   one LDS read per lane over the 64 slots home .. home + 63; slot = (0x8000 | disp << 7 | tag)
//   << 16 | estimator, 0 = free.
// The HBM table is cleared lazily and sparsely: an entry stored there carries bit 15 (estimators
// use 15 bits: neg - 1 <= 0x60), so its first store is recognised and its index appended to the
// table's write log; the next model using the table zeroes the logged entries (the whole table
// only if the log overflowed) instead of clearing 588 KB per slice.
constexpr int kEtabBits = 12;
constexpr int kEtabSize = 1 << kEtabBits;
constexpr uint32_t kEstKeyMul = 0x4F1BBu;   // odd: multiplication mod 2^19 is a bijection
constexpr uint32_t kEstWritten = 0x8000u;
static_assert(kEstTable < (1 << 19), "estimator key space");

// Producer -> consumer ring of coding operations (see "Two waves per slice" below).
constexpr int kFifo = 512;

struct Shared {
  HotTables tab;          // copy of EngineTables::hot (per-bin lookups stay in LDS)
  uint32_t fifo[2][kFifo];   // [0] walker -> next wave, [1] modeler -> coder (compress only)
  uint32_t fifo_head[2];     // operations published by the ring's producer (monotonic)
  uint32_t fifo_tail[2];     // operations retired by the ring's consumer (monotonic)
  int32_t p_status, p_stop_ok, c_err;  // slice results of the two waves
  uint32_t elog_n;           // entries appended to the HBM table's write log by this model
  uint32_t prio;             // the slice's current wave priority (walker -> modeler / coder)
  uint32_t qnext;            // persistent launches: the queue entry this workgroup drew
#if defined(AVR_QUEUE_EAGER) && AVR_QUEUE_EAGER == 1
  uint32_t qcell;            // experiment build: the walker's board cell, set before the first draw
#endif
#ifdef AVR_WATCHDOG
  uint32_t wd_epoch[4];      // watchdog build: barrier checkpoints passed, per wave
#endif
  uint32_t c_len, c_last;
  uint32_t bill[6];          // the coder's h264_model billing by CodingType (kFlagBill launches)
  uint32_t blk[64];       // residual blocks of the current macroblock (packed, see push_block)
  uint8_t state[1024];
  uint16_t est[kEstDefault + 2];
  uint8_t in_stage[kStage];
  MbRec cur, left;
  union {
    uint32_t etab[kEtabSize + 64]; // compress/decompress: LDS hash table of the SIG + NZ estimators
                                   //   (home slots 0 .. kEtabSize - 1, probe windows do not wrap)
    uint16_t gen_p[1024];          // generator: P(bin = 1) in 1/65536 per context
  };
};

// ---------------------------------------------------------------------------------------
// Several waves per slice.  The hot path is a chain of serial recurrences that only meet in the
// bin value, so each runs on its own wave and they overlap on the SIMD instead of adding up:
//   compress:   walker (CABAC decode + slice_data parse + model keys)  --ring 0-->
//               modeler (estimator lookup/update, recode.cpp:816-820, 1030-1047)  --ring 1-->
//               coder (arithmetic_code<uint64_t,uint8_t> encoder, recode.cpp:1074, 1092-1094)
//   decompress: walker (recoded decode + model + parse: the parse needs each bin at once)
//               --ring 0--> coder (cabac::encoder, cabac_code.h:33-67)
// Consumers retire a ring in batches of up to 64 ops (one entry per lane, plus whatever table
// record that lane can gather), then run their serial chain over the batch from registers.
//
// ring 0, compress (model ops): bit 0 bin, bit 1 SIG/NZ estimator (else per-context), bit 2
//   significance-map threshold 0x50 (else 0x60), bits 3-21 estimator index.
// ring 1, compress (coder ops): bit 0 bin, bits 1-7 pos, bits 8-14 pos+neg of the estimator
//   before its update.
// ring 0, decompress: bit 0 bin, bits 1-2 kind (0 decision, 1 bypass, 2 terminate), bits 3-12
//   ctxIdx.
// Billing classes (h264_model::coding_type at the put, recode.cpp:615-661): compress coder ops
//   carry it in bits 15-16 (0 UNKNOWN, 1 SIGNIFICANCE_MAP, 2 SIGNIFICANCE_NZ), decompress walker
//   ops in bits 13-14 (0 UNKNOWN, 1 SIGNIFICANCE_MAP, 2 SIGNIFICANCE_EOB).
// OP_FINISH = arithmetic_code::encoder::finish (terminate = 1); OP_END closes a slice's stream.
enum { PIPC_UNKNOWN = 0, PIPC_UNREACHABLE, PIPC_SIG_MAP, PIPC_SIG_EOB, PIPC_SIG_NZ, PIPC_RESIDUALS };
constexpr uint32_t OPC_SHIFT_C = 15, OPC_SHIFT_D = 13;
__host__ __device__ inline int op_class_pip_c(uint32_t c) { return c == 1 ? PIPC_SIG_MAP : c == 2 ? PIPC_SIG_NZ : PIPC_UNKNOWN; }
__host__ __device__ inline int op_class_pip_d(uint32_t c) { return c == 1 ? PIPC_SIG_MAP : c == 2 ? PIPC_SIG_EOB : PIPC_UNKNOWN; }
constexpr uint32_t OP_FINISH = 1u << 30;
constexpr uint32_t OP_END = 1u << 31;
// compress rings of the long-slice split (SPL): with OP_FINISH at a cut -- the modeler starts a fresh
// model after it, the coder a fresh stream (bit 29: no model or coder op reaches it)
constexpr uint32_t OP_RESTART = 1u << 29;
enum { OPK_DECISION = 0, OPK_BYPASS = 1, OPK_TERMINATE = 2, OPK_MACRO = 3 };

constexpr uint32_t OPM_CACHE = 2, OPM_THR50 = 4;
AVR_FI uint32_t op_model(int bin, uint32_t flags, uint32_t idx) { return (uint32_t)bin | flags | idx << 3; }
AVR_FI uint32_t op_recode(int bin, uint32_t est) {
  const uint32_t pos = (est & 0xff) + 1, tot = pos + (est >> 8) + 1;
  return (uint32_t)bin | pos << 1 | tot << 8;
}
// Decompress macro ops (kind OPK_MACRO, progressive walkers): the coder expands them into the bins
// and contexts the walker would have sent one by one.  Bits 3-4 select the op:
//   0 map segment: ctxBlockCat bits 5-8, positions coded in this 16-position segment - 1 bits 9-12,
//     bit 13 = the map ended on a last_significant_coeff_flag of 1 at its highest significant
//     position (else: a full segment, or the map ran to max - 1), bits 14-29 the
//     significant_coeff_flag of each position.  The coder tracks the segment's first position; a
//     map's last segment resets it and the level counters (gt1 / eq1 of residual_block_cabac);
//   1 level: ctxBlockCat bits 5-8, sign bit 9, min(coeff_abs_level_minus1 + 1, 15) bits 10-13 (15:
//     the prefix only; the escape's suffix and the sign follow as bypass ops);
//   2 mvd component: vertical bit 5 (ctxIdxOffset 47, else 40), ctxIdxInc of the first bin bits 6-7,
//     sign bit 8, min(|mvd|, 9) bits 9-12 (9: the prefix only; the UEG3 suffix and the sign follow
//     as bypass ops).
AVR_FI uint32_t op_map(int cat, int npos, int ended, uint32_t mask) {
  return OPK_MACRO << 1 | (uint32_t)cat << 5 | (uint32_t)(npos - 1) << 9 | (uint32_t)ended << 13 | mask << 14;
}
AVR_FI uint32_t op_level(int cat, int absl, int sign) {
  return OPK_MACRO << 1 | 1u << 3 | (uint32_t)cat << 5 | (uint32_t)sign << 9 | (uint32_t)absl << 10;
}
AVR_FI uint32_t op_mvd(int comp, int inc, int amvd, int sign) {
  return OPK_MACRO << 1 | 2u << 3 | (uint32_t)comp << 5 | (uint32_t)inc << 6 | (uint32_t)sign << 8 | (uint32_t)amvd << 9;
}
// Watchdog build (-DAVR_WATCHDOG, diagnostics only): every wait of a slice workgroup is bounded in
// time, and the kernels check their own invariants.  A wait that lasts kWdTicks records where it
// was (site, workgroup, wave, the counters it waited on, the queue entry, HW_ID) in avr_prof and
// ends its wave, so a workgroup that would hang drains instead and the host reads the records
// (avr_debug_profile).  Layout of avr_prof: [0] records written, [1 + 3 i .. 3 + 3 i] record i
// (i < 16), [50] invariant violations, [51..53] the first one's record.  Sites: 1-4 ring waits
// (push, push_v, take, modeler -> coder room); 10 board cell out of range; 11 ring overfilled;
// 12 queue entries drawn out of order; 13 waves of a workgroup at different barriers.
enum { WD_PUSH = 1, WD_PUSHV = 2, WD_TAKE = 3, WD_ROOM1 = 4, WD_CELL = 10, WD_RING = 11, WD_QORDER = 12,
       WD_EPOCH = 13 };
#ifdef AVR_WATCHDOG
constexpr uint64_t kWdTicks = 300000000ull;   // s_memrealtime runs at 100 MHz: 3 s
AVR_FI void wd_put(unsigned long long* rec, uint32_t site, uint32_t a, uint32_t b, uint32_t k) {
  rec[0] = (unsigned long long)site << 48 | (unsigned long long)(threadIdx.x >> 6) << 40 | blockIdx.x;
  rec[1] = (unsigned long long)a << 32 | b;
  rec[2] = (unsigned long long)k << 32 | __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID
}
AVR_FI void wd_violation(uint32_t site, uint32_t a, uint32_t b, uint32_t k) {
  if (__lane_id() != 0) return;
  if (atomicAdd(&avr_prof[50], 1ull) == 0) wd_put(&avr_prof[51], site, a, b, k);
  __threadfence();
}
// One poll of a wait that started at *t0 (0: not yet): past kWdTicks, record and end the wave.
AVR_FI void wd_poll(uint64_t* t0, uint32_t site, uint32_t a, uint32_t b, uint32_t k) {
  const uint64_t t = __builtin_amdgcn_s_memrealtime();
  if (*t0 == 0) { *t0 = t; return; }
  if (t - *t0 < kWdTicks) return;
  if (__lane_id() == 0) {
    const unsigned long long i = atomicAdd(&avr_prof[0], 1ull);
    if (i < 16) wd_put(&avr_prof[1 + 3 * i], site, a, b, k);
    __threadfence();
  }
  __builtin_amdgcn_endpgm();
}
#define WD_T0 uint64_t wd_t0 = 0
#define WD_POLL(site, a, b, k) wd_poll(&wd_t0, site, a, b, k)
#define WD_CHECK(cond, site, a, b, k) do { if (!(cond)) wd_violation(site, a, b, k); } while (0)
#else
#define WD_T0
#define WD_POLL(site, a, b, k)
#define WD_CHECK(cond, site, a, b, k)
#endif

// Queue trace build (-DAVR_QTRACE, diagnostics only): each workgroup of a persistent launch writes
// its progress to host-mapped coherent memory (avr_debug_qtrace, compress kernel only), so the
// host can read where every workgroup and wave is while a launch has not returned.  Per
// workgroup 8 u32: [0..2] wave w's (slices drawn << 8 | phase), [3] the queue entry drawn, [4]
// the walker's macroblocks of the current slice.  Phases: 1 drawn, 2 estimator table reset,
// 3 slice state set up, 4 the wave's role done, 5 slice finished, 6 left the loop.
// -DAVR_QTRACE=1 records only the queue entries drawn and the exit (the least perturbation),
// -DAVR_QTRACE=2 every phase and the walker's macroblocks too.
#ifdef AVR_QTRACE
static __device__ uint32_t* avr_qtrace;
AVR_FI void qtrace(uint32_t slot, uint32_t v) {
  uint32_t* t = avr_qtrace;
  if (t && __lane_id() == 0) __hip_atomic_store(&t[blockIdx.x * 8 + slot], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define QTRACE1(slot, v) qtrace(slot, v)
#if AVR_QTRACE >= 2
#define QTRACE(slot, v) qtrace(slot, v)
#else
#define QTRACE(slot, v)
#endif
#else
#define QTRACE1(slot, v)
#define QTRACE(slot, v)
#endif

// Ring counters: plain LDS accesses.  LDS is one memory per CU and executes each wave's accesses
// in program order, so a counter store issued after the entry stores cannot be seen before them;
// the asm statements only keep the compiler from reordering (an acquire/release fence would
// also wait for, or write back, this wave's outstanding global stores).
// The casts to address space 3 matter: a volatile access through a generic pointer stays a
// flat access with cache-bypass bits and a vmcnt(0) wait (the address-space inference pass does
// not rewrite volatile accesses), which costs a global-memory round trip per counter update.
typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
AVR_FI uint32_t ld_volatile(const uint32_t* p) {
  const uint32_t v = *(lds_vu32*)p;
  asm volatile("" ::: "memory");
  return __builtin_amdgcn_readfirstlane(v);
}
AVR_FI void st_volatile(uint32_t* p, uint32_t v) {
  asm volatile("" ::: "memory");
  *(lds_vu32*)p = v;
}
// LDS hand-offs between the lanes of ONE wave need no barrier (a wave's LDS operations execute in
// order); only the compiler must not move memory operations across the hand-off.
AVR_FI void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Wave priority (s_setprio): the SQ issues from higher-priority waves first, then the oldest.
// A batch's time is its longest slice's, and the slices sharing a CU compete for the issue slots,
// so every wave of a slice runs at a priority that grows with the slice's remaining input
// (longest-remaining-first); the walker sets it once per macroblock and publishes it in LDS,
// the modeler and coder follow it once per ring batch.
AVR_FI void set_prio(uint32_t p) {
  switch (p) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}
// The slices that share a CU (up to 4 resident workgroups) rank themselves by remaining input on
// a per-CU board in global memory (one copy per kernel): each walker registers a cell of its CU
// (HW_ID / XCC_ID registers), posts its remaining bytes there once per macroblock and takes
// priority 3 - (number of CU neighbours with more input left), so the CU's issue slots go to the
// longest remaining slice first and the co-resident slices tend to finish together.  The board
// is shared by waves of one CU only, so workgroup-scope accesses (through the CU's own vector
// cache and the XCD's L2) suffice; agent scope would send every post to memory.  A stale read
// only delays a priority change.
constexpr int kCuIds = 2048;   // XCC (3 bits) x SE (3) x SH (1) x CU (4)
static __device__ uint32_t avr_cu_count[kCuIds];
static __device__ uint32_t avr_cu_rem[kCuIds * 4];
AVR_FI uint32_t cu_cell() {
  const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));  // HW_REG_XCC_ID
  const uint32_t cu = (((xcc & 7) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15);
  uint32_t slot = 0;
  if (__lane_id() == 0) slot = atomicAdd(&avr_cu_count[cu], 1u);
  return cu * 4 + (__builtin_amdgcn_readfirstlane(slot) & 3);
}
// Host side: zero this translation unit's board before a launch (stream-ordered).
static inline hipError_t reset_cu_board(hipStream_t stream) {
  void *cnt = nullptr, *rem = nullptr;
  hipError_t e = hipGetSymbolAddress(&cnt, HIP_SYMBOL(avr_cu_count));
  if (e == hipSuccess) e = hipGetSymbolAddress(&rem, HIP_SYMBOL(avr_cu_rem));
  if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(avr_cu_count), stream);
  if (e == hipSuccess) e = hipMemsetAsync(rem, 0, sizeof(avr_cu_rem), stream);
  return e;
}
constexpr uint32_t kNoCell = 0xffffffffu;   // Walker::prio_cell not assigned yet
AVR_FI void cu_post(uint32_t cell, uint32_t rem) {
  if (__lane_id() == 0) __hip_atomic_store(&avr_cu_rem[cell], rem, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
AVR_FI uint32_t cu_rank_prio(uint32_t cell, uint32_t rem) {
  const uint32_t lane = __lane_id(), me = cell & 3;
  uint32_t v = 0;
  if (lane < 4) v = __hip_atomic_load(&avr_cu_rem[(cell & ~3u) + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const uint64_t ahead = __ballot(lane < 4 && lane != me && (v > rem || (v == rem && lane < me)));
  return 3u - (uint32_t)__builtin_popcountll(ahead);
}

AVR_FI void follow_prio(Shared* sh, uint32_t* cur) {
  const uint32_t p = __builtin_amdgcn_readfirstlane(*(volatile __attribute__((address_space(3))) uint32_t*)&sh->prio);
  if (p != *cur) {
    *cur = p;
    set_prio(p);
  }
}

AVR_FI uint64_t readlane64(uint64_t v, uint32_t j) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, j);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), j);
  return (uint64_t)hi << 32 | lo;
}

// v_writelane_b32 (clang has no builtin for it; the LLVM intrinsic by its name)
extern "C" __device__ int avr_llvm_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// Producer end of ring r: entries go to LDS at once, the head counter every 32 entries (and on
// demand), the tail is re-read only when the ring looks full.
template <bool STAGED>
struct RingOutT {
  Shared* sh;
  int r;
  uint32_t head, room;
  AVR_FI void init(Shared* s, int ring) {
    sh = s;
    r = ring;
    head = 0;
    room = kFifo;
    stage_v = 0;
    stage_n = 0;
  }
  AVR_FI void publish() {
    flush();
    st_volatile(&sh->fifo_head[r], head);
  }
#ifdef AVR_PROFILE
  uint64_t wait_cycles = 0;
#endif
  // STAGED: single ops are staged in a VGPR (lane k = k-th op) and stored 64 at a time (fewer
  // instructions per op on the producer; measured 1 % faster for the decompress walker, 2 %
  // slower for the compress walker, whose consumer then waits in bursts)
  uint32_t stage_v, stage_n;
  AVR_FI void flush() {
    if (STAGED && stage_n) {
      const uint32_t k = stage_n;
      stage_n = 0;
      push_v_raw(stage_v, k);
    }
  }
  AVR_FI void push_v(uint32_t op_v, uint32_t n) {
    flush();
    push_v_raw(op_v, n);
  }
  // a staged run of ops on either ring kind (stage, then flush_stage before any other push)
  AVR_FI void stage(uint32_t op) {
    stage_v = __lane_id() == stage_n ? op : stage_v;
    if (++stage_n == 64) flush_stage();
  }
  AVR_FI void flush_stage() {
    if (stage_n) {
      const uint32_t k = stage_n;
      stage_n = 0;
      push_v_raw(stage_v, k);
    }
  }
  AVR_FI void push(uint32_t op) {
    if (STAGED) {
#ifdef AVR_WL_PUSH
      stage_v = (uint32_t)avr_llvm_writelane((int)op, (int)stage_n, (int)stage_v);
#else
      stage_v = __lane_id() == stage_n ? op : stage_v;
#endif
      if (++stage_n == 64) flush();
      return;
    }
    if (room == 0) {
      st_volatile(&sh->fifo_head[r], head);
#ifdef AVR_PROFILE
      const uint64_t tw = PROF_T();
#endif
      WD_T0;
      for (;;) {
        const uint32_t used = head - ld_volatile(&sh->fifo_tail[r]);
        WD_CHECK(used <= (uint32_t)kFifo, WD_RING, head, used, (uint32_t)r);
        if (used < (uint32_t)kFifo) { room = kFifo - used; break; }
        WD_POLL(WD_PUSH, head, used, sh->qnext);
        __builtin_amdgcn_s_sleep(1);
      }
#ifdef AVR_PROFILE
      wait_cycles += PROF_T() - tw;
#endif
    }
    sh->fifo[r][head & (kFifo - 1)] = op;
    head++;
    room--;
    if ((head & 31) == 0) st_volatile(&sh->fifo_head[r], head);
  }
  // n <= 64 ops at once, op k in lane k (one vector store)
  AVR_FI void push_v_raw(uint32_t op_v, uint32_t n) {
    if (room < n) {
      st_volatile(&sh->fifo_head[r], head);
#ifdef AVR_PROFILE
      const uint64_t tw = PROF_T();
#endif
      WD_T0;
      for (;;) {
        const uint32_t used = head - ld_volatile(&sh->fifo_tail[r]);
        WD_CHECK(used <= (uint32_t)kFifo, WD_RING, head, used, (uint32_t)r);
        if (used + n <= (uint32_t)kFifo) { room = kFifo - used; break; }
        WD_POLL(WD_PUSHV, head, used, sh->qnext);
        __builtin_amdgcn_s_sleep(1);
      }
#ifdef AVR_PROFILE
      wait_cycles += PROF_T() - tw;
#endif
    }
    if (__lane_id() < n) sh->fifo[r][(head + __lane_id()) & (kFifo - 1)] = op_v;
    const uint32_t h0 = head;
    head += n;
    room -= n;
    if ((h0 ^ head) & ~31u) st_volatile(&sh->fifo_head[r], head);
  }
};
// Consumer end: wait for a batch, load it one entry per lane.  Returns the batch size.
AVR_FI uint32_t ring_take(Shared* sh, int r, uint32_t tail, uint32_t* op_v, uint64_t* waited) {
  uint32_t head;
#ifdef AVR_PROFILE
  const uint64_t tw = PROF_T();
#endif
  WD_T0;
  for (;;) {
    head = ld_volatile(&sh->fifo_head[r]);
    if (head != tail) break;
    WD_POLL(WD_TAKE, head, tail, sh->qnext);
    __builtin_amdgcn_s_sleep(1);
  }
  WD_CHECK(head - tail <= (uint32_t)kFifo, WD_RING, head, tail, (uint32_t)r | 0x100u);
#ifdef AVR_PROFILE
  *waited += PROF_T() - tw;
#endif
  const uint32_t n = min(head - tail, 64u);
  const uint32_t lane = __lane_id();
  *op_v = lane < n ? sh->fifo[r][(tail + lane) & (kFifo - 1)] : 0u;
  return n;
}
AVR_FI void ring_retire(Shared* sh, int r, uint32_t tail) { st_volatile(&sh->fifo_tail[r], tail); }

// SIG / NZ estimators: probe the LDS hash table (see kEtabBits).  Returns the estimator and in
// *slot where est_store writes it back (0: the HBM table).  Called by a whole wave.
AVR_FI uint32_t est_load(Shared* sh, const uint16_t* est_g, uint32_t idx, uint32_t* slot, bool claim = false) {
  const uint32_t p = (idx * kEstKeyMul) & ((1u << 19) - 1);
  const uint32_t home = p >> 7, tag = p & 127;
  const uint32_t lane = __lane_id();
  const uint32_t ent = sh->etab[home + lane];
  const uint64_t hit = __ballot((ent >> 16) == (0x8000u | lane << 7 | tag));
#ifdef AVR_PROFILE_EST   // with AVR_PROFILE: estimator lookups that go to HBM (scripts/diag_est.py)
  if (lane == 0) atomicAdd(&avr_prof[22], 1ull);
  if (lane == 0 && !hit && !__ballot(ent == 0)) atomicAdd(&avr_prof[23], 1ull);
#endif
  if (hit) {
    // the entry's upper half is the slot's tag word already
    const uint32_t j = (uint32_t)__builtin_ctzll(hit);
    const uint32_t ej = __builtin_amdgcn_readlane(ent, j);
    *slot = (ej & 0xffff0000u) | (home + j);
    return ej & 0xffff;
  }
  const uint64_t free_v = __ballot(ent == 0);
  if (free_v) {
    const uint32_t j = (uint32_t)__builtin_ctzll(free_v);
    *slot = (0x8000u | j << 7 | tag) << 16 | (home + j);
    // a caller that defers its store claims the slot now (a later key of the window must not take it)
    if (claim && lane == j) sh->etab[home + j] = *slot & 0xffff0000u;
    return 0;
  }
  // HBM: slot 1 marks the entry's first store (to be logged), 0 a stored one
  const uint32_t raw = __builtin_amdgcn_readfirstlane(est_g[idx]);
  *slot = __builtin_amdgcn_readfirstlane((raw >> 15 & 1u) ^ 1u);   // a scalar, like the LDS slots
  return raw & (kEstWritten - 1);
}
AVR_FI void est_store(Shared* sh, uint16_t* est_g, uint32_t idx, uint32_t slot, uint32_t e) {
  if (slot >> 31) {
    sh->etab[slot & 0xffff] = (slot & 0xffff0000u) | e;
  } else if (__lane_id() == 0) {
    est_g[idx] = (uint16_t)(e | kEstWritten);
    if (slot) {
      const uint32_t n = sh->elog_n;
      sh->elog_n = n + 1;
      uint32_t* lg = (uint32_t*)(est_g + kEstLog);
      if (n < (uint32_t)kEstLogCap) lg[n] = idx;
      *(uint32_t*)(est_g + kEstLogN) = n < (uint32_t)kEstLogCap ? n + 1 : kEstLogOverflow;
    }
  }
}
// Lane-parallel lookup of each lane's key in the first four slots of its window: true (with the
// estimator and its slot) when found there.  A key found stays where it is, so a hit is final;
// a miss (new key, deeper or HBM-resident one) goes through est_load.
AVR_FI bool est_probe4(const Shared* sh, uint32_t idx, uint32_t* e, uint32_t* slot) {
  const uint32_t p = (idx * kEstKeyMul) & ((1u << 19) - 1);
  const uint32_t home = p >> 7, t0 = 0x8000u | (p & 127);
  const uint32_t s0 = sh->etab[home], s1 = sh->etab[home + 1], s2 = sh->etab[home + 2], s3 = sh->etab[home + 3];
  // branch-free (selects): callers run it on every lane
  const bool h0 = (s0 >> 16) == t0, h1 = (s1 >> 16) == (t0 | 1u << 7);
  const bool h2 = (s2 >> 16) == (t0 | 2u << 7), h3 = (s3 >> 16) == (t0 | 3u << 7);
  const uint32_t d = h0 ? 0u : h1 ? 1u : h2 ? 2u : 3u;
  *e = (h0 ? s0 : h1 ? s1 : h2 ? s2 : s3) & 0xffff;
  *slot = (t0 | d << 7) << 16 | (home + d);
  return h0 | h1 | h2 | h3;
}

// A fresh model on a table the last model may have written: zero the logged entries (or the
// whole table), reset the log.  Called by the whole workgroup; ends with a barrier.
AVR_FI void est_table_reset(uint16_t* est_g, Shared* sh) {
  const uint32_t n = *(volatile uint32_t*)(est_g + kEstLogN);
  __syncthreads();   // every thread has read the count before it is reset
  if (n == kEstLogOverflow) {
    uint4* e4 = (uint4*)est_g;
    for (int i = threadIdx.x; i < kEstTable / 8; i += blockDim.x) e4[i] = make_uint4(0, 0, 0, 0);
  } else if (n) {
    const uint32_t* lg = (const uint32_t*)(est_g + kEstLog);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) est_g[lg[i]] = 0;
  }
  if (threadIdx.x == 0) {
    *(uint32_t*)(est_g + kEstLogN) = 0;
    sh->elog_n = 0;
  }
  __syncthreads();
}

// FLD: field-coded slices (PAFF, MBAFF) -- a second instantiation (kernels of their own, launched
// only when a batch may hold such slices: kFlagFields), so that the progressive walker carries no
// field tests in its per-bin and per-macroblock code

// SPL: the long-slice split's kernels (slices_split_kernel): a piece may start from a seam record
// and stop after n macroblocks, and compress takes the cut records (avr_kernels.h SeamRec)
template <int MODE, bool RM, bool FLD = false, bool P32 = false, bool SPL = false>
struct Walker {
  static constexpr bool DEC = MODE == MODE_COMPRESS || MODE == MODE_TRACE;  // CABAC decoding side
  const HotTables* T;     // LDS copy
  const EngineTables* G;  // global (init-only tables)
  const avr_slice_desc* d;
  Shared* sh;
  // the upper row's edge records: full EdgeRecs for the field walkers (their MBAFF views and pair
  // records), EdgeCore plus the separate model row (mring) for the progressive ones
  typedef typename std::conditional<FLD, EdgeRec, EdgeCore>::type ERec;
  ERec* ring;
  uint32_t* mring;        // progressive, parallel model: 13 dwords per column (LDS or global)
  bool mring_global;
  uint16_t* est_g;        // SIG + NZ estimators (global)
  uint8_t* frames;        // RM: 2 frames of W*H*52 model bytes
  int64_t cur_off, prev_off;   // RM: byte offsets of the current / previous frame's model bytes (prev < 0: zeros)
  // RM scan (rscan_kernel): model ops go to global memory instead of the modeler's ring
  bool gmode;
  uint32_t* gsink;        // nullptr: count only
  uint32_t gcount;
  // engines
  InStream in;
  OutStream out;
  CabacDecoder cd;
  CabacEncoder ce;
  RecodedEncoder re;
  // the model's decisions go through the reference's arithmetic_code<uint64_t, uint8_t> (both
  // models' default containers); P32 = the parallel model's optional 32-bit coder (avr_engine.h,
  // PDecoder; container tag avrecode-amd:P32)
  typename std::conditional<P32, PDecoder, RecodedDecoder>::type rd;
  uint64_t rng;
  // slice state
  int W, H, mb_x, mb_y, slice_type, is_b, cat_, t8mode;
  // field coding: fld = the current macroblocks are field coded (their significance contexts use
  // the field tables); my = the model's row of the current macroblock, FFmpeg's sl->mb_y (frame
  // rows: a field picture's row r is frame row 2 r + bottom), stepped by ystep per parse row
  int fld, fld_pic, my, ystep;
  // RM parallel compress (rscan_kernel): this slice belongs to the first-coded field of its frame,
  // so the other field's rows -- already in the frame buffer, which that kernel fills before it
  // reads -- must read as the zeros the sequential model still sees there
  int top_pending;
  AVR_FI int mrow() const { return FLD ? my : mb_y; }   // the model's row (progressive: the parse row)
  // MBAFF frame (AVR_STRUCT_MBAFF): macroblock pairs; pst = the pair's state (PST_*); ring_cols =
  // EdgeRec slots the launch gave the LDS ring (an MBAFF slice needs 3 W + 7, see pair_edge)
  int mbaff;
  uint32_t pst, ring_cols;
  int left_ok, top_ok, last_dqp_nz;
  // flags (bits 0-6, F_*) and coded_block_pattern (bits 16-31) of the current macroblock and of
  // its left / upper neighbours, in one scalar register each for the whole macroblock (the
  // neighbours' read once at its start): context selection reads no LDS for them.  Bit 7 of cf:
  // the current macroblock has an 8x8 residual block (finished_queueing's is_8x8).
  uint32_t cf, lf, tf;
  static constexpr uint32_t CF_8X8 = 0x80;
  uint32_t edge_src;      // lane j < 23: the MbRec dword that becomes EdgeRec dword j (set per slice)
  int err, finished;
  uint32_t bins;
  int target_mbs, mbs_done, last_mb;
  int nref0, nref1, d8x8inf, x264_build, first_mb;
  // the long-slice split (SPL): the piece's start record (nullptr: the slice's own start) and
  // macroblock count (0: to end_of_slice); compress: where the cut records go (snap, snap_cap of
  // them, rec_stride apart; snap_n made, count to *snap_count), a candidate every split_bits decoded
  // bits (snap_last: the previous one; snap_q: the previous cut's first byte)
  const SeamRec* seam;
  uint8_t* snap;
  uint32_t* snap_count;
  uint32_t snap_cap, snap_n, snap_last, snap_q, split_bits, rec_stride, piece_mbs;
  int cut;                // the walk stopped at the piece's end (not at end_of_slice)
  // The re-encoder's state where the decoder stands (the oracle's avr_seam_encoder): L = V - offset,
  // V the payload's first bitpos bits, as bytes Z = F[sb..e) - (offset << r) (r = 8 e - bitpos pad
  // bits); q = the last byte below m = (bitpos - 10) / 8 that is not 0xFF, the 0xFF bytes after it
  // outstanding, the bits of L from byte m on in low.  A dozen scalar byte loads, at a cut candidate.
  AVR_FI bool seam_place(uint32_t bitpos, uint32_t offset, uint32_t* ce) const {
    if (bitpos < 26) return false;
    const uint32_t m = (bitpos - 10) >> 3, sb = m > 12 ? m - 12 : 0, e = (bitpos + 7) >> 3, r = 8 * e - bitpos;
    const uint32_t sub = offset << r;
    uint32_t borrow = 0, low = 0, q = ~0u, cache = 0;
    for (uint32_t j = e; j-- > sb;) {
      const uint32_t t = e - 1 - j;
      const uint32_t sbyte = t < 4 ? (sub >> (8 * t)) & 0xff : 0u;
      const uint32_t f = j < in.limit ? (uint32_t)in.g[j] : 0u;
      const uint32_t v = f - sbyte - borrow;
      borrow = v >> 31;
      const uint32_t z = v & 0xff;
      if (j >= m) low |= z << (8 * t);
      else if (q == ~0u && z != 0xff) q = j, cache = z;
    }
    if (borrow || q == ~0u) return false;
    const uint32_t lowbits = bitpos - 8 * m;
    ce[0] = (low >> r) & ((1u << lowbits) - 1);    // ce_low
    ce[1] = cd.range;                               // ce_range
    ce[2] = m - 1 - q;                              // ce_outstanding
    ce[3] = cache;                                  // ce_cache
    ce[4] = lowbits - 18;                           // ce_queue
    ce[5] = q;
    return true;
  }
  // A cut candidate at this row start (compress, SPL; the rule of oracle/oracle_recode.c
  // c_row_start): at least split_bits decoded bits since the last candidate, half of that still ahead
  // in the payload.  Where the re-encoder's state can be placed (and moves forward), the slice is cut
  // here: the record (decoder, re-encoder, contexts with the cached lanes written back, last_dqp_nz,
  // the ring's upper-row edges), then the piece's re-coded stream ends (encoder::finish) and the
  // modeler starts a fresh model (OP_RESTART, taken alone: the walker waits until the modeler has
  // retired it), and the model row reads zero for the new piece's first row.
  AVR_FI void seam_cut(int addr) {
    const uint32_t pos = cd_bitpos(cd);
    if (pos - snap_last < split_bits || (uint64_t)pos + split_bits / 2 > 8ull * d->payload_size) return;
    snap_last = pos;
    if (snap_n >= snap_cap) return;
    uint32_t ce[6];
    if (!seam_place(pos, cd.low >> cd.k, ce) || (snap_n && ce[5] <= snap_q)) return;
    snap_q = ce[5];
    rc_writeback();
    mc_store();
    uint32_t* r32 = (uint32_t*)(snap + (size_t)snap_n * rec_stride);
    const uint32_t lane = __lane_id();
    if (lane < 16) {
      const uint32_t v = lane == 0 ? (uint32_t)addr : lane == 1 ? (uint32_t)last_dqp_nz : lane == 2 ? cd.low
                       : lane == 3 ? cd.range : lane == 4 ? (uint32_t)cd.k : lane == 5 ? cd.next
                       : lane == 6 ? ce[0] : lane == 7 ? ce[1] : lane == 8 ? ce[2] : lane == 9 ? ce[3]
                       : lane == 10 ? ce[4] : lane == 11 ? ce[5] : 0u;
      r32[lane] = v;
    }
    const uint32_t* st = (const uint32_t*)sh->state;
    for (uint32_t i = lane; i < 256; i += 64) r32[16 + i] = st[i];
    const uint32_t* e = (const uint32_t*)ring;
    for (uint32_t i = lane; i < (uint32_t)W * 10; i += 64) r32[16 + 256 + i] = i % 10 ? e[i] : e[i] & ~kEdgeMringNz;
    snap_n++;
    if constexpr (MODE == MODE_COMPRESS) {
      push(OP_FINISH | OP_RESTART);
      publish();
      WD_T0;
      while (ld_volatile(&sh->fifo_tail[0]) != ring0.head) {
        WD_POLL(WD_TAKE, ring0.head, 0, sh->qnext);
        __builtin_amdgcn_s_sleep(1);
      }
      for (uint32_t i = lane; i < (uint32_t)W * kMringDwords; i += 64) mring[i] = 0;
      wave_sync();
    }
  }
  uint32_t prio_cell, prio_cur;   // this slice's cell on the CU board, current priority
  AVR_FI void update_prio() {
    const uint32_t pos = MODE == MODE_DECOMPRESS ? rd.next : cd.next;
    const uint32_t size = d->payload_size;
    const uint32_t rem = pos < size ? size - pos : 0u;
    cu_post(prio_cell, rem);
    const uint32_t p = cu_rank_prio(prio_cell, rem);
    if (p != prio_cur) {
      prio_cur = p;
      set_prio(p);
      if (__lane_id() == 0) *(volatile __attribute__((address_space(3))) uint32_t*)&sh->prio = p;
    }
  }
  RingOutT<MODE == MODE_DECOMPRESS> ring0;   // walker -> modeler (compress) / coder (decompress)
  // compress: a residual block's level ops are staged in a VGPR and stored together after the
  // block (measured: batch compress -0.4 %, profiles/r04h_lstage_ab.log)
  static constexpr bool kStageLevels = true;
  VTab vt;                // CABAC state records (compress / generate: the walker's engine)

  // ------------------------------------------------------------------ residual context registers
  // The residual contexts of one ctxBlockCat (significant_coeff_flag lanes 0-15,
  // last_significant lanes 16-31, coeff_abs_level_minus1 lanes 32-41, coded_block_flag lanes
  // 42-45) live in one VGPR, lane j
  // holding the walker's per-context value for ctx rc_addr(j): the CABAC state byte (compress,
  // generate) or the estimator (decompress).  A residual bin then costs a v_readlane /
  // v_writelane instead of an LDS round trip.  Switching category writes the lanes back.
  uint32_t rc_v;
  int rc_cat;
  uint32_t sig8_v, last8_v;   // 8x8 significant / last ctxIdxInc tables, lane = scan position
  uint32_t byp_e;         // decompress: the estimator of &bypass_context (recode.cpp:1049), Shared::est[1024] while walking
  // lane L of v := x (L and x wave-uniform).  Decompress: one v_writelane, no lane-mask compare
  // to keep live (R-mode decompress -1 %); compress keeps the select (v_writelane there: +2 %).
  AVR_FI static uint32_t wlane(uint32_t v, uint32_t L, uint32_t x) {
    return (uint32_t)avr_llvm_writelane((int)x, (int)L, (int)v);
  }
  AVR_FI int rc_addr(int cat, uint32_t j) const {
    // Only the contexts the category can use: a lane past them would alias another syntax
    // element's context and write a stale copy back over it at rc_writeback -- within the
    // category (8x8 sig ctxIdxInc 0-14 / last 0-8 then the next element) or, with the field
    // offsets, transform_size_8x8_flag (ctxIdx 399-400 = chroma AC's last lanes 30-31), which
    // bin() updates in LDS while the category stays loaded across macroblocks.
    const bool c8 = cat == 5 || cat == 9 || cat == 13;
    if (!FLD) {   // frame offsets: only the 8x8 categories' lanes alias (within the category)
      if (c8 && (j == 15 || (j >= 25 && j < 32))) return -1;
      return j < 16 ? T->sig_base[cat] + (int)j : j < 32 ? T->last_base[cat] + (int)j - 16
           : j < 42 ? T->abs_base[cat] + (int)j - 32 : j < 46 ? T->cbf_base[cat] + (int)j - 42 : -1;
    }
    const int ns = c8 ? 15 : cat == 3 ? 3 : (cat == 1 || cat == 4 || cat == 7 || cat == 11) ? 14 : 15;
    const int nl = c8 ? 9 : ns;
    if (j < 16) return (int)j < ns ? T->sig_base[cat] + (int)j : -1;
    if (j < 32) return (int)j - 16 < nl ? T->last_base[cat] + (int)j - 16 : -1;
    return j < 42 ? T->abs_base[cat] + (int)j - 32 : j < 46 ? T->cbf_base[cat] + (int)j - 42 : -1;
  }
  AVR_FI void rc_writeback() {
    if (rc_cat < 0) return;
    const int a = rc_addr(rc_cat, __lane_id());
    if (a >= 0) {
      if (MODE == MODE_DECOMPRESS) sh->est[a] = (uint16_t)rc_v;
      else sh->state[a] = (uint8_t)rc_v;
    }
    wave_sync();
    rc_cat = -1;
  }
  AVR_FI void rc_select(int cat) {
    if (cat == rc_cat) return;
    rc_writeback();
    const int a = rc_addr(cat, __lane_id());
    rc_v = a < 0 ? 0u : MODE == MODE_DECOMPRESS ? (uint32_t)sh->est[a] : (uint32_t)sh->state[a];
    rc_cat = cat;
  }
  // compress: one CABAC decision on cached context lane L (no op pushed)
  AVR_FI int rdecide(uint32_t L) {
    bins++;
    const uint32_t s = __builtin_amdgcn_readlane(rc_v, L);
    uint32_t ns;
    const int b = cd_decide(cd, in, s, crec(s), &ns);
    rc_v = wlane(rc_v, L, ns);
    if (MODE == MODE_TRACE) trace(b, OPK_DECISION, s);
    return b;
  }
  AVR_FI void trace(int b, uint32_t kind, uint32_t s) {
    out_byte(out, (uint32_t)b | kind << 1);
    out_byte(out, s);
  }
  AVR_FI void trace_map_begin(int cat, int n, int max, int is_dc, int c422) {
    const uint32_t y = (uint32_t)mrow();
    out_byte(out, 3u << 1);
    out_byte(out, TRACE_EV_MAP_BEGIN);
    out_byte(out, (uint32_t)mb_x & 0xff);
    out_byte(out, (uint32_t)mb_x >> 8);
    out_byte(out, y & 0xff);
    out_byte(out, y >> 8);
    out_byte(out, (uint32_t)cat);
    out_byte(out, (uint32_t)n);
    out_byte(out, (uint32_t)max);
    out_byte(out, (uint32_t)is_dc | (uint32_t)c422 << 1);
  }
  AVR_FI void trace_map_end() {
    out_byte(out, 3u << 1);
    out_byte(out, TRACE_EV_MAP_END);
  }
  // a residual bin through the model on cached lane L; ctx = rc_addr(rc_cat, L)
  AVR_FI int rbin(uint32_t L, int ctx) {
    if (DEC) {
      const int b = rdecide(L);
      if (MODE == MODE_COMPRESS) push(op_model(b, 0, ctx));
      return b;
    } else if (MODE == MODE_DECOMPRESS) {
      bins++;
      const uint32_t e = __builtin_amdgcn_readlane(rc_v, L);
      const int b = rdec(e);
      rc_v = wlane(rc_v, L, est_update(e, b, 0x60));
      push((uint32_t)b | OPK_DECISION << 1 | (uint32_t)ctx << 3);
      return b;
    } else {
      bins++;
      const uint32_t s = __builtin_amdgcn_readlane(rc_v, L);
      const int b = rnd() < sh->gen_p[ctx];
      uint32_t ns;
      ce_encode(ce, out, b, s, vtab_rec(vt, s), &ns);
      rc_v = wlane(rc_v, L, ns);
      return b;
    }
  }

  // decompress: a residual bin / a bypass bin without its coder op (the macro ops below carry it)
  AVR_FI int rdec_lane(uint32_t L) {
    bins++;
    const uint32_t e = __builtin_amdgcn_readlane(rc_v, L);
    const int b = rdec(e);
    rc_v = wlane(rc_v, L, est_update(e, b, 0x60));
    return b;
  }
  AVR_FI int rdec_mc(int ctx) {   // a macroblock-layer context bin (kMcBase .. + 63)
    bins++;
    const uint32_t L = (uint32_t)(ctx - kMcBase);
    const uint32_t e = __builtin_amdgcn_readlane(mc_v, L);
    const int b = rdec(e);
    mc_v = wlane(mc_v, L, est_update(e, b, 0x60));
    return b;
  }
  AVR_FI int rdec_bypass() {
    bins++;
    const uint32_t e = byp_e;
    const int b = rdec(e);
    byp_e = est_update(e, b, 0x60);
    return b;
  }

  // recoded-decoder probability (recode.cpp:816-820).  The reciprocal comes by a scalar load
  // from the constant table (s_load_dwordx4 into SGPRs, scalar-cache hit): fewer instructions on
  // the walker than three v_readlane pairs and selects from a VGPR table (measured 10 % slower).
  typedef const __attribute__((address_space(4))) uint64_t cu64;
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  AVR_FI auto p1(uint32_t e) const {
    const uint32_t pos = (e & 0xff) + 1, tot = (e & 0xff) + (e >> 8) + 2;   // the sum est_update tests
    if constexpr (!P32) {
      cu64* dv = (cu64*)&G->hot.div[tot][0];
      return (__umul64hi(rd.range, dv[0]) >> (uint32_t)dv[1]) * pos;
    } else {
      return __umulhi(rd.range, ((cu32*)G->hot.rcp32)[tot]) * pos;   // the P-format rule
    }
  }
  // One decision of the model's coder with estimator e (recode.cpp:1435-1449).
  AVR_FI int rdec(uint32_t e) { return rd_get(rd, in, p1(e)); }
  // CABAC state record of state byte s: VGPR table (two v_readlane) or, with AVR_CABAC_SMEM, a
  // scalar load
  AVR_FI CabacRec crec(uint32_t s) const {
#ifdef AVR_CABAC_SMEM
    return rec_of(((cu64*)G->hot.cabac)[s]);
#else
    return vtab_rec(vt, s);
#endif
  }
  AVR_FI void publish() {
    if (RM && gmode) return;
    ring0.publish();
  }
  AVR_FI void push(uint32_t op) {
    if (RM && gmode) {
      if (gsink && __lane_id() == 0) gsink[gcount] = op;
      gcount++;
      return;
    }
    ring0.push(op);
  }
  AVR_FI void push_v(uint32_t op_v, uint32_t n) {
    if (RM && gmode) {
      if (gsink && __lane_id() < n) gsink[gcount + __lane_id()] = op_v;
      gcount += n;
      return;
    }
    ring0.push_v(op_v, n);
  }
#ifdef AVR_PROFILE
  uint64_t prof[8], sprof[8];
  uint32_t profb[8], sprofb[8];
#endif

  // Frame or field significance contexts for the macroblocks that follow: the walker's LDS copy of
  // the ctxIdx bases (rc_addr, sig_map) and the 8x8 ctxIdxInc map in sig8_v (for decompress also
  // the frame map in bits 8-15: the model keys 8x8 positions by the frame map, recode.cpp:703-704,
  // as does T->sig8x8, which is never patched).  Only this wave reads the patched entries.
  AVR_FI void set_fld(int f) {
    if (f == fld) return;
    rc_writeback();
    fld = f;
    const uint32_t L = __lane_id();
    HotTables* t = &sh->tab;
    if (L < 16) t->sig_base[L] = f ? G->sig_base_fld[L] : G->hot.sig_base[L];
    else if (L < 32) t->last_base[L - 16] = f ? G->last_base_fld[L - 16] : G->hot.last_base[L - 16];
    const uint32_t fr = T->sig8x8[L];
    const uint32_t cm = f ? (uint32_t)G->sig8x8_fld[L] : fr;
    sig8_v = (MODE == MODE_DECOMPRESS && FLD) ? (cm | fr << 8) : cm;
    wave_sync();
  }

  // ------------------------------------------------------------------ bins through the model
  // Macroblock-layer contexts kMcBase .. kMcBase + 63 (sub_mb_type, B mb_type, mvd, ref_idx,
  // mb_qp_delta, intra_chroma_pred_mode, prev/rem_intra_pred_mode, coded_block_pattern) stay in
  // one VGPR for the whole slice, lane ctx - kMcBase, like the residual contexts.
  static constexpr int kMcBase = 21;
  uint32_t mc_v;
  AVR_FI void mc_load() {
    const int a = kMcBase + (int)__lane_id();
    mc_v = MODE == MODE_DECOMPRESS ? (uint32_t)sh->est[a] : (uint32_t)sh->state[a];
  }
  AVR_FI void mc_store() {
    const int a = kMcBase + (int)__lane_id();
    if (MODE == MODE_DECOMPRESS) sh->est[a] = (uint16_t)mc_v;
    else sh->state[a] = (uint8_t)mc_v;
    wave_sync();
  }
  AVR_FI int mbin(int se, int k, int ctx) {
    bins++;
    const uint32_t L = (uint32_t)(ctx - kMcBase);
    if (DEC) {
      const uint32_t s = __builtin_amdgcn_readlane(mc_v, L);
      uint32_t ns;
      const int b = cd_decide(cd, in, s, crec(s), &ns);
      mc_v = wlane(mc_v, L, ns);
      if (MODE == MODE_TRACE) trace(b, OPK_DECISION, s);
      else push(op_model(b, 0, ctx));
      return b;
    } else if (MODE == MODE_DECOMPRESS) {
      const uint32_t e = __builtin_amdgcn_readlane(mc_v, L);
      const int b = rdec(e);
      mc_v = wlane(mc_v, L, est_update(e, b, 0x60));
      push((uint32_t)b | OPK_DECISION << 1 | (uint32_t)ctx << 3);
      return b;
    } else {
      const uint32_t s = __builtin_amdgcn_readlane(mc_v, L);
      const int b = gen_bin(se, k, ctx);
      uint32_t ns;
      ce_encode(ce, out, b, s, vtab_rec(vt, s), &ns);
      mc_v = wlane(mc_v, L, ns);
      return b;
    }
  }
  AVR_FI int bin(int se, int k, int ctx) {
    if ((uint32_t)(ctx - kMcBase) < 64u) return mbin(se, k, ctx);
    bins++;
    if (DEC) {
      const uint32_t s = sh->state[ctx];
      uint32_t ns;
      const int b = cd_decide(cd, in, s, crec(s), &ns);
      sh->state[ctx] = (uint8_t)ns;
      if (MODE == MODE_TRACE) trace(b, OPK_DECISION, s);
      else push(op_model(b, 0, ctx));
      return b;
    } else if (MODE == MODE_DECOMPRESS) {
      const uint32_t e = sh->est[ctx];
      const int b = rdec(e);
      sh->est[ctx] = (uint16_t)est_update(e, b, 0x60);
      push((uint32_t)b | OPK_DECISION << 1 | (uint32_t)ctx << 3);
      return b;
    } else {
      int b = gen_bin(se, k, ctx);
      ce_decision(ce, out, b, &sh->state[ctx], T);
      return b;
    }
  }
  AVR_FI int bypass(int se, int k) {
    bins++;
    if (DEC) {
      const int b = cd_bypass(cd, in);
      if (MODE == MODE_TRACE) trace(b, OPK_BYPASS, 0);
      else push(op_model(b, 0, 1024));
      return b;
    } else if (MODE == MODE_DECOMPRESS) {
      const uint32_t e = byp_e;   // the bypass estimator lives in a scalar register
      const int b = rdec(e);
      byp_e = est_update(e, b, 0x60);
      push((uint32_t)b | OPK_BYPASS << 1);
      return b;
    } else {
      int b = gen_bypass(se, k);
      ce_bypass(ce, out, b);
      return b;
    }
  }
  AVR_FI int terminate(int se) {
    bins++;
    int b;
    if (DEC) {
      b = cd_terminate(cd, in);
      if (MODE == MODE_TRACE) {
        trace(b, OPK_TERMINATE, 0);
      } else {
        push(op_model(b, 0, 1025));
        if (b) push(OP_FINISH);
      }
    } else if (MODE == MODE_DECOMPRESS) {
      const uint32_t e = sh->est[1025];
      b = rdec(e);
      sh->est[1025] = (uint16_t)est_update(e, b, 0x60);
      push((uint32_t)b | OPK_TERMINATE << 1);
    } else {
      b = se == SE_EOS ? (mbs_done >= target_mbs || last_mb) : 0;
      ce_terminate(ce, out, b);
    }
    if (b && se == SE_EOS) finished = 1;
    return b;
  }

  // ------------------------------------------------------------------ synthetic bin policy
  AVR_FI uint32_t rnd() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 16) & 0xffff;
  }
  AVR_FI int gen_bin(int se, int k, int ctx) {
    if (se == SE_REF && k >= avr_limit) return 0;
    if (se == SE_QPDELTA && k >= 2) return 0;
    return rnd() < sh->gen_p[ctx];
  }
  AVR_FI int gen_bypass(int se, int k) {
    if ((se == SE_MVD_SUFFIX || se == SE_LEVEL_SUFFIX) && k >= 5 && k < 100) return 0;
    return rnd() & 1;
  }
  int avr_limit;

  // ------------------------------------------------------------------ neighbours (parser)
  AVR_FI const ERec& top() const { return ring[mb_x]; }
  AVR_FI uint16_t nb_cbp_left() const {
    return left_ok ? (lf >> 16) : ((cf & F_INTRA) ? 0x7CF : 0x00F);
  }
  AVR_FI uint16_t nb_cbp_top() const {
    return top_ok ? (tf >> 16) : ((cf & F_INTRA) ? 0x7CF : 0x00F);
  }
  // FFmpeg 4:4:4 8x8 coded_block_flag quirk for x264 < r151 (see oracle_walker.c)
  AVR_FI int nnz_override(uint32_t nbflags, int* v) const {
    if (cat_ != 3 || !(cf & F_T8) || (nbflags & F_T8)) return 0;
    *v = (uint32_t)x264_build < 151u ? ((cf & F_INTRA) ? 64 : 0) : 0;
    return 1;
  }
  AVR_FI int nnz_left(int p, int pw, int x4, int y4) const {
    if (x4 > 0) return sh->cur.nnz[p][y4 * 4 + x4 - 1];
    if (!left_ok) return (cf & F_INTRA) ? 64 : 0;
    int v;
    // MBAFF: rows of one left macroblock come from both macroblocks of the left pair; the view's
    // flags byte holds each row's source 8x8-transform flag
    if (nnz_override((FLD && mbaff) ? (((uint32_t)sh->left.flags >> y4) & 1u) * (uint32_t)F_T8 : lf, &v)) return v;
    return sh->left.nnz[p][y4 * 4 + pw - 1];
  }
  AVR_FI int nnz_top(int p, int x4, int y4) const {
    if (y4 > 0) return sh->cur.nnz[p][(y4 - 1) * 4 + x4];
    if (!top_ok) return (cf & F_INTRA) ? 64 : 0;
    int v;
    if (nnz_override(tf, &v)) return v;
    return ring[mb_x].nnz[p][x4];
  }

  // ------------------------------------------------------------------ MBAFF (field / frame pairs)
  // The per-bin code reads its neighbours from sh->left (the left macroblock), ring[mb_x] (the
  // bottom edge of the upper one) and lf / tf / left_ok / top_ok.  In an MBAFF frame the
  // neighbours of a macroblock follow ITU-T H.264 Table 6-4 (6.4.12.2): rows of the left one may
  // come from either macroblock of the left pair, the upper one depends on the field / frame
  // coding of both pairs, and vertical mvd / ref_idx of a neighbour of the other kind are scaled
  // (9.3.3.1.1.6-7, FFmpeg fill_decode_caches MAP_F2F).  mbaff_view writes exactly that view into
  // sh->left and ring[mb_x] before each coded macroblock, so the per-bin code is the same.
  // LDS of an MBAFF launch (ring_cols >= 3 W + 7): ring[0, W) the views, ring[W + x] /
  // ring[2 W + x] the bottom edges of the last top / bottom macroblock of column x, then three
  // MbRec (this pair's top, the left pair's top and bottom, dword 0 = their cf) and four words:
  // the dword 0 of the left pair's top / bottom and of the upper pair's top / bottom edges.
  static constexpr uint32_t F_FLD = 0x100;   // cf: field macroblock
  static constexpr uint32_t PST_FLD = 1, PST_SKIPT = 2, PST_SKIPB = 4, PST_BOT = 8;
  AVR_FI ERec* pair_edge(int bot) const { return ring + (1 + bot) * W; }
  AVR_FI MbRec* pair_rec() const { return (MbRec*)(ring + 3 * W); }
  AVR_FI uint32_t* pair_nb() const { return (uint32_t*)(pair_rec() + 3); }
  AVR_FI uint32_t lds_u32(const uint32_t* p) const { return __builtin_amdgcn_readfirstlane(*p); }

  // top macroblock of a pair: the neighbour pairs' words and the inferred field flag (7.4.4: the
  // left pair's in the slice, else the upper pair's, else frame)
  AVR_FI void mbaff_pair_start() {
    const uint32_t L = __lane_id();
    uint32_t v = 0;
    if (L < 2) v = mb_x > 0 ? *(const uint32_t*)&pair_rec()[1 + L] : 0u;
    else if (L < 4) v = *(const uint32_t*)&pair_edge((int)L - 2)[mb_x];
    if (L < 4) pair_nb()[L] = v;
    wave_sync();
    const uint32_t lt = __builtin_amdgcn_readlane(v, 0), at = __builtin_amdgcn_readlane(v, 2);
    pst = ((lt & F_DEC) ? (lt & F_FLD) : (at & F_DEC) ? (at & F_FLD) : 0u) ? PST_FLD : 0u;
  }
  // mb_skip_flag ctxIdx (FFmpeg decode_cabac_mb_skip); top_d0 = this pair's top macroblock's cf
  AVR_FI int mbaff_skip_ctx(int bottom, uint32_t fld, uint32_t top_d0) const {
    const uint32_t* nb = pair_nb();
    const uint32_t lt = lds_u32(nb), lb = lds_u32(nb + 1), at = lds_u32(nb + 2), ab = lds_u32(nb + 3);
    uint32_t a = 0, b = 0;
    if (lt & F_DEC) a = (bottom && fld == ((lt & F_FLD) ? 1u : 0u)) ? lb : lt;
    if (fld) {
      if (at & F_DEC) b = (!bottom && (at & F_FLD)) ? at : ab;
    } else {
      b = bottom ? top_d0 : ab;
    }
    return (is_b ? 24 : 11) + ((a & F_DEC) && !(a & F_SKIP)) + ((b & F_DEC) && !(b & F_SKIP));
  }
  // mb_field_decoding_flag, ctxIdx 70-72 (FFmpeg decode_cabac_field_decoding_flag)
  AVR_FI uint32_t mbaff_field_flag(uint32_t inferred) {
    const uint32_t at = lds_u32(pair_nb() + 2);
    return (uint32_t)bin(SE_OTHER, 0, 70 + (mb_x > 0 && inferred) + ((at & F_DEC) && (at & F_FLD)));
  }
  // FFmpeg's order: a skipped top macroblock takes the bottom's skip flag next and, when the bottom
  // is coded, the pair's field flag; a coded top reads the field flag after its skip flag
  AVR_FI int mbaff_skip() {
    const int bottom = (pst & PST_BOT) != 0;
    uint32_t fld = pst & PST_FLD;
    int skip;
    if (bottom && (pst & PST_SKIPT)) skip = (pst & PST_SKIPB) != 0;
    else skip = bin(SE_OTHER, 0, mbaff_skip_ctx(bottom, fld, lds_u32((const uint32_t*)&pair_rec()[0])));
    if (skip && !bottom) {
      pst |= PST_SKIPT;
      if (bin(SE_OTHER, 0, mbaff_skip_ctx(1, fld, F_DEC | F_SKIP))) {
        pst |= PST_SKIPB;
      } else {
        fld = mbaff_field_flag(fld);
        pst = (pst & ~PST_FLD) | fld;
      }
    }
    if (skip && fld) cf |= F_FLD;
    return skip;
  }
  // Table 6-4, xN < 0: the left pair's macroblock (s: 0 top, 1 bottom) and 4x4 row r holding row y4
  // of a plane maxH samples high, for a field (fld) or frame current macroblock and a frame
  // (afrm) or field left pair
  AVR_FI static void left_src(uint32_t fld, int afrm, int bottom, int y4, int maxH, int* s, int* r) {
    const int yN = 4 * y4;
    if (!fld) {
      if (afrm) { *s = bottom; *r = y4; return; }
      *s = 0;
      *r = (bottom ? (yN + maxH) >> 1 : yN >> 1) >> 2;
      return;
    }
    if (afrm) {
      const int y2 = 2 * yN + bottom;
      if (yN < maxH / 2) { *s = 0; *r = y2 >> 2; }
      else { *s = 1; *r = (y2 - maxH) >> 2; }
      return;
    }
    *s = bottom;
    *r = y4;
  }
  // vertical |mvd| bytes (1, 3) and ref_idx bytes of a neighbour of the other coding: a field
  // neighbour of a frame macroblock counts double motion and half the references, and vice versa
  AVR_FI static uint32_t scale_mvd(uint32_t v, uint32_t fld) {
    return fld ? ((v & 0x00ff00ffu) | ((v >> 1) & 0x7f007f00u)) : ((v & 0x00ff00ffu) | ((v & 0xff00ff00u) << 1));
  }
  AVR_FI static uint32_t scale_ref(uint32_t v, uint32_t fld) {
    uint32_t o = 0;
    for (int k = 0; k < 4; k++) {
      int r = (int8_t)(v >> (8 * k));
      if (r >= 0) r = fld ? r * 2 : r >> 1;
      o |= (uint32_t)(uint8_t)r << (8 * k);
    }
    return o;
  }
  AVR_FI void mbaff_view(int bottom, uint32_t fld) {
    set_fld((int)fld);
    nref0 = d->num_ref_idx_l0 << fld;   // a field macroblock addresses fields: twice the references
    nref1 = d->num_ref_idx_l1 << fld;
    const uint32_t L = __lane_id();
    const uint32_t* nb = pair_nb();
    const uint32_t lt = lds_u32(nb), lb = lds_u32(nb + 1), at = lds_u32(nb + 2);
    // ---- left: sh->left, lane j = dword j, gathered from the left pair's records
    left_ok = (lt & F_DEC) != 0;
    if (left_ok) {
      const int afrm = !(lt & F_FLD);
      const MbRec* lp = pair_rec() + 1;
      int s0, r0, s2, r2;
      left_src(fld, afrm, bottom, 0, 16, &s0, &r0);
      left_src(fld, afrm, bottom, 2, 16, &s2, &r2);
      const uint32_t A = s0 ? lb : lt, C = s2 ? lb : lt;
      const uint32_t cbpA = A >> 16, cbpC = C >> 16;
      const uint32_t cbp = (cbpA & 0x7F0u) | (((cbpA >> ((r0 >> 1) * 2 + 1)) & 1u) << 1) |
                           (((cbpC >> ((r2 >> 1) * 2 + 1)) & 1u) << 3);
      lf = (A & 0xffffu) | cbp << 16;
      uint32_t t8rows = 0;
      for (int y4 = 0; y4 < 4; y4++) {
        int sy, ry;
        left_src(fld, afrm, bottom, y4, 16, &sy, &ry);
        t8rows |= (((sy ? lb : lt) & F_T8) ? 1u : 0u) << y4;
      }
      int s = 0, dw = 0;
      if (L >= 1 && L < 13) {          // nnz rows
        const int p = ((int)L - 1) >> 2;
        int r;
        left_src(fld, afrm, bottom, ((int)L - 1) & 3, (cat_ == 1 && p) ? 8 : 16, &s, &r);
        dw = 1 + p * 4 + min(r, 3);
      } else if (L >= 13 && L < 29) {  // mvd rows (two dwords per row)
        const int k = ((int)L - 13) & 7;
        int r;
        left_src(fld, afrm, bottom, k >> 1, 16, &s, &r);
        dw = 13 + (((int)L - 13) >> 3) * 8 + r * 2 + (k & 1);
      } else if (L == 29 || L == 30 || L == 31) {
        s = s0;
        dw = (int)L;
      } else if (L >= 32 && L < 45) {  // model bytes: the left macroblock in the same row
        s = bottom;
        dw = (int)L;
      }
      uint32_t v = L < 45 ? ((const uint32_t*)&lp[s])[dw] : 0u;
      const uint32_t v2 = (L >= 29 && L < 32) ? ((const uint32_t*)&lp[s2])[L] : 0u;
      if (L == 0) {
        v = t8rows | cbp << 16;
      } else if (L >= 13 && L < 29) {
        if (fld != (uint32_t)(!afrm)) v = scale_mvd(v, fld);
      } else if (L == 29 || L == 30 || L == 31) {
        // b8 1 <- row 0's source, b8 3 <- row 2's (the only left 8x8 blocks read: ref_idx / direct
        // of partitions at y4 = 0 and 2)
        const uint32_t b1 = (v >> (8 * ((r0 >> 1) * 2 + 1))) & 0xff, b3 = (v2 >> (8 * ((r2 >> 1) * 2 + 1))) & 0xff;
        v = (L == 31 ? 0u : 0xff00ffu) | b1 << 8 | b3 << 24;
        if (L != 31 && fld != (uint32_t)(!afrm)) v = scale_ref(v, fld);
      }
      if (L < 45) ((uint32_t*)&sh->left)[L] = v;
    }
    // ---- upper: ring[mb_x] from the pair edges (parse neighbour B) + the model's upper macroblock
    const int above = (at & F_DEC) != 0;
    const int sel = !fld ? (bottom ? 1 : above ? 2 : 0) : above ? ((!bottom && (at & F_FLD)) ? 1 : 2) : 0;
    const int msel = bottom ? 1 : above ? 2 : 0;
    uint32_t v = 0;
    if (L < 10 && sel) v = ((const uint32_t*)&pair_edge(sel - 1)[mb_x])[L];
    else if (L >= 10 && L < 23 && msel) v = ((const uint32_t*)&pair_edge(msel - 1)[mb_x])[L];
    const uint32_t t0 = __builtin_amdgcn_readlane(v, 0);
    if (sel && ((t0 & F_FLD) ? 1u : 0u) != fld) {
      if (L >= 4 && L < 8) v = scale_mvd(v, fld);
      else if (L == 8) v = scale_ref(v, fld);
    }
    if (L < 23) ((uint32_t*)&ring[mb_x])[L] = v;
    tf = t0;
    top_ok = sel != 0;
    wave_sync();
  }
  AVR_FI void mbaff_layer_begin() {
    const int bottom = (pst & PST_BOT) != 0;
    uint32_t fld = pst & PST_FLD;
    if (!bottom) {
      fld = mbaff_field_flag(fld);
      pst = (pst & ~PST_FLD) | fld;
    }
    if (fld) cf |= F_FLD;
    mbaff_view(bottom, fld);
  }

  // ------------------------------------------------------------------ model neighbours
  // model num_nonzeros of a neighbouring macroblock (get_neighbor_sub_mb, recode.cpp:419-471)
  AVR_FI int mnnz_left(int idx) const {
    if (RM) return frames[cur_off + ((int64_t)mrow() * W + mb_x - 1) * 52 + idx];
    return left_ok ? sh->left.mnnz[idx] : 0;
  }
  AVR_FI int mnnz_top(int idx) const {
    if (RM) return (FLD && top_pending) ? 0 : frames[cur_off + ((int64_t)(mrow() - 1) * W + mb_x) * 52 + idx];
    // fresh model per slice: in a field picture the model's upper row belongs to the other field
    if (FLD && fld_pic) return 0;
    if constexpr (FLD) {
      return (top_ok | mbaff) ? ring[mb_x].mnnz[idx] : 0;   // MBAFF: the view holds the model's upper macroblock
    } else {
      if (!top_ok) return 0;
      const uint32_t at = (uint32_t)mb_x * (kMringDwords * 4) + mring_dword((uint32_t)idx >> 2) * 4 + ((uint32_t)idx & 3);
      if (mring_global) return (tf & kEdgeMringNz) ? ((const __attribute__((address_space(1))) uint8_t*)mring)[at] : 0;
      return ((const __attribute__((address_space(3))) uint8_t*)mring)[at];
    }
  }
  AVR_FI int mnnz_prev(int idx) const {
    if (RM) return prev_off < 0 ? 0 : frames[prev_off + ((int64_t)mrow() * W + mb_x) * 52 + idx];
    return 0;
  }

  // finished_queueing (recode.cpp:845-930): the 2/4/6 nnz bits, LSB first
  AVR_FI int nz_bits(int cat, int n, int max, int is_dc, int c422, int count) {
    const int bits = max > 16 ? 6 : max > 4 ? 4 : 2;
    // the R-mode compress's count pass (rscan without a sink) needs the number of ops only: skip
    // the neighbours' frame loads (measured: R-mode compress -2 % clip, -4 % cockatoo)
    if (MODE == MODE_COMPRESS && RM && gmode && !gsink) {
      gcount += (uint32_t)bits;
      return count & ((1 << bits) - 1);
    }
    int has_left, has_above, lv = 0, av = 0;
    if (n >= 48) {
      has_left = mb_x > 0;
      has_above = mrow() > 0;
      if (has_left) lv = mnnz_left(n);
      if (has_above) av = mnnz_top(n);
    } else {
      uint8_t L = T->nb_left[n], U = T->nb_up[n];
      int li = L & 63, ui = U & 63;
      if (max >= 32) { li &= ~3; ui &= ~3; }
      has_left = !(L & 128) || mb_x > 0;
      has_above = !(U & 128) || mrow() > 0;
      if (has_left) lv = (L & 128) ? mnnz_left(li) : sh->cur.mnnz[li];
      if (has_above) av = (U & 128) ? mnnz_top(ui) : sh->cur.mnnz[ui];
    }
    const int pv = mnnz_prev(n);
    const int t = (((cf & CF_8X8) || max > 32) ? 1 : 0) + 2 * is_dc + c422 + 4 * cat;
    if (MODE == MODE_COMPRESS) {
      // all bits at once, bit i in lane i (so_far = the count's bits below i)
      const int i = (int)__lane_id();
      const int cur_bit = 1 << (i & 7);
      const int so_far = count & (cur_bit - 1);
      const int lb = has_left ? (lv >= cur_bit) : 2;
      const int ab = av ? (av >= cur_bit) : 2;
      const int pb = pv >= cur_bit;
      const int idx = kSigEst + (((((cur_bit - 1 + so_far) * 2 + pb) * 3 + lb) * 3 + ab) * 57 + t);
      push_v(op_model((count >> (i & 7)) & 1, OPM_CACHE, idx), (uint32_t)bits);
      return count & ((1 << bits) - 1);
    }
    if (MODE == MODE_DECOMPRESS) {
      // every key of the bit tree at once (lane (1 << i) - 1 + so_far: bit i after so_far; the
      // keys are distinct), then the bits in order with the estimators already in registers
      const uint32_t L = __lane_id();
      const int i = 31 - __clz((int)L + 1);
      const int cur_bit = 1 << i;
      const int lb = has_left ? (lv >= cur_bit) : 2;
      const int ab = av ? (av >= cur_bit) : 2;
      const int pb = pv >= cur_bit;
      const uint32_t idx_v = kSigEst + ((((L * 2 + pb) * 3 + lb) * 3 + ab) * 57 + t);
      uint32_t e_v = 0, slot_v = 0;
      const bool hit = est_probe4(sh, idx_v, &e_v, &slot_v);   // lanes past the tree are never read
      const uint64_t hit_m = __ballot(hit);
      int so_far = 0;
      for (int k = 0; k < bits; k++) {
        const uint32_t j = (1u << k) - 1 + (uint32_t)so_far;
        const uint32_t idx = __builtin_amdgcn_readlane(idx_v, j);
        uint32_t e, slot;
        if ((hit_m >> j) & 1) {
          e = __builtin_amdgcn_readlane(e_v, j);
          slot = __builtin_amdgcn_readlane(slot_v, j);
        } else {
          e = est_load(sh, est_g, idx, &slot);
        }
        const int b = rdec(e);
        est_store(sh, est_g, idx, slot, est_update(e, b, 0x60));
        so_far |= b << k;
      }
      return so_far;
    }
    int so_far = 0;
    for (int i = 0; i < bits; i++) {
      const int cur_bit = 1 << i;
      const int lb = has_left ? (lv >= cur_bit) : 2;
      const int ab = av ? (av >= cur_bit) : 2;
      const int pb = pv >= cur_bit;
      const int idx = kSigEst + (((((cur_bit - 1 + so_far) * 2 + pb) * 3 + lb) * 3 + ab) * 57 + t);
      int b;
      if (MODE == MODE_COMPRESS) {
        b = (count >> i) & 1;
        push(op_model(b, OPM_CACHE, idx));
      } else {
        uint32_t slot;
        const uint32_t e = est_load(sh, est_g, idx, &slot);
        b = rdec(e);
        est_store(sh, est_g, idx, slot, est_update(e, b, 0x60));
      }
      if (b) so_far |= cur_bit;
    }
    return so_far;
  }

  AVR_FI int sig_est_index(int cat, int max, int is_dc, int c422, int zz, int nnz_m, int obs) const {
    if (max == 64) return T->sig_est_base[cat] + (T->sig8x8[zz] * 64 + nnz_m) * 64 + obs;
    int zo = (is_dc && c422) ? (zz < 2 ? 0 : zz < 4 ? 1 : 2) : zz;
    return T->sig_est_base[cat] + (zo * 16 + nnz_m) * 16 + obs;
  }

  // significance map of one residual block; returns the coefficient count
  AVR_FI int sig_map(int cat, int n, int max, int is_dc, int c422) {
    const int numc8x8 = cat_ == 2 ? 2 : 1;
    const int sb = T->sig_base[cat], lb = T->last_base[cat], seb = (int)opaque_u32((uint32_t)T->sig_est_base[cat]);
    const int bits = max > 16 ? 6 : max > 4 ? 4 : 2;
    const int mask = (1 << bits) - 1;
    int cnt = 0;
    if (DEC) {
      uint64_t sigmask = 0;
      int pos, end = max - 2;
      PROF_BEGIN(t3);
      if (MODE == MODE_TRACE) trace_map_begin(cat, n, max, is_dc, c422);
      // the loop once per block kind (K: 0 4x4-class, 1 chroma DC, 2 8x8), so that no per-bin
      // code selects between them (one call site, kinds known only at run time)
      auto map_loop = [&](auto K) {
        constexpr int k = decltype(K)::value;
        for (pos = 0; pos < max - 1; pos++) {
          int sc, lc;
          if constexpr (k == 2) {
            sc = (int)__builtin_amdgcn_readlane(sig8_v, (uint32_t)pos);
            lc = (int)__builtin_amdgcn_readlane(last8_v, (uint32_t)pos);
          } else if constexpr (k == 1) {
            sc = lc = min(pos / numc8x8, 2);
          } else {
            sc = lc = pos;
          }
          if (rdecide(sc)) {
            sigmask |= 1ull << pos;
            cnt++;
            if (rdecide(16 + lc)) { end = pos; break; }
          }
        }
      };
      if (max == 64) map_loop(std::integral_constant<int, 2>());
      else if (cat == 3) map_loop(std::integral_constant<int, 1>());
      else map_loop(std::integral_constant<int, 0>());
      if (pos == max - 1) cnt++;
      if (MODE == MODE_TRACE) trace_map_end();
      PROF_END(3, t3);
      if (MODE == MODE_COMPRESS) {
        // model: nnz first (recode.cpp:1208-1221), then the buffered map (1244-1255)
        PROF_BEGIN(t4);
        nz_bits(cat, n, max, is_dc, c422, cnt);
        PROF_END(4, t4);
        PROF_BEGIN(t5);
        const int nnz_m = cnt & mask;
        // positions 0..end at once, position zz in lane zz (obs = significant positions before it)
        const int zz = (int)__lane_id();
        const int b = (int)((sigmask >> zz) & 1);
        const int obs = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(sigmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sigmask, 0u));
        const int idx = sig_est_index(cat, max, is_dc, c422, zz, nnz_m, obs);
        push_v(op_model(b, OPM_CACHE | OPM_THR50, idx), (uint32_t)end + 1);
        PROF_END(5, t5);
      }
    } else if (MODE == MODE_DECOMPRESS) {
      PROF_BEGIN(t4);
      const int nnz_m = nz_bits(cat, n, max, is_dc, c422, 0);   // recode.cpp:1476-1486
      PROF_END(4, t4);
      PROF_BEGIN(t3);
      int pos;
      // the coder ops of the map's bins: scalar bases, one add of (ctxIdxInc << 3) + bin each
      const uint32_t sop = opaque_u32((uint32_t)sb << 3 | OPK_DECISION << 1 | 1u << OPC_SHIFT_D);
      const uint32_t lop = opaque_u32((uint32_t)lb << 3 | OPK_DECISION << 1 | 2u << OPC_SHIFT_D);
      // one loop per block kind (K: 0 4x4-class, 1 chroma DC, 2 8x8; see the DEC side)
      auto map_loop = [&](auto K) {
        constexpr int k = decltype(K)::value;
        constexpr int stride = k == 2 ? 64 : 16;
        uint32_t mk = 0;   // progressive walker: the significance bits of this 16-position segment
        // 4x4-class maps key each position's estimator by the position itself, so no key repeats
        // within the map: the LDS write-backs wait in two VGPRs (lane = position) for one store
        // after the loop (a new key claims its slot at once, est_load).  Chroma DC and 8x8 maps
        // reuse keys within the map and store at once.
        constexpr bool defer = k == 0;
        uint32_t dslot_v = 0, de_v = 0;
        for (pos = 0; pos < max - 1; pos++) {
          int sc, lc, zo;
          if constexpr (k == 2) {
            const uint32_t v = __builtin_amdgcn_readlane(sig8_v, (uint32_t)pos);   // CABAC inc | key inc << 8 (FLD)
            sc = FLD ? (int)(v & 0xff) : (int)v;
            zo = FLD ? (int)(v >> 8) : (int)v;
            lc = (int)__builtin_amdgcn_readlane(last8_v, (uint32_t)pos);
          } else if constexpr (k == 1) {
            sc = lc = min(pos / numc8x8, 2);
            zo = (is_dc && c422) ? (pos < 2 ? 0 : pos < 4 ? 1 : 2) : pos;
          } else {
            sc = lc = zo = pos;
          }
          const int idx = seb + (zo * stride + nnz_m) * stride + cnt;   // sig_est_index
          uint32_t slot;
          uint32_t e = est_load(sh, est_g, idx, &slot, defer);
          int b = rdec(e);
          const uint32_t ne = est_update(e, b, 0x50);
          if (defer && (slot >> 31)) {
            dslot_v = wlane(dslot_v, (uint32_t)pos, slot);
            de_v = wlane(de_v, (uint32_t)pos, ne);
          } else {
            est_store(sh, est_g, idx, slot, ne);
          }
          bins++;
          if constexpr (FLD) push(sop + ((uint32_t)sc << 3) + (uint32_t)b);
          else mk |= (uint32_t)b << (pos & 15);
          if (b) {
            cnt++;
            int last = nnz_m == cnt;   // derived EOB (recode.cpp:1437-1438)
            bins++;
            if constexpr (FLD) push(lop + ((uint32_t)lc << 3) + (uint32_t)last);
            if (last) break;
          }
          if constexpr (!FLD && k == 2) {
            if ((pos & 15) == 15) {
              push(op_map(cat, 16, 0, mk));
              mk = 0;
            }
          }
        }
        if constexpr (defer) {
          if (dslot_v >> 31) sh->etab[dslot_v & 0xffff] = (dslot_v & 0xffff0000u) | de_v;
          wave_sync();
        }
        if constexpr (!FLD) {
          const int ended = pos < max - 1;
          push(op_map(cat, (pos & 15) + ended, ended, mk));
        }
      };
      if (max == 64) map_loop(std::integral_constant<int, 2>());
      else if (cat == 3) map_loop(std::integral_constant<int, 1>());
      else map_loop(std::integral_constant<int, 0>());
      if (pos == max - 1) cnt++;
      PROF_END(3, t3);
    } else {
      int pos;
      for (pos = 0; pos < max - 1; pos++) {
        int sc, lc;
        if (max == 64) {
          sc = (int)__builtin_amdgcn_readlane(sig8_v, (uint32_t)pos);
          lc = (int)__builtin_amdgcn_readlane(last8_v, (uint32_t)pos);
        }
        else if (cat == 3) { sc = lc = min(pos / numc8x8, 2); }
        else sc = lc = pos;
        if (rbin(sc, sb + sc)) {
          cnt++;
          if (rbin(16 + lc, lb + lc)) break;
        }
      }
      if (pos == max - 1) cnt++;
    }
    return cnt;
  }

  // residual_block_cabac() of one block; p/x4/y4 locate it in the walker's nnz grid
  AVR_FI void residual_block(int cat, int n, int max, int is_dc, int c422, int p, int pw, int x4, int y4) {
    if (err) return;
    MbRec& cur = sh->cur;
    int coded = 1;
    if (max != 64 || cat_ == 3) {
      int nza, nzb;
      if (is_dc) {
        int bit = cat == 3 ? (0x40 << (n - 49)) : (0x100 << (n - 48));
        nza = (nb_cbp_left() & bit) != 0;
        nzb = (nb_cbp_top() & bit) != 0;
      } else {
        nza = nnz_left(p, pw, x4, y4) > 0;
        nzb = nnz_top(p, x4, y4) > 0;
      }
      rc_select(cat);
      coded = rbin(42 + nza + 2 * nzb, T->cbf_base[cat] + nza + 2 * nzb);
    }
    int cnt = 0;
    if (coded) {
      rc_select(cat);
      cnt = sig_map(cat, n, max, is_dc, c422);
      // coeff_abs_level_minus1 + sign, reverse scan order
      const int ab = (int)opaque_u32((uint32_t)T->abs_base[cat]);   // scalar: the coder ops' base
      int gt1 = 0, eq1 = 0;
      PROF_BEGIN(t6);
      if constexpr (MODE == MODE_DECOMPRESS && !FLD) {
        // one coder op per coefficient (op_level): the coder derives the level bins' contexts
        for (int i = cnt - 1; i >= 0 && !err; i--) {
          int absl;
          const int i0 = gt1 ? 0 : min(4, 1 + eq1);
          if (!rdec_lane(32 + i0)) {
            absl = 1;
          } else {
            const int i1 = 5 + min(4 - (cat == 3), gt1);
            absl = 2;
            while (absl < 15 && rdec_lane(32 + i1)) absl++;
          }
          if (absl < 15) {
            push(op_level(cat, absl, rdec_bypass()));
          } else {   // escape: the prefix as one op, suffix and sign bin by bin
            push(op_level(cat, 15, 0));
            int k = 0;
            while (bypass(SE_LEVEL_SUFFIX, k)) {
              if (++k > 30) { err = AVR_SLICE_BAD_LEVEL; break; }
            }
            while (k-- > 0) bypass(SE_LEVEL_SUFFIX, 100);
            bypass(SE_OTHER, 0);
          }
          if (absl == 1) eq1++;
          else gt1++;
        }
      } else if constexpr (MODE == MODE_COMPRESS && kStageLevels) {
        // the block's level ops staged in a VGPR and stored together after the block
        const bool st = !(RM && gmode);
        auto lpush = [&](uint32_t op) {
          if (st) ring0.stage(op);
          else push(op);
        };
        auto lbyp = [&]() {
          bins++;
          const int b = cd_bypass(cd, in);
          lpush(op_model(b, 0, 1024));
          return b;
        };
        for (int i = cnt - 1; i >= 0 && !err; i--) {
          int absl;
          const int i0 = gt1 ? 0 : min(4, 1 + eq1);
          int b = rdecide(32 + i0);
          lpush(op_model(b, 0, ab + i0));
          if (!b) {
            absl = 1;
          } else {
            const int i1 = 5 + min(4 - (cat == 3), gt1);
            absl = 2;
            while (absl < 15) {
              b = rdecide(32 + i1);
              lpush(op_model(b, 0, ab + i1));
              if (!b) break;
              absl++;
            }
            if (absl >= 15) {
              int k = 0;
              while (lbyp()) {
                if (++k > 30) { err = AVR_SLICE_BAD_LEVEL; break; }
              }
              while (k-- > 0) lbyp();
            }
          }
          lbyp();
          if (absl == 1) eq1++;
          else gt1++;
        }
        if (st) ring0.flush_stage();
      } else
      for (int i = cnt - 1; i >= 0 && !err; i--) {
        int absl;
        const int i0 = gt1 ? 0 : min(4, 1 + eq1);
        if (!rbin(32 + i0, ab + i0)) {
          absl = 1;
        } else {
          const int i1 = 5 + min(4 - (cat == 3), gt1);
          absl = 2;
          while (absl < 15 && rbin(32 + i1, ab + i1)) absl++;
          if (absl >= 15) {
            int k = 0;
            while (bypass(SE_LEVEL_SUFFIX, k)) {
              if (++k > 30) { err = AVR_SLICE_BAD_LEVEL; break; }
            }
            int v = 1;
            while (k-- > 0) v += v + bypass(SE_LEVEL_SUFFIX, 100);
            absl = 14 + v;
          }
        }
        bypass(SE_OTHER, 0);
        if (absl == 1) eq1++;
        else gt1++;
      }
      PROF_END(6, t6);
      cur.mnnz[n] = (uint8_t)cnt;             // end_coding_type recount (recode.cpp:935-947)
      if (max > 32) cf |= CF_8X8;
    }
    if (is_dc) {
      if (cnt) cf |= (uint32_t)(cat == 3 ? (0x40 << (n - 49)) : (0x100 << (n - 48))) << 16;
    } else if (max == 64) {
      cur.nnz[p][y4 * 4 + x4] = cur.nnz[p][y4 * 4 + x4 + 1] = (uint8_t)cnt;
      cur.nnz[p][y4 * 4 + 4 + x4] = cur.nnz[p][y4 * 4 + 4 + x4 + 1] = (uint8_t)cnt;
    } else {
      cur.nnz[p][y4 * 4 + x4] = (uint8_t)cnt;
    }
  }

  AVR_FI void blk_pos(int n, int* x4, int* y4) const {
    int s = c_scan8[n];
    int row = s >> 3;
    *x4 = (s & 7) - 4;
    *y4 = row <= 4 ? row - 1 : row <= 9 ? row - 6 : row - 11;
  }

  // The macroblock's residual blocks in bitstream order (residual(), 7.3.5.3) are listed in LDS
  // first and then coded through ONE inlined residual_block site, so the per-bin code exists
  // once in the kernel instead of once per block kind.
  AVR_FI int push_block(int nb, int cat, int n, int max, int is_dc, int c422, int p, int pw, int x4, int y4) {
    sh->blk[nb] = (uint32_t)cat | (uint32_t)n << 4 | (uint32_t)max << 10 | (uint32_t)is_dc << 17 |
                  (uint32_t)c422 << 18 | (uint32_t)p << 19 | (uint32_t)pw << 21 | (uint32_t)x4 << 24 |
                  (uint32_t)y4 << 26;
    return nb + 1;
  }
  AVR_FI int list_luma(int nb, int p, int i16, int cbp) {
    const int cat_dc = p == 0 ? 0 : p == 1 ? 6 : 10;
    const int cat_ac = cat_dc + 1, cat_4 = cat_dc + 2, cat_8 = p == 0 ? 5 : p == 1 ? 9 : 13;
    int x4, y4;
    if (i16) {
      nb = push_block(nb, cat_dc, 48 + p, 16, 1, 0, p, 4, 0, 0);
      if (cbp & 15)
        for (int i = 0; i < 16; i++) {
          blk_pos(16 * p + i, &x4, &y4);
          nb = push_block(nb, cat_ac, 16 * p + i, 15, 0, 0, p, 4, x4, y4);
        }
      return nb;
    }
    for (int i8 = 0; i8 < 4; i8++) {
      if (!(cbp & (1 << i8))) continue;
      if (cf & F_T8) {
        blk_pos(16 * p + 4 * i8, &x4, &y4);
        nb = push_block(nb, cat_8, 16 * p + 4 * i8, 64, 0, 0, p, 4, x4, y4);
      } else {
        for (int i4 = 0; i4 < 4; i4++) {
          int n = 16 * p + 4 * i8 + i4;
          blk_pos(n, &x4, &y4);
          nb = push_block(nb, cat_4, n, 16, 0, 0, p, 4, x4, y4);
        }
      }
    }
    return nb;
  }

  AVR_FI void residual(int i16, int cbp) {
    int nb = list_luma(0, 0, i16, cbp);
    if (cat_ == 3) {
      nb = list_luma(nb, 1, i16, cbp);
      nb = list_luma(nb, 2, i16, cbp);
    } else if (cat_ == 1 || cat_ == 2) {
      const int c422 = cat_ == 2;
      if (cbp & 0x30)
        for (int c = 0; c < 2; c++) nb = push_block(nb, 3, 49 + c, c422 ? 8 : 4, 1, c422, 1 + c, 2, 0, 0);
      if (cbp & 0x20)
        for (int c = 0; c < 2; c++)
          for (int i8 = 0; i8 < (c422 ? 2 : 1); i8++)
            for (int i = 0; i < 4; i++) {
              int n = 16 + 16 * c + 8 * i8 + i, x4, y4;
              blk_pos(n, &x4, &y4);
              nb = push_block(nb, 4, n, 15, 0, 0, 1 + c, 2, x4, y4);
            }
    }
    PROF_BEGIN(t2);
    for (int j = 0; j < nb && !err; j++) {
      const uint32_t b = sh->blk[j];
      residual_block(b & 15, (b >> 4) & 63, (b >> 10) & 127, (b >> 17) & 1, (b >> 18) & 1, (b >> 19) & 3,
                     (b >> 21) & 7, (b >> 24) & 3, (b >> 26) & 3);
    }
    PROF_END(2, t2);
  }

  // ------------------------------------------------------------------ prediction syntax
  AVR_FI int ref_gt0(int list, int x4, int y4, int use_left) const {
    uint8_t dir;
    int r;
    if (use_left) {
      if (x4 > 0) {
        int b8 = (y4 >> 1) * 2 + ((x4 - 1) >> 1);
        dir = sh->cur.direct8[b8]; r = sh->cur.ref[list][b8];
      } else {
        if (!left_ok) return 0;
        int b8 = (y4 >> 1) * 2 + 1;
        dir = sh->left.direct8[b8]; r = sh->left.ref[list][b8];
      }
    } else {
      if (y4 > 0) {
        int b8 = ((y4 - 1) >> 1) * 2 + (x4 >> 1);
        dir = sh->cur.direct8[b8]; r = sh->cur.ref[list][b8];
      } else {
        if (!top_ok) return 0;
        dir = ring[mb_x].direct8[x4 >> 1]; r = ring[mb_x].ref[list][x4 >> 1];
      }
    }
    if (is_b && dir) return 0;
    return r > 0;
  }
  AVR_FI int decode_ref(int list, int x4, int y4) {
    int ctx = ref_gt0(list, x4, y4, 1) + 2 * ref_gt0(list, x4, y4, 0);
    int ref = 0;
    avr_limit = (list ? nref1 : nref0) - 1;
    while (bin(SE_REF, ref, 54 + ctx)) {
      ref++;
      ctx = (ctx >> 2) + 4;
      if (ref >= 32) { err = AVR_SLICE_BAD_REF_IDX; return 0; }
    }
    return ref;
  }
  AVR_FI int mvd_nb(int list, int comp, int x4, int y4, int use_left) const {
    if (use_left) {
      if (x4 > 0) return sh->cur.mvd[list][y4 * 4 + x4 - 1][comp];
      return left_ok ? sh->left.mvd[list][y4 * 4 + 3][comp] : 0;
    }
    if (y4 > 0) return sh->cur.mvd[list][(y4 - 1) * 4 + x4][comp];
    return top_ok ? ring[mb_x].mvd[list][x4][comp] : 0;
  }
  AVR_FI int decode_mvd(int list, int comp, int x4, int y4) {
    const int base = comp ? 47 : 40;
    const int amvd = mvd_nb(list, comp, x4, y4, 1) + mvd_nb(list, comp, x4, y4, 0);
    const int inc = amvd < 3 ? 0 : amvd <= 32 ? 1 : 2;
    if constexpr (MODE == MODE_DECOMPRESS && !FLD) {   // one op_mvd (+ an escape's bins)
      if (!rdec_mc(base + inc)) {
        push(op_mvd(comp, inc, 0, 0));
        return 0;
      }
      int mvd = 1, ctx = base + 3;
      while (mvd < 9 && rdec_mc(ctx)) {
        if (mvd < 4) ctx++;
        mvd++;
      }
      if (mvd < 9) {
        push(op_mvd(comp, inc, mvd, rdec_bypass()));
        return mvd;
      }
      push(op_mvd(comp, inc, 9, 0));
      int k = 3;
      while (bypass(SE_MVD_SUFFIX, k - 3)) {
        mvd += 1 << k;
        if (++k > 24) { err = AVR_SLICE_BAD_MVD; return 0; }
      }
      while (k--) mvd += bypass(SE_MVD_SUFFIX, 100) << k;
      bypass(SE_OTHER, 0);
      return mvd < 70 ? mvd : 70;
    }
    if (!bin(SE_OTHER, 0, base + inc)) return 0;
    int mvd = 1, ctx = base + 3;
    while (mvd < 9 && bin(SE_OTHER, 0, ctx)) {
      if (mvd < 4) ctx++;
      mvd++;
    }
    if (mvd >= 9) {
      int k = 3;
      while (bypass(SE_MVD_SUFFIX, k - 3)) {
        mvd += 1 << k;
        if (++k > 24) { err = AVR_SLICE_BAD_MVD; return 0; }
      }
      while (k--) mvd += bypass(SE_MVD_SUFFIX, 100) << k;
    }
    bypass(SE_OTHER, 0);
    return mvd < 70 ? mvd : 70;
  }
  AVR_FI void mvd_part(int list, int px, int py, int pw, int ph) {
    int mx = decode_mvd(list, 0, px, py);
    int my = decode_mvd(list, 1, px, py);
    for (int y = py; y < py + ph; y++)
      for (int x = px; x < px + pw; x++) {
        sh->cur.mvd[list][y * 4 + x][0] = (uint8_t)mx;
        sh->cur.mvd[list][y * 4 + x][1] = (uint8_t)my;
      }
  }

  AVR_FI int intra_mb_type(int base, int intra_slice, int* i16_cbp) {
    // returns 0 = I_NxN, 1 = I_16x16, 2 = I_PCM
    int ctx = 0;
    if (intra_slice) {
      if (left_ok && (lf & F_I16)) ctx++;
      if (top_ok && (tf & F_I16)) ctx++;
      if (!bin(SE_OTHER, 0, base + ctx)) return 0;
      base += 2;
    } else {
      if (!bin(SE_OTHER, 0, base)) return 0;
    }
    if (terminate(SE_PCM)) return 2;
    int luma = bin(SE_OTHER, 0, base + 1) ? 15 : 0;
    int chroma = 0;
    if (bin(SE_OTHER, 0, base + 2)) chroma = 1 + bin(SE_OTHER, 0, base + 2 + intra_slice);
    bin(SE_OTHER, 0, base + 3 + intra_slice);
    bin(SE_OTHER, 0, base + 3 + 2 * intra_slice);
    *i16_cbp = luma | (chroma << 4);
    return 1;
  }

  // ------------------------------------------------------------------ one macroblock
  AVR_FI void decode_mb() {
    MbRec& cur = sh->cur;
    const int nlists = is_b ? 2 : 1;
    PROF_BEGIN(ps1);
    if (slice_type != 2) {
      int skip;
      if (FLD && mbaff) skip = mbaff_skip();
      else skip = bin(SE_OTHER, 0, (is_b ? 24 : 11) + (left_ok && !(lf & F_SKIP)) + (top_ok && !(tf & F_SKIP)));
      if (skip) {
        cf |= F_SKIP;
        if (is_b) {
          cf |= F_D16;
          cur.direct8[0] = cur.direct8[1] = cur.direct8[2] = cur.direct8[3] = 1;
        } else {
          cur.ref[0][0] = cur.ref[0][1] = cur.ref[0][2] = cur.ref[0][3] = 0;
        }
        last_dqp_nz = 0;
        SPROF_END(1, ps1);
        return;
      }
    }
    if (FLD && mbaff) mbaff_layer_begin();
    SPROF_END(1, ps1);
    PROF_BEGIN(ps2);
    // mb_type
    int intra = 0, kind = 0, i16_cbp = 0, nparts = 0, vertical = 0, pred0 = 0, pred1 = 0, direct16 = 0;
    if (slice_type == 2) {
      intra = 1;
      kind = intra_mb_type(3, 1, &i16_cbp);
    } else if (slice_type == 0) {
      if (!bin(SE_OTHER, 0, 14)) {
        int mt;
        if (!bin(SE_OTHER, 0, 15)) mt = 3 * bin(SE_OTHER, 0, 16);
        else mt = 2 - bin(SE_OTHER, 0, 17);
        if (mt == 0) { nparts = 1; pred0 = 1; }
        else if (mt == 1) { nparts = 2; pred0 = pred1 = 1; }
        else if (mt == 2) { nparts = 2; vertical = 1; pred0 = pred1 = 1; }
        else nparts = 4;
      } else {
        intra = 1;
        kind = intra_mb_type(17, 0, &i16_cbp);
      }
    } else {
      int ctx = (left_ok && !(lf & F_D16)) + (top_ok && !(tf & F_D16));
      if (!bin(SE_OTHER, 0, 27 + ctx)) {
        direct16 = 1;
        nparts = 4;
      } else if (!bin(SE_OTHER, 0, 27 + 3)) {
        nparts = 1;
        pred0 = 1 + bin(SE_OTHER, 0, 27 + 5);
      } else {
        int bits = bin(SE_OTHER, 0, 27 + 4) << 3;
        bits |= bin(SE_OTHER, 0, 27 + 5) << 2;
        bits |= bin(SE_OTHER, 0, 27 + 5) << 1;
        bits |= bin(SE_OTHER, 0, 27 + 5);
        int mt = -1;
        if (bits < 8) mt = bits + 3;
        else if (bits == 13) { intra = 1; kind = intra_mb_type(32, 0, &i16_cbp); }
        else if (bits == 14) mt = 11;
        else if (bits == 15) mt = 22;
        else mt = ((bits << 1) | bin(SE_OTHER, 0, 27 + 5)) - 4;
        if (!intra) {
          if (mt == 3) { nparts = 1; pred0 = 3; }
          else if (mt == 22) nparts = 4;
          else {
            int k = mt - 4;
            nparts = 2;
            vertical = k & 1;
            pred0 = c_b_pairs[k >> 1][0];
            pred1 = c_b_pairs[k >> 1][1];
          }
        }
      }
    }
    SPROF_END(2, ps2);
    if (err) return;
    if (intra && kind == 2) { err = AVR_SLICE_PCM; return; }  // I_PCM (skip_bytes hook, recode.cpp:161-163)
    int no_sub_lt8x8 = 1;
    int t8 = 0;
    PROF_BEGIN(ps3);
    if (intra) {
      cf |= F_INTRA;
      if (kind == 1) cf |= F_I16;
      if (kind == 0) {
        if (t8mode) {
          t8 = bin(SE_OTHER, 0, 399 + (left_ok && (lf & F_T8)) + (top_ok && (tf & F_T8)));
          if (t8) cf |= F_T8;
        }
        const int nmodes = t8 ? 4 : 16;
        for (int i = 0; i < nmodes; i++)
          if (!bin(SE_OTHER, 0, 68)) {
            bin(SE_OTHER, 0, 69);
            bin(SE_OTHER, 0, 69);
            bin(SE_OTHER, 0, 69);
          }
      }
      if (cat_ == 1 || cat_ == 2) {
        int ctx = (left_ok && (lf & F_INTRA) && (lf & F_CPRED)) +
                  (top_ok && (tf & F_INTRA) && (tf & F_CPRED));
        if (bin(SE_OTHER, 0, 64 + ctx)) {
          cf |= F_CPRED;
          if (bin(SE_OTHER, 0, 67)) bin(SE_OTHER, 0, 67);
        }
      }
      SPROF_END(3, ps3);
    } else if (nparts == 4) {
      if (direct16) {
        cf |= F_D16;
        cur.direct8[0] = cur.direct8[1] = cur.direct8[2] = cur.direct8[3] = 1;
        if (!d8x8inf) no_sub_lt8x8 = 0;
      } else {
        uint32_t sub = 0;  // per 8x8: parts b0-2, vertical b3, pred b4-5 (no private arrays)
        for (int i = 0; i < 4; i++) {
          int t, sp, sv, spr;
          if (!is_b) {
            if (bin(SE_OTHER, 0, 21)) t = 0;
            else if (!bin(SE_OTHER, 0, 22)) t = 1;
            else if (bin(SE_OTHER, 0, 23)) t = 2;
            else t = 3;
            sp = t == 0 ? 1 : t == 3 ? 4 : 2;
            sv = t == 2;
            spr = 1;
          } else {
            if (!bin(SE_OTHER, 0, 36)) t = 0;
            else if (!bin(SE_OTHER, 0, 37)) t = 1 + bin(SE_OTHER, 0, 39);
            else {
              t = 3;
              if (bin(SE_OTHER, 0, 38)) {
                if (bin(SE_OTHER, 0, 39)) t = 11 + bin(SE_OTHER, 0, 39);
                else {
                  t += 4;
                  t += 2 * bin(SE_OTHER, 0, 39);
                  t += bin(SE_OTHER, 0, 39);
                }
              } else {
                t += 2 * bin(SE_OTHER, 0, 39);
                t += bin(SE_OTHER, 0, 39);
              }
            }
            if (t == 0) { sp = 0; sv = 0; spr = 0; }
            else if (t <= 3) { sp = 1; sv = 0; spr = t; }
            else if (t <= 9) { int k = t - 4; sp = 2; sv = k & 1; spr = (k >> 1) + 1; }
            else { sp = 4; sv = 0; spr = t - 9; }
          }
          sub |= (uint32_t)(sp | sv << 3 | spr << 4) << (8 * i);
          if (sp == 0) {
            cur.direct8[i] = 1;
            if (!d8x8inf) no_sub_lt8x8 = 0;
          } else if (sp > 1) {
            no_sub_lt8x8 = 0;
          }
        }
        SPROF_END(2, ps3);
        PROF_BEGIN(ps4);
        for (int list = 0; list < nlists; list++)
          for (int i = 0; i < 4; i++) {
            const int sp = (sub >> (8 * i)) & 7, spr = (sub >> (8 * i + 4)) & 3;
            if (!sp || !(spr & (1 << list))) continue;
            int nref = list ? nref1 : nref0;
            cur.ref[list][i] = (int8_t)(nref > 1 ? decode_ref(list, 2 * (i & 1), 2 * (i >> 1)) : 0);
          }
        SPROF_END(4, ps4);
        PROF_BEGIN(ps5);
        for (int list = 0; list < nlists; list++)
          for (int i = 0; i < 4; i++) {
            const int sp = (sub >> (8 * i)) & 7, sv = (sub >> (8 * i + 3)) & 1, spr = (sub >> (8 * i + 4)) & 3;
            if (!sp || !(spr & (1 << list))) continue;
            const int x0 = 2 * (i & 1), y0 = 2 * (i >> 1);
            for (int j = 0; j < sp; j++) {
              if (sp == 1) mvd_part(list, x0, y0, 2, 2);
              else if (sp == 4) mvd_part(list, x0 + (j & 1), y0 + (j >> 1), 1, 1);
              else if (!sv) mvd_part(list, x0, y0 + j, 2, 1);
              else mvd_part(list, x0 + j, y0, 1, 2);
            }
          }
        SPROF_END(5, ps5);
      }
    } else {
      SPROF_END(4, ps3);
      PROF_BEGIN(ps4);
      for (int list = 0; list < nlists; list++)
        for (int i = 0; i < nparts; i++) {
          const int pr = i ? pred1 : pred0;
          if (!(pr & (1 << list))) continue;
          const int px = (nparts == 2 && vertical) ? 2 * i : 0, py = (nparts == 2 && !vertical) ? 2 * i : 0;
          const int nref = list ? nref1 : nref0;
          const int ref = nref > 1 ? decode_ref(list, px, py) : 0;
          if (nparts == 1) cur.ref[list][0] = cur.ref[list][1] = cur.ref[list][2] = cur.ref[list][3] = (int8_t)ref;
          else if (!vertical) cur.ref[list][2 * i] = cur.ref[list][2 * i + 1] = (int8_t)ref;
          else cur.ref[list][i] = cur.ref[list][i + 2] = (int8_t)ref;
        }
      SPROF_END(4, ps4);
      PROF_BEGIN(ps5);
      for (int list = 0; list < nlists; list++)
        for (int i = 0; i < nparts; i++) {
          const int pr = i ? pred1 : pred0;
          if (!(pr & (1 << list))) continue;
          if (nparts == 1) mvd_part(list, 0, 0, 4, 4);
          else if (vertical) mvd_part(list, 2 * i, 0, 2, 4);
          else mvd_part(list, 0, 2 * i, 4, 2);
        }
      SPROF_END(5, ps5);
    }
    if (err) return;
    PROF_BEGIN(ps6);
    int cbp;
    if (intra && kind == 1) {
      cbp = i16_cbp;
    } else {
      const uint16_t ca = nb_cbp_left(), cb = nb_cbp_top();
      int c = 0;
      c |= bin(SE_OTHER, 0, 73 + !(ca & 0x02) + 2 * !(cb & 0x04));
      c |= bin(SE_OTHER, 0, 73 + !(c & 0x01) + 2 * !(cb & 0x08)) << 1;
      c |= bin(SE_OTHER, 0, 73 + !(ca & 0x08) + 2 * !(c & 0x01)) << 2;
      c |= bin(SE_OTHER, 0, 73 + !(c & 0x04) + 2 * !(c & 0x02)) << 3;
      if (cat_ == 1 || cat_ == 2) {
        const int a = (ca >> 4) & 3, b = (cb >> 4) & 3;
        if (bin(SE_OTHER, 0, 77 + (a > 0) + 2 * (b > 0)))
          c |= (1 + bin(SE_OTHER, 0, 77 + 4 + (a == 2) + 2 * (b == 2))) << 4;
      }
      cbp = c;
      if ((cbp & 15) && t8mode && !intra && no_sub_lt8x8 && (!direct16 || d8x8inf)) {
        if (bin(SE_OTHER, 0, 399 + (left_ok && (lf & F_T8)) + (top_ok && (tf & F_T8))))
          cf |= F_T8;
      }
    }
    cf |= (uint32_t)cbp << 16;
    if ((cbp & 0x3f) || (intra && kind == 1)) {
      int ctx = last_dqp_nz ? 1 : 0, val = 0;
      while (bin(SE_QPDELTA, val, 60 + ctx)) {
        ctx = ctx < 2 ? 2 : 3;
        if (++val > 102) { err = AVR_SLICE_BAD_QP_DELTA; return; }
      }
      last_dqp_nz = val != 0;
      SPROF_END(6, ps6);
      residual(intra && kind == 1, cbp);
    } else {
      last_dqp_nz = 0;
      SPROF_END(6, ps6);
    }
  }
};

// ---------------------------------------------------------------------------------------
template <int MODE, bool RM, bool FLD, bool P32, bool SPL>
AVR_FI void init_slice_state(Walker<MODE, RM, FLD, P32, SPL>& w, const EngineTables* T) {
  const int lane = threadIdx.x, nt = blockDim.x;  // every wave of the workgroup takes part
  const avr_slice_desc* d = w.d;
  // cabac contexts: 9.3.1.1
  const int tbl = d->slice_type == 2 ? 0 : 1 + d->cabac_init_idc;
  const int qp = d->slice_qp < 0 ? 0 : d->slice_qp > 51 ? 51 : d->slice_qp;
  const SeamRec* seam = nullptr;
  if constexpr (SPL) seam = w.seam;
  if (seam) {   // a piece after a cut: the contexts as they stood there
    const uint32_t* s32 = (const uint32_t*)seam->state;
    uint32_t* st32 = (uint32_t*)w.sh->state;
    for (int i = lane; i < 256; i += nt) st32[i] = s32[i];
  }
  for (int i = seam ? 1024 : lane; i < 1024; i += nt) {
    int m = T->mn[tbl][i][0], n = T->mn[tbl][i][1];
    int pre = ((m * qp) >> 4) + n;
    pre = pre < 1 ? 1 : pre > 126 ? 126 : pre;
    uint8_t s = pre <= 63 ? (uint8_t)((63 - pre) << 1) : (uint8_t)(((pre - 64) << 1) | 1);
    w.sh->state[i] = s;
    if (MODE == MODE_GENERATE) {
      // P(bin = 1) of the initial state: p_LPS = 0.5 * alpha^pStateIdx
      uint32_t plps = T->gen_plps[s >> 1];
      w.sh->gen_p[i] = (uint16_t)((s & 1) ? 65536 - plps : plps);
    }
  }
  if (!RM) {
    for (int i = lane; i < kEstDefault + 2; i += nt) w.sh->est[i] = 0;
    if (MODE != MODE_GENERATE)
      for (int i = lane; i < kEtabSize + 64; i += nt) w.sh->etab[i] = 0;
  }
  uint32_t* ring32 = (uint32_t*)w.ring;
  // MBAFF: the pair edges and records too (walk_slice refuses the slice when they do not fit).  The
  // progressive model row needs no clear: a column's model bytes are read only under a decoded
  // upper macroblock of this slice (top_ok), which wrote them.
  const int cols = (FLD && d->structure == AVR_STRUCT_MBAFF && (int)w.ring_cols >= 3 * w.W + 7) ? 3 * w.W + 7 : w.W;
  if (seam) {   // the upper row's edges from the cut, and a model row of zeros (a fresh model sees none)
    const uint32_t* e32 = (const uint32_t*)(seam + 1);
    for (int i = lane; i < w.W * kEdgeBytes / 4; i += nt) ring32[i] = i % 10 ? e32[i] : e32[i] & ~kEdgeMringNz;
    if (!w.mring_global)
      for (int i = lane; i < w.W * kMringDwords; i += nt) w.mring[i] = 0;
  } else {
    for (int i = lane; i < cols * (int)sizeof(typename Walker<MODE, RM, FLD, P32, SPL>::ERec) / 4; i += nt) ring32[i] = 0;
  }
  if (lane < 2) {
    w.sh->fifo_head[lane] = 0;
    w.sh->fifo_tail[lane] = 0;
  }
  __syncthreads();
}

template <int MODE, bool RM, bool FLD, bool P32, bool SPL>
AVR_FI void walk_slice(Walker<MODE, RM, FLD, P32, SPL>& w) {
  const avr_slice_desc* d = w.d;
  w.W = d->mb_width;
  // a field picture is a picture of half the frame's rows (d->mb_height is the frame's)
  w.H = (FLD && w.fld_pic) ? d->mb_height >> 1 : d->mb_height;
  w.slice_type = d->slice_type;
  w.is_b = d->slice_type == 1;
  w.cat_ = d->chroma_array_type;
  w.t8mode = d->transform_8x8_mode;
  w.nref0 = d->num_ref_idx_l0;   // descriptor fields used while parsing: kept in registers
  w.nref1 = d->num_ref_idx_l1;
  w.d8x8inf = d->direct_8x8_inference;
  w.x264_build = d->x264_build;
  w.first_mb = d->first_mb;
  w.last_dqp_nz = 0;
  if constexpr (SPL) {
    if (w.seam) w.last_dqp_nz = (int)w.seam->last_dqp_nz;
  }
  w.err = 0;
  w.finished = 0;
  w.bins = 0;
  w.mbs_done = 0;
  int addr = d->first_mb;
  const int lane = threadIdx.x;
  const int npic = w.W * w.H;
  w.mb_x = addr % w.W;   // then stepped: no integer division per macroblock
  w.mb_y = addr / w.W;
  w.ystep = (FLD && w.fld_pic) ? 2 : 1;
  w.my = w.mb_y * w.ystep + (d->structure == AVR_STRUCT_BOTTOM_FIELD ? 1 : 0);
  w.mbaff = FLD && d->structure == AVR_STRUCT_MBAFF;
  w.pst = 0;
  if ((FLD && w.mbaff)) {   // pairs in raster order: mb_y = pair row, my = 2 mb_y + bottom
    if ((int)w.ring_cols < 3 * w.W + 7 || (addr & 1)) { w.err = AVR_SLICE_MBAFF_RING; return; }
    w.mb_x = (addr >> 1) % w.W;
    w.mb_y = (addr >> 1) / w.W;
    w.ystep = 2;
    w.my = 2 * w.mb_y;
  }
  {
    const int j = lane, ph_c = (w.cat_ == 2 || w.cat_ == 3) ? 4 : 2;
    int src = 0;
    if (j >= 1 && j < 4) src = 1 + (j - 1) * 4 + (j == 1 ? 3 : ph_c - 1);   // nnz: bottom row of plane j - 1
    else if (j >= 4 && j < 8) src = 13 + ((j - 4) >> 1) * 8 + 6 + ((j - 4) & 1);   // mvd[l][12..15]
    else if (j == 8) src = 29;                       // ref[0][2..3] (| ref[1][2..3] from dword 30)
    else if (j == 9) src = 31;                       // direct8[2..3]
    else if (j >= 10 && j < 23) src = 32 + (j - 10); // mnnz[52]
    w.edge_src = (uint32_t)src;
  }
  for (;;) {
    if (addr >= npic) { w.err = AVR_SLICE_BAD_MB_ADDR; break; }
    if constexpr (SPL && MODE == MODE_COMPRESS) {
      if (w.snap && w.mb_x == 0 && w.mbs_done > 0) w.seam_cut(addr);
    }
    PROF_BEGINW(ps0);
    if (!(FLD && w.mbaff)) {
      w.left_ok = w.mb_x > 0 && addr - 1 >= w.first_mb;
      // the upper neighbour's flags + cbp: the first dword of its edge record
      w.tf = *(const uint32_t*)&w.ring[w.mb_x];
      w.top_ok = (w.tf & F_DEC) != 0;
    } else if (!(w.pst & Walker<MODE, RM, FLD, P32, SPL>::PST_BOT)) {
      w.mbaff_pair_start();
    }
    w.cf = 0;
    // clear the current record (one dword per lane; ref[2][4] = dwords 29-30 to -1)
    {
      uint32_t* c32 = (uint32_t*)&w.sh->cur;
      if (lane < (int)sizeof(MbRec) / 4) c32[lane] = (lane == 29 || lane == 30) ? 0xffffffffu : 0u;
      wave_sync();
    }
    SPROF_ENDW(0, ps0);
#ifdef AVR_PROFILE
    w.sprofb[0]++;   // sub-section 0 counts macroblocks
#endif
    PROF_BEGINW(t1);
    w.decode_mb();
    PROF_ENDW(1, t1);
    PROF_BEGINW(t7);
    if (w.err) break;
    w.cf |= F_DEC;
    w.mbs_done++;
    w.last_mb = addr + 1 >= npic;
    // publish: bottom edge to the ring, full record to `left`, model bytes to the frame (RM) --
    // two lane-parallel LDS reads of the record (whole, and the edge's dwords), then the stores
    wave_sync();
    {
      const uint32_t* c32 = (const uint32_t*)&w.sh->cur;
      const uint32_t v = c32[lane < 45 ? lane : 44];
      const uint32_t ve = c32[w.edge_src], ref1 = c32[30];
      const uint32_t ev = lane == 8 ? (ve >> 16) | (ref1 & 0xffff0000u) : lane == 9 ? ve >> 16 : ve;
      if (!(FLD && w.mbaff)) {
        uint32_t* l32 = (uint32_t*)&w.sh->left;
        if (lane < 45) l32[lane] = v;
        uint32_t* e32 = (uint32_t*)&w.ring[w.mb_x];
        if constexpr (FLD) {
          if (lane < 23) e32[lane] = lane == 0 ? (w.cf & 0xffff017fu) : ev;   // dword 0: flags, pad, cbp
        } else {
          // a model row in global scratch: a column whose kept model bytes are all zero (a skipped or
          // residual-free bottom row) is not stored; bit 9 of the edge's dword 0 (EdgeCore::pad)
          // says which, and the lookups under it read zero without a load (4K P-slices: most rows)
          const bool mz = !RM && w.mring_global &&
                          __ballot(lane >= 10 && lane < 23 && ((kMringUsed >> (lane - 10)) & 1) && ev != 0) != 0;
          if (lane < 10) e32[lane] = lane == 0 ? ((w.cf & 0xffff017fu) | (mz ? kEdgeMringNz : 0u)) : ev;
          else if (!RM && lane < 23 && ((kMringUsed >> (lane - 10)) & 1)) {   // the model row (RM reads the frame)
            const uint32_t at = (uint32_t)w.mb_x * kMringDwords + mring_dword((uint32_t)lane - 10);
            if (w.mring_global) {
              if (mz) ((__attribute__((address_space(1))) uint32_t*)w.mring)[at] = ev;
            } else {
              ((__attribute__((address_space(3))) uint32_t*)w.mring)[at] = ev;
            }
          }
        }
        w.lf = w.cf;
      } else {   // the pair edge of this macroblock; the pair's records move left after its bottom
        const int bot = (w.pst & Walker<MODE, RM, FLD, P32, SPL>::PST_BOT) != 0;
        uint32_t* e32 = (uint32_t*)&w.pair_edge(bot)[w.mb_x];
        if (lane < 23) e32[lane] = lane == 0 ? (w.cf & 0xffff017fu) : ev;
        uint32_t* pr = (uint32_t*)w.pair_rec();
        const uint32_t t = pr[lane < 45 ? lane : 44];
        if (!bot) {
          if (lane < 45) pr[lane] = lane == 0 ? w.cf : v;
        } else if (lane < 45) {
          pr[45 + lane] = t;
          pr[90 + lane] = lane == 0 ? w.cf : v;
        }
      }
      if (RM) {   // MbRec dwords 32-44 are the 52 model bytes
        uint32_t* f32 = (uint32_t*)(w.frames + w.cur_off + ((int64_t)w.mrow() * w.W + w.mb_x) * 52);
        if (lane >= 32 && lane < 45) f32[lane - 32] = v;
      }
      wave_sync();
    }
    PROF_ENDW(7, t7);
    PROF_BEGINW(ps7);
    if (MODE == MODE_COMPRESS || MODE == MODE_DECOMPRESS) {
      w.publish();
      if (!RM) w.update_prio();
      QTRACE(4, (uint32_t)w.mbs_done);
    }
    // MBAFF: end_of_slice_flag follows the bottom macroblock of a pair only (7.3.4)
    const int eos = (!(FLD && w.mbaff) || (w.pst & Walker<MODE, RM, FLD, P32, SPL>::PST_BOT)) ? w.terminate(SE_EOS) : 0;
    SPROF_ENDW(7, ps7);
    if (eos) break;
    if constexpr (SPL) {   // the piece ends at the next cut (its last macroblock's end_of_slice_flag was 0)
      if (w.piece_mbs && (uint32_t)w.mbs_done >= w.piece_mbs) {
        w.finished = 1;
        w.cut = 1;
        break;
      }
    }
    if (Walker<MODE, RM, FLD, P32, SPL>::DEC && w.in.limit && w.cd.next > w.in.limit + 8) { w.err = AVR_SLICE_OVERREAD; break; }
    // a parallel-model decoder reads at most 8 bytes past its stream (the recoded decoder's 63-bit
    // window; P32: 4): a damaged stream is stopped within a macroblock of running off its end
    if (MODE == MODE_DECOMPRESS && !RM && w.in.limit && w.rd.next > w.in.limit + 16) { w.err = AVR_SLICE_OVERREAD; break; }
    addr++;
    if ((FLD && w.mbaff) && !(w.pst & Walker<MODE, RM, FLD, P32, SPL>::PST_BOT)) {
      w.pst |= Walker<MODE, RM, FLD, P32, SPL>::PST_BOT;
      w.my++;
      continue;
    }
    if ((FLD && w.mbaff)) {
      w.pst = 0;
      w.my--;
    }
    if (++w.mb_x == w.W) {
      w.mb_x = 0;
      w.mb_y++;
      if (FLD) w.my += w.ystep;
    }
  }
}

// Run f on the walker instantiation of the slice's structure: w itself for a progressive frame,
// a field-capable copy (FLD = true, set up from w) for field pictures and MBAFF frames.
// --------------------------------------------------------------------------- kernel bodies
template <int MODE, bool RM, bool FLD, bool P32, bool SPL>
AVR_FI void begin_slice(Walker<MODE, RM, FLD, P32, SPL>& w, const avr_slice_desc* d, const uint8_t* in, uint8_t* out) {
  w.d = d;
  w.in.g = in + d->payload_offset;
  w.in.limit = MODE == MODE_GENERATE ? 0 : d->read_limit;
  w.in.lds = w.sh->in_stage;
  w.in.win = 0xffffffffu - kStage;  // force a fill on first use
  w.out.g = out + d->out_offset;
  w.out.cap = d->out_capacity;
  w.out.n = 0;
  w.out.last = 0;
  w.ring0.init(w.sh, 0);
  vtab_load(w.vt, w.T);
  w.rc_cat = -1;
  w.rc_v = 0;
  w.fld_pic = FLD && (d->structure == AVR_STRUCT_TOP_FIELD || d->structure == AVR_STRUCT_BOTTOM_FIELD);
  w.fld = -1;
  // the progressive kernels never run a field slice: their LDS tables are the frame ones
  if (FLD) w.set_fld(w.fld_pic);
  else w.sig8_v = w.T->sig8x8[__lane_id()];
  w.top_pending = 0;
  w.last8_v = w.T->last8x8[__lane_id()];
  if (MODE == MODE_DECOMPRESS) w.byp_e = w.sh->est[1024];
  w.mc_load();
  if (!RM && (MODE == MODE_COMPRESS || MODE == MODE_DECOMPRESS)) {
    if (w.prio_cell == kNoCell) w.prio_cell = cu_cell();
    w.prio_cur = 0xffffffffu;   // set on the first macroblock
  }
  if (MODE == MODE_COMPRESS || MODE == MODE_TRACE) {
    cd_init(w.cd, w.in);
    if constexpr (SPL) {
      if (w.seam) {   // a piece after a cut: the decoder where the cut left it
        w.cd.low = w.seam->cd_low;
        w.cd.range = w.seam->cd_range;
        w.cd.k = (int)w.seam->cd_k;
        w.cd.next = w.seam->cd_next;
      }
    }
  } else if (MODE == MODE_DECOMPRESS) {
    rd_init(w.rd, w.in);
  } else {
    ce_init(w.ce);
    w.rng = d->payload_offset * 0x9E3779B97F4A7C15ull + 0x1234567ull + (uint64_t)d->picture_id;
    w.target_mbs = d->payload_size ? (int)d->payload_size : 1 << 30;
  }
#ifdef AVR_PROFILE
  for (int i = 0; i < 8; i++) w.prof[i] = 0, w.profb[i] = 0, w.sprof[i] = 0, w.sprofb[i] = 0;
#endif
}

template <int MODE, bool RM, bool FLD, bool P32, bool SPL>
AVR_FI void profile_slice(Walker<MODE, RM, FLD, P32, SPL>& w) {
#ifdef AVR_PROFILE
  w.bins = 0;
  const uint64_t t0 = PROF_T();
  const uint32_t t0_b = 0;
  walk_slice(w);
  PROF_ENDW(0, t0);
  if (__lane_id() == 0) {
    for (int i = 0; i < 8; i++) {
      atomicAdd(&avr_prof[i], (unsigned long long)w.prof[i]);
      atomicAdd(&avr_prof[8 + i], (unsigned long long)w.profb[i]);
      atomicAdd(&avr_prof[32 + i], (unsigned long long)w.sprof[i]);
      atomicAdd(&avr_prof[40 + i], (unsigned long long)w.sprofb[i]);
    }
  }
#else
  walk_slice(w);
#endif
}

// The walker wave of a pipelined slice: parse + model, one op per bin into the ring, OP_END at
// the end whatever happened.  Leaves its status in LDS for finish_slice.
template <int MODE, bool RM, bool FLD, bool P32, bool SPL>
AVR_FI void walker_slice(Walker<MODE, RM, FLD, P32, SPL>& w, const avr_slice_desc* d, const uint8_t* in, avr_slice_result* res) {
  begin_slice(w, d, in, nullptr);
  profile_slice(w);
  if constexpr (SPL) {
    if (MODE == MODE_COMPRESS && w.snap && __lane_id() == 0) *w.snap_count = w.snap_n;
  }
  if (!RM) cu_post(w.prio_cell, 0);   // leave the CU board
  w.rc_writeback();  // estimators persist across slices in the reference model
  w.mc_store();
  if (MODE == MODE_DECOMPRESS && __lane_id() == 0) w.sh->est[1024] = (uint16_t)w.byp_e;
  w.push(OP_END);
#ifdef AVR_PROFILE
  if (__lane_id() == 0) atomicAdd(&avr_prof[16], (unsigned long long)w.ring0.wait_cycles);
#endif
  w.publish();
  int status = w.err;
  if (!status && !w.finished) status = AVR_SLICE_NO_END;
  bool cut = false;
  if constexpr (SPL) {
    cut = w.cut;
    if (!status && w.piece_mbs && !cut) status = AVR_SLICE_NO_END;   // end_of_slice inside a non-last piece
  }
  int stop_ok = 1;
  if (MODE == MODE_COMPRESS && !status && !cut) {
    // predicted decompressor output (recode.cpp:1345-1356, 1503-1505): the regenerated CABAC
    // bytes equal the payload through the stop bit, then zero bits
    const uint32_t sbi = cd_bitpos(w.cd) - 1;
    const uint32_t k = sbi >> 3, size = d->payload_size;
    const uint32_t b = in_byte(w.in, k);
    const uint32_t masked = b & (0xffu << (7 - (sbi & 7))) & 0xff;
    if (masked == 0x80) stop_ok = (k == size) || (k + 1 == size);
    else stop_ok = (k + 1 == size) || (k + 2 == size && b == masked);
  }
  if (__lane_id() == 0) {
    w.sh->p_status = status;
    w.sh->p_stop_ok = stop_ok;
    res->bins = w.bins;
    res->mbs = (uint32_t)w.mbs_done;
  }
}

AVR_FI uint32_t vgpr_zero() {
  uint32_t z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}
// The modeler wave (compress): the estimator recurrences (recode.cpp:816-820, 1030-1047),
// lane-parallel over each batch of ring-0 ops (lane j = op j):
//  1. every lane loads its op's estimator at once: per-context ones from Shared::est, SIG/NZ
//     ones by probing the first four slots of the key's window in the LDS hash table; keys not
//     resolved there (new keys, deep or HBM-resident ones) go through est_load one key at a time,
//     a new key claiming its slot immediately;
//  2. a scalar loop walks the batch key by key (ballot of equal keys) and, within a key, op by op
//     in order: the recurrence runs in a scalar register and each op's estimator before its update
//     goes into its lane of the output vector -- no memory access on this chain;
//  3. the last op of each key writes the estimator back (lane-parallel), and the whole batch
//     goes to ring 1 as one vector store.
// Ops of one key stay in order, different keys are independent, so this equals processing the
// ops one by one.
// lane L of v := x (x, L wave-uniform)
AVR_FI uint32_t writelane(uint32_t v, uint32_t L, uint32_t x) { return __lane_id() == L ? x : v; }
// SPL: a batch that holds OP_RESTART (the walker's cut, the batch's last op) ends with a fresh model:
// the HBM table's logged entries, the LDS hash and the per-context estimators cleared
template <bool SPL = false>
AVR_FI void model_slice(Shared* sh, uint16_t* est_g) {
  uint32_t tail = 0, head1 = 0, tail1 = 0;
  uint64_t waited = 0;
  uint32_t prio = 0;
  const uint32_t lane = __lane_id();
#ifdef AVR_PROFILE
  uint64_t out_wait = 0;
  const uint64_t t_start = PROF_T();
#endif
  for (bool done = false; !done;) {
    uint32_t op_v;
    const uint32_t n = ring_take(sh, 0, tail, &op_v, &waited);
    follow_prio(sh, &prio);
    asm volatile("; MARK_MODEL_BEGIN");
    const bool live = lane < n;
    const bool ctrl = (op_v & (OP_END | OP_FINISH)) != 0;
    const bool est_op = live && !ctrl;
    if (__ballot(live && (op_v & OP_END))) done = true;
    const uint32_t idx = (op_v >> 3) & 0x7ffffu;
    const bool cache = (op_v & OPM_CACHE) != 0;
    // ---- 1. loads
    uint32_t e_v = 0, slot_v = 0;
    bool resolved = true;
    if (est_op && !cache) e_v = sh->est[idx];
    if (est_op && cache) resolved = est_probe4(sh, idx, &e_v, &slot_v);
    // keys the short probe did not find: one at a time through the wave-wide probe
    uint64_t slow = __ballot(est_op && !resolved);
    while (slow) {
      const uint32_t l = (uint32_t)__builtin_ctzll(slow);
      const uint32_t idx_l = __builtin_amdgcn_readlane(idx, l);
      uint32_t slot;
      const uint32_t e = est_load(sh, est_g, idx_l, &slot);
      if (slot >> 31) {
        if (lane == 0) sh->etab[slot & 0xffff] = (slot & 0xffff0000u) | e;   // claim / keep the slot
        wave_sync();
      }
      const uint64_t same = __ballot(est_op && cache && idx == idx_l);
      if ((same >> lane) & 1) { e_v = e; slot_v = slot; }
      slow &= ~same;
    }
    // ---- 2. the recurrences, key by key, ops in order
    const uint32_t key_v = (op_v >> 1) & 0xfffffdu;            // cache bit + index (bin, threshold excluded)
    const uint64_t bins_m = __ballot(op_v & 1), thr_m = __ballot(op_v & OPM_THR50);
    // billing class of op j: significance map (threshold 0x50), nnz bits (the other SIG/NZ
    // estimators), or anything else
    const uint64_t nz_m = __ballot(cache && !(op_v & OPM_THR50));
    auto cls_of = [&](uint32_t j) -> uint32_t { return ((thr_m >> j) & 1) ? 1u : ((nz_m >> j) & 1) ? 2u : 0u; };
    uint32_t out_v = op_v;                                     // control ops pass through
    uint32_t fin_v = 0;
    uint64_t last_m = 0;
    uint64_t todo = __ballot(est_op);
    while (todo) {
      const uint32_t l = (uint32_t)__builtin_ctzll(todo);
      const uint32_t k = __builtin_amdgcn_readlane(key_v, l);
      uint64_t m = __ballot(key_v == k) & todo;
      todo &= ~m;
      uint32_t e = __builtin_amdgcn_readlane(e_v, l);
      uint32_t j = l;
      for (;;) {
        const uint32_t b = (uint32_t)(bins_m >> j) & 1u;
        out_v = writelane(out_v, j, op_recode((int)b, e) | cls_of(j) << OPC_SHIFT_C);
        e = est_update(e, (int)b, ((thr_m >> j) & 1) ? 0x50u : 0x60u);
        m &= m - 1;
        if (!m) break;
        j = (uint32_t)__builtin_ctzll(m);
      }
      fin_v = writelane(fin_v, j, e);
      last_m |= 1ull << j;
    }
    // ---- 3. write-back by the last op of each key
    const bool is_last = (last_m >> lane) & 1;
    if (is_last && !cache) sh->est[idx] = (uint16_t)fin_v;
    if (is_last && cache && (slot_v >> 31)) sh->etab[slot_v & 0xffff] = (slot_v & 0xffff0000u) | fin_v;
    const bool hbm = is_last && cache && !(slot_v >> 31);
    if (__ballot(hbm)) {
      if (hbm) est_g[idx] = (uint16_t)(fin_v | kEstWritten);
      const uint64_t first = __ballot(hbm && slot_v == 1);
      if (first) {   // append first stores to the table's write log (est_store)
        const uint32_t base = __builtin_amdgcn_readfirstlane(sh->elog_n);
        const uint32_t cnt = (uint32_t)__builtin_popcountll(first);
        const uint32_t pos = base + (uint32_t)__builtin_popcountll(first & ((1ull << lane) - 1));
        uint32_t* lg = (uint32_t*)(est_g + kEstLog);
        if (((first >> lane) & 1) && pos < (uint32_t)kEstLogCap) lg[pos] = idx;
        if (lane == 0) {
          sh->elog_n = base + cnt;
          *(uint32_t*)(est_g + kEstLogN) = base + cnt <= (uint32_t)kEstLogCap ? base + cnt : kEstLogOverflow;
        }
      }
    }
    asm volatile("; MARK_MODEL_END");
    // ---- the batch to ring 1 (room for n entries), then retire it from ring 0
    if (head1 + n - tail1 > (uint32_t)kFifo) {
#ifdef AVR_PROFILE
      const uint64_t tw = PROF_T();
#endif
      WD_T0;
      for (;;) {
        tail1 = ld_volatile(&sh->fifo_tail[1]);
        if (head1 + n - tail1 <= (uint32_t)kFifo) break;
        WD_POLL(WD_ROOM1, head1, tail1, sh->qnext);
        __builtin_amdgcn_s_sleep(1);
      }
#ifdef AVR_PROFILE
      out_wait += PROF_T() - tw;
#endif
    }
    if (live) sh->fifo[1][(head1 + lane) & (kFifo - 1)] = out_v;
    head1 += n;
    st_volatile(&sh->fifo_head[1], head1);
    if constexpr (SPL) {
      if (__ballot(live && (op_v & OP_RESTART))) {
        const uint32_t nl = *(volatile uint32_t*)(est_g + kEstLogN);
        if (nl == kEstLogOverflow) {
          uint4* e4 = (uint4*)est_g;
          for (uint32_t i = lane; i < (uint32_t)kEstTable / 8; i += 64) e4[i] = make_uint4(0, 0, 0, 0);
        } else {
          const uint32_t* lg = (const uint32_t*)(est_g + kEstLog);
          for (uint32_t i = lane; i < nl; i += 64) est_g[lg[i]] = 0;
        }
        if (lane == 0) {
          *(uint32_t*)(est_g + kEstLogN) = 0;
          sh->elog_n = 0;
        }
        for (uint32_t i = lane; i < (uint32_t)kEstDefault + 2; i += 64) sh->est[i] = 0;
        for (uint32_t i = lane; i < (uint32_t)kEtabSize + 64; i += 64) sh->etab[i] = 0;
        __threadfence_block();
        wave_sync();
      }
    }
    tail += n;
    ring_retire(sh, 0, tail);
  }
#ifdef AVR_PROFILE
  if (__lane_id() == 0) {
    atomicAdd(&avr_prof[17], (unsigned long long)waited);
    atomicAdd(&avr_prof[18], (unsigned long long)out_wait);
    atomicAdd(&avr_prof[20], (unsigned long long)(PROF_T() - t_start));
  }
#endif
}

// The coder wave: compress retires ring 1 (arithmetic_code<uint64_t,uint8_t>::encoder::put /
// finish, recode.cpp:1074, 1092-1094), gathering each op's reciprocal record with its lane;
// decompress retires ring 0 (cabac::encoder::put / put_bypass / put_terminate,
// recode.cpp:1443-1474, cabac_code.h:33-67).
// SEQ: the reference model's per-file kernels (one slice chain per CU, where the coder can hold the
// walker up): the level / mvd prefixes on one context with the state in a register, and the map
// loops unswitched by block kind.  The slice batch keeps the plain loops (measured: the variants
// cost the batch 0.3-0.8 % and gain R-mode 1-2 %, profiles/r04o_coder2_ab.log, r04q_crunmvd_ab.log).
// SPL (decompress): a piece after a cut starts the re-encoder from the seam record; a piece that ends
// at a cut (seam_end) writes its pending bytes out at the end instead of a flush (the oracle's
// avr_ce_seam_flush): the bytes of the arithmetic's low up to the next piece's first byte
// SPL (compress): every OP_FINISH ends a piece's stream -- its length goes to piece_end[k] and a fresh
// encoder starts the next piece's
template <int MODE, bool P32, bool SEQ = false, bool SPL = false>
AVR_FI void coder_slice(Shared* sh, const HotTables* T, const avr_slice_desc* d, uint8_t* out, uint32_t flags,
                        const SeamRec* seam = nullptr, bool seam_end = false, uint32_t* piece_end = nullptr) {
  uint32_t pieces = 0;
  const bool billing = (flags & kFlagBill) != 0;
  uint32_t bill[6] = {0, 0, 0, 0, 0, 0};
  uint32_t bill_pend = 0;
  CabacBill cbill;
  cb_init(cbill);
  OutStream o;
  o.g = out + d->out_offset;
  o.cap = d->out_capacity;
  o.n = 0;
  o.last = 0;
  typename std::conditional<P32, PEncoder, RecodedEncoder>::type re;   // see Walker::rd
  CabacEncoder ce;
  VTab vt;
  if (MODE == MODE_COMPRESS) {
    re_init(re);
    // Keep the coder's interval in VGPRs: every wave of the CU shares one scalar unit, and the
    // walker wave (the critical path) is scalar-bound; 64-bit multiply-adds are also cheaper on
    // the vector unit (v_mad_u64_u32).  A value the compiler cannot prove uniform stays vector.
#ifndef AVR_CODER_SALU
    const uint32_t z = vgpr_zero();
    re.range += z;
    re.low += z;
#endif
  } else {
    ce_init(ce);
    if constexpr (SPL) {
      if (seam) {
        ce.low = seam->ce_low;
        ce.range = seam->ce_range;
        ce.queue = seam->ce_queue;
        ce.outstanding = seam->ce_outstanding;
        ce.cache = seam->ce_cache;
        ce.have_cache = 1;
      }
    }
    vtab_load(vt, T);
  }
  const int r = MODE == MODE_COMPRESS ? 1 : 0;
  uint32_t gt1 = 0, eq1 = 0;   // decompress: level counters of the block in progress (op_level)
  uint32_t mpos = 0;           // decompress: first position of the next op_map segment
  const uint32_t numc = d->chroma_array_type == 2 ? 2u : 1u;   // chroma DC: NumC8x8
  uint32_t tail = 0;
  uint64_t waited = 0;
#ifdef AVR_PROFILE
  const uint64_t t_start = PROF_T();
#endif
  uint32_t prio = 0;
  for (bool done = false; !done;) {
    uint32_t op_v;
    const uint32_t n = ring_take(sh, r, tail, &op_v, &waited);
    follow_prio(sh, &prio);
    if (MODE == MODE_COMPRESS) {
      const uint32_t tot_v = (op_v >> 8) & 127;
      const uint64_t m_v = !P32 ? T->div[tot_v][0] : T->rcp32[tot_v];
      const uint32_t s_v = !P32 ? (uint32_t)T->div[tot_v][1] : 0u;
      // r1 of op j: the reference coder's exact quotient, or the P-format rule (avr_engine.h)
      auto r1_of = [&](uint32_t j, uint32_t op) {
        if constexpr (!P32) {
          const uint64_t m = readlane64(m_v, j);
          const uint32_t shift = __builtin_amdgcn_readlane(s_v, j);
          return (__umul64hi(re.range, m) >> shift) * ((op >> 1) & 127);
        } else {
          return __umulhi(re.range, __builtin_amdgcn_readlane((uint32_t)m_v, j)) * ((op >> 1) & 127);
        }
      };
      asm volatile("; MARK_CODER_BEGIN");
      // control ops (FINISH, END: once per slice) located up front, so the put loop has no checks
      uint64_t ctrl = __ballot(__lane_id() < n && (op_v & (OP_END | OP_FINISH)));
      for (uint32_t j = 0;;) {
        const uint32_t stop = ctrl ? (uint32_t)__builtin_ctzll(ctrl) : n;
        if (billing) {
          for (; j < stop; j++) {
            const uint32_t op = __builtin_amdgcn_readlane(op_v, j);
            const uint32_t bytes = re_put_billed(re, o, op & 1, r1_of(j, op), &bill_pend);
            const int c = op_class_pip_c((op >> OPC_SHIFT_C) & 3);
            if (bytes) bill[c] += bytes;
          }
        } else {
          for (; j < stop; j++) {
            const uint32_t op = __builtin_amdgcn_readlane(op_v, j);
            re_put(re, o, op & 1, r1_of(j, op));
          }
        }
        if (j >= n) break;
        const uint32_t op = __builtin_amdgcn_readlane(op_v, j);
        if (op & OP_END) { done = true; break; }
        re_finish(re, o);
        if constexpr (SPL) {
          if (piece_end && __lane_id() == 0) piece_end[pieces] = out_total(o);
          pieces++;
          re_init(re);
#ifndef AVR_CODER_SALU
          const uint32_t z = vgpr_zero();
          re.range += z;
          re.low += z;
#endif
        }
        ctrl &= ctrl - 1;
        j++;
      }
      asm volatile("; MARK_CODER_END");
    } else {
      // billing: the generic coder's emission counts beside the re-encode, bin by bin
      auto run = [&](auto BILL) {
        constexpr bool bl = decltype(BILL)::value;
        auto put_dec = [&](int b, uint32_t ctx, uint32_t cls) {
          uint8_t* stp = &sh->state[ctx];
          if constexpr (bl) {
            const uint32_t st = *stp;
            const uint32_t bytes = cb_decision(cbill, b, st, vtab_rec(vt, st));
            if (bytes) bill[op_class_pip_d(cls)] += bytes;
          }
          ce_decision_v(ce, o, b, stp, vt);
        };
        // n ones then (if zero) a zero on one context, class 0 (level / mvd prefixes)
        auto put_run = [&](uint32_t ctx, uint32_t n, bool zero) {
          uint8_t* stp = &sh->state[ctx];
          uint32_t st = *stp;
          for (uint32_t k = 0; k < n + (zero ? 1u : 0u); k++) {
            const int b = k < n;
            const CabacRec r = vtab_rec(vt, st);
            if constexpr (bl) {
              const uint32_t bytes = cb_decision(cbill, b, st, r);
              if (bytes) bill[0] += bytes;
            }
            uint32_t ns;
            ce_encode(ce, o, b, st, r, &ns);
            st = ns;
          }
          *stp = (uint8_t)st;
        };
        auto put_byp = [&](int b, uint32_t cls) {
          if constexpr (bl) {
            const uint32_t bytes = cb_bypass(cbill, b);
            if (bytes) bill[op_class_pip_d(cls)] += bytes;
          }
          ce_bypass(ce, o, b);
        };
        for (uint32_t j = 0; j < n; j++) {
          const uint32_t op = __builtin_amdgcn_readlane(op_v, j);
          if (op & OP_END) { done = true; break; }
          const int b = op & 1;
          const uint32_t kind = (op >> 1) & 3;
          const uint32_t cls = (op >> OPC_SHIFT_D) & 3;
          if (kind == OPK_DECISION) {
            put_dec(b, (op >> 3) & 1023, cls);
          } else if (kind == OPK_BYPASS) {
            put_byp(b, cls);
          } else if (kind == OPK_MACRO) {
            const uint32_t sub = (op >> 3) & 3, cat = (op >> 5) & 15;
            if (sub == 0) {   // op_map: significant / last_significant_coeff_flag of one segment
              const uint32_t npos = ((op >> 9) & 15) + 1, ended = (op >> 13) & 1;
              const uint32_t mask = op >> 14, lastq = ended ? npos - 1 : 16u;
              const uint32_t sb = (uint32_t)T->sig_base[cat], lb = (uint32_t)T->last_base[cat];
              // one loop per block kind (K: 0 4x4-class, 1 chroma DC, 2 8x8), as the walker's
              auto seg_loop = [&](auto K) {
                constexpr int k = decltype(K)::value;
                for (uint32_t q = 0; q < npos; q++) {
                  const uint32_t p = mpos + q;
                  uint32_t sc, lc;
                  if constexpr (k == 2) {
                    sc = T->sig8x8[p];
                    lc = T->last8x8[p];
                  } else if constexpr (k == 1) {
                    sc = lc = min(p / numc, 2u);
                  } else {
                    sc = lc = p;
                  }
                  const int sig = (mask >> q) & 1;
                  put_dec(sig, sb + sc, 1);
                  if (sig) put_dec(q == lastq, lb + lc, 2);
                }
              };
              if constexpr (!SEQ) {
                const bool c8 = cat == 5 || cat == 9 || cat == 13;
                for (uint32_t q = 0; q < npos; q++) {
                  const uint32_t p = mpos + q;
                  uint32_t sc, lc;
                  if (c8) {
                    sc = T->sig8x8[p];
                    lc = T->last8x8[p];
                  } else if (cat == 3) {
                    sc = lc = min(p / numc, 2u);
                  } else {
                    sc = lc = p;
                  }
                  const int sig = (mask >> q) & 1;
                  put_dec(sig, sb + sc, 1);
                  if (sig) put_dec(q == lastq, lb + lc, 2);
                }
              } else if (cat == 5 || cat == 9 || cat == 13) {
                seg_loop(std::integral_constant<int, 2>());
              } else if (cat == 3) {
                seg_loop(std::integral_constant<int, 1>());
              } else {
                seg_loop(std::integral_constant<int, 0>());
              }
              if (npos != 16 || ended) {   // the map's last segment: its block's levels follow
                mpos = 0;
                gt1 = eq1 = 0;
              } else {
                mpos += 16;
              }
            } else if (sub == 1) {   // op_level: coeff_abs_level_minus1 prefix (+ sign)
              const uint32_t sg = (op >> 9) & 1, absl = (op >> 10) & 15;
              const uint32_t ab = (uint32_t)T->abs_base[cat];
              put_dec(absl > 1, ab + (gt1 ? 0u : min(4u, 1 + eq1)), 0);
              if (absl > 1) {
                const uint32_t c1 = ab + 5 + min(4u - (cat == 3), gt1);
                if constexpr (SEQ) {
                  put_run(c1, absl - 2, absl < 15);   // one context: its state stays in a register
                } else {
                  for (uint32_t a = 2; a < 15; a++) {
                    const int more = a < absl;
                    put_dec(more, c1, 0);
                    if (!more) break;
                  }
                }
              }
              if (absl < 15) put_byp((int)sg, 0);
              if (absl == 1) eq1++;
              else gt1++;
            } else {   // op_mvd: mvd_lX[][][comp] prefix (+ sign), 9.3.3.1.1.7 / 9.3.3.1.2
              const uint32_t base = (op & 32) ? 47u : 40u, sg = (op >> 8) & 1, am = (op >> 9) & 15;
              put_dec(am > 0, base + ((op >> 6) & 3), 0);
              if (am > 0) {
                // bins m = 1, 2, 3 on contexts base + 3, 4, 5, then m = 4 .. 8 on base + 6
                uint32_t m = 1;
                for (; m < 4; m++) {
                  const int more = m < am;
                  put_dec(more, base + m + 2, 0);
                  if (!more) break;
                }
                if (m == 4) {
                  if constexpr (SEQ) {
                    put_run(base + 6, min(am, 9u) - 4, am < 9);
                  } else {
                    for (; m < 9; m++) {
                      const int more = m < am;
                      put_dec(more, base + 6, 0);
                      if (!more) break;
                    }
                  }
                }
                if (am < 9) put_byp((int)sg, 0);
              }
            }
          } else {
            if constexpr (bl) {
              const uint32_t bytes = cb_terminate(cbill, b);
              if (bytes) bill[op_class_pip_d(cls)] += bytes;
            }
            ce_terminate(ce, o, b);
          }
        }
      };
      if (billing) run(std::true_type());
      else run(std::false_type());
    }
    tail += n;
    ring_retire(sh, r, tail);
  }
#ifdef AVR_PROFILE
  if (__lane_id() == 0) {
    atomicAdd(&avr_prof[19], (unsigned long long)waited);
    atomicAdd(&avr_prof[21], (unsigned long long)(PROF_T() - t_start));
  }
#endif
  if constexpr (SPL) {
    if (MODE == MODE_DECOMPRESS && seam_end) {
      const uint32_t carry = ce.low >> (ce.queue + 18);
      if (ce.have_cache) {
        if (ce.cache + carry > 0xff) ce.err = 1;
        out_byte(o, ce.cache + carry);
      } else if (carry) {
        ce.err = 1;
      }
      if (ce.outstanding) out_repeat(o, (0xff + carry) & 0xff, ce.outstanding);
    }
  }
  if (__lane_id() == 0) {
    sh->c_err = MODE == MODE_COMPRESS ? re.err : ce.err;
    sh->c_len = out_total(o);
    sh->c_last = o.last;
    for (int i = 0; i < 6; i++) sh->bill[i] = bill[i];
  }
}

// Combine the two waves' results (after a workgroup barrier), with run_slice_inline's semantics.
// seam_end: a piece that ends at a cut (its last byte is not the slice's)
template <int MODE>
AVR_FI void finish_slice(const Shared* sh, const avr_slice_desc* d, avr_slice_result* res, bool seam_end = false) {
  int status = sh->p_status;
  if (sh->c_err) status = AVR_SLICE_CODER;
  if (MODE == MODE_COMPRESS && !status && !sh->p_stop_ok) status = AVR_SLICE_NO_STOP;
  uint32_t len = sh->c_len;
  if (len > d->out_capacity) {   // nothing past the capacity was written: report what was
    status = AVR_SLICE_OVERFLOW;
    len = d->out_capacity;
  }
  if (MODE == MODE_DECOMPRESS && !status && len && sh->c_last == 0x80 && !seam_end) len--;  // recode.cpp:1503-1505
  res->out_len = len;
  res->status = status;
  for (int i = 0; i < 6; i++) res->bill[i] = sh->bill[i];
}

// Single-wave slice (the generator: CABAC encode inline, no coder wave).
template <int MODE, bool RM, bool FLD, bool P32, bool SPL>
AVR_FI void run_slice_inline(Walker<MODE, RM, FLD, P32, SPL>& w, const avr_slice_desc* d, const uint8_t* in, uint8_t* out,
                             avr_slice_result* res) {
  begin_slice(w, d, in, out);
  profile_slice(w);
  w.rc_writeback();
  w.mc_store();
  int status = w.err;
  if (!status && !w.finished) status = AVR_SLICE_NO_END;
  if (MODE == MODE_GENERATE && w.ce.err) status = AVR_SLICE_CODER;
  if (out_overflow(w.out)) status = AVR_SLICE_OVERFLOW;
  if (__lane_id() == 0) {
    res->out_len = out_total(w.out);
    res->status = status;
    res->bins = w.bins;
    res->mbs = (uint32_t)w.mbs_done;
    for (int i = 0; i < 6; i++) res->bill[i] = 0;
  }
}

// Copy the per-bin lookup tables into this workgroup's LDS (16 B per thread per step).
AVR_FI void load_hot_tables(Shared* sh, const EngineTables* G) {
  const uint4* src = (const uint4*)&G->hot;
  uint4* dst = (uint4*)&sh->tab;
  for (int i = threadIdx.x; i < (int)(sizeof(HotTables) / 16); i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

// Threads per workgroup: two waves (walker + coder) for compress / decompress, one for generate.
template <int MODE>
constexpr int slice_threads() {
  return MODE == MODE_GENERATE || MODE == MODE_TRACE ? 64 : MODE == MODE_COMPRESS ? 192 : 128;
}

// One slice of a parallel launch on this workgroup (every thread): the hot tables are in LDS
// already; est_g is the slice's estimator scratch; cell = the walker's CU-board cell (kNoCell:
// register one).
// MG: the launch may keep the model row in global scratch (the persistent kernel, which every wide
// launch uses); the resident kernel's row is always in LDS (a constant: no branch at its accesses).
template <int MODE, bool FLD, bool P32, bool MG, bool SPL = false>
AVR_FI void parallel_slice(uint8_t* smem, const EngineTables* G, const avr_slice_desc* descs, int s, const uint8_t* in,
                           uint8_t* out, avr_slice_result* res, uint16_t* est_g, uint32_t flags, uint32_t cell,
                           uint32_t qiter = 0, const SplitArgs* sp = nullptr) {
  const avr_slice_desc* d = &descs[s];
  Walker<MODE, false, FLD, P32, SPL> w;
  w.sh = (Shared*)smem;
  w.ring = (typename Walker<MODE, false, FLD, P32, SPL>::ERec*)(smem + sizeof(Shared));
  bool seam_end = false;
  uint32_t* piece_end = nullptr;
  if constexpr (SPL) {
    const PieceCtl c = sp->ctl[s];
    w.seam = c.seam >= 0 ? (const SeamRec*)(sp->recs + (size_t)c.seam * sp->rec_stride) : nullptr;
    w.piece_mbs = c.n_mbs;
    w.cut = 0;
    seam_end = c.n_mbs != 0;
    piece_end = MODE == MODE_COMPRESS && c.snap >= 0 && sp->piece_end ? sp->piece_end + c.snap : nullptr;
    w.snap = MODE == MODE_COMPRESS && c.snap >= 0 ? sp->recs + (size_t)c.snap * sp->rec_stride : nullptr;
    w.snap_cap = c.snap_cap;
    w.snap_n = 0;
    w.snap_last = 0;
    w.snap_q = 0;
    w.split_bits = sp->split_bits;
    w.rec_stride = sp->rec_stride;
    w.snap_count = sp->snap_n ? sp->snap_n + s : nullptr;
  }
  w.mring_global = MG && !FLD && (flags & kFlagMringGlobal);
  w.mring = w.mring_global ? (uint32_t*)(est_g + kEstMring)
                           : (uint32_t*)(smem + sizeof(Shared) + (size_t)(flags >> kFlagRingShift) * sizeof(EdgeCore));
  w.prio_cell = cell;
  w.T = &w.sh->tab;
  w.G = G;
  w.frames = nullptr;
  w.cur_off = 0;
  w.prev_off = -1;
  w.gmode = false;
  w.gsink = nullptr;
  w.gcount = 0;
  w.est_g = est_g;
  w.ring_cols = flags >> kFlagRingShift;
  if (!d->coded) {
    if (threadIdx.x == 0) {
      res[s].out_len = 0;
      res[s].status = 1;
      res[s].bins = 0;
      res[s].mbs = 0;
      for (int i = 0; i < 6; i++) res[s].bill[i] = 0;
    }
    return;
  }
  // fresh model for this slice: undo the last model's stores to the HBM estimator table
  if (MODE == MODE_COMPRESS || MODE == MODE_DECOMPRESS) est_table_reset(w.est_g, w.sh);
  if (MG) QTRACE(threadIdx.x >> 6, qiter << 8 | 2);
  w.d = d;
  w.W = d->mb_width;
  if ((MODE == MODE_COMPRESS || MODE == MODE_DECOMPRESS) && threadIdx.x == 0) w.sh->prio = 0;   // before init_slice_state's barrier
  init_slice_state(w, G);
  if (MG) QTRACE(threadIdx.x >> 6, qiter << 8 | 3);
  if (MODE == MODE_GENERATE || MODE == MODE_TRACE) {
    run_slice_inline(w, d, in, out, &res[s]);
    return;
  }
  const int wave = threadIdx.x >> 6;
  AVR_PLACE(s, wave);
  if (wave == 0) {
    AVR_PLACE_T(s, 0);
    walker_slice(w, d, in, &res[s]);
    AVR_PLACE_T(s, 1);
  }
  else if (MODE == MODE_COMPRESS && wave == 1) model_slice<SPL>(w.sh, w.est_g);
  else if constexpr (SPL) coder_slice<MODE, P32, false, true>(w.sh, w.T, d, out, flags, w.seam, seam_end, piece_end);
  else coder_slice<MODE, P32>(w.sh, w.T, d, out, flags);
  if (MG) QTRACE(wave, qiter << 8 | 4);
  __syncthreads();
  if (MG) QTRACE(wave, qiter << 8 | 5);
  if (threadIdx.x == 0) finish_slice<MODE>(w.sh, d, &res[s], seam_end);
}

// The long-slice split's launches (avr_kernels.h SplitArgs): progressive frame slices and pieces of
// the parallel model on arithmetic_code<uint64_t, uint8_t>, the model row in LDS; each workgroup
// takes descriptors blockIdx.x, blockIdx.x + gridDim.x, ... (a grid of at most the resident slots:
// one estimator scratch per workgroup).  MODE_TRACE: the cut scan -- the CABAC parse of whole long
// slices (one wave, no model, no output) taking the cut records (PieceCtl::snap).  Compress: the
// pieces (seam >= 0: started from a record, n_mbs > 0: stopped at the next cut).  Decompress: the
// pieces, from records the host wrote (the container's seams).
template <int MODE>
__global__ __launch_bounds__(192, 4) void slices_split_kernel(const EngineTables* G, const avr_slice_desc* descs, int n,
                                                             const uint8_t* in, uint8_t* out, avr_slice_result* res,
                                                             uint16_t* est_scratch, SplitArgs sp, uint32_t flags) {
  extern __shared__ __align__(16) uint8_t smem[];
  uint32_t cell = kNoCell;
  bool loaded = false;
  for (int s = blockIdx.x; s < n; s += gridDim.x) {
    __syncthreads();   // the previous descriptor's finish_slice has read the workgroup's LDS
    if (!loaded) {
      load_hot_tables((Shared*)smem, G);
      loaded = true;
      if (threadIdx.x < 64) cell = cu_cell();
    }
    parallel_slice<MODE, false, false, false, true>(smem, G, descs, s, in, out, res,
                                                    est_scratch + (size_t)blockIdx.x * kEstGlobal, flags, cell, 0, &sp);
  }
}

// FLD = false: the progressive frames of the batch; FLD = true: its field pictures and MBAFF frames
// (a second launch over the same batch: each kernel leaves the other's slices alone).
//
// Two ways to run a batch:
//  - qhead == nullptr: workgroup b runs slice order[b] (the CU grouping of schedule_kernel) or b,
//    with the estimator scratch of that slice -- a batch that is resident all at once;
//  - qhead != nullptr (a batch larger than the chip holds at once): a persistent grid of about one
//    workgroup per resident slot; each workgroup takes the next entry of the queue `order` (the
//    slices sorted largest first, queue_order_kernel) by an atomic on *qhead until the queue is
//    empty, with one estimator scratch per workgroup (est_table_reset undoes the previous slice's
//    stores).  Every workgroup leaves when it draws past the end, so the grid always drains.
//    Largest first is LPT: the batch ends on small slices instead of on a large one started late,
//    and there are no launch boundaries inside the batch to wait at.
template <int MODE, bool FLD, bool P32 = false>
__global__ __launch_bounds__(192, 4) void slices_parallel_kernel(const EngineTables* G, const avr_slice_desc* descs, int n,
                                                                const uint8_t* in, uint8_t* out, avr_slice_result* res,
                                                                uint16_t* est_scratch, const int* order,
                                                                uint32_t flags) {
  extern __shared__ __align__(16) uint8_t smem[];
  if ((int)blockIdx.x >= n) return;
  const int s = order ? order[blockIdx.x] : (int)blockIdx.x;   // CU grouping (schedule_kernel)
  if ((descs[s].structure != AVR_STRUCT_FRAME) != FLD) return;
  load_hot_tables((Shared*)smem, G);
  parallel_slice<MODE, FLD, P32, false>(smem, G, descs, s, in, out, res, est_scratch + (size_t)s * kEstGlobal, flags,
                                        kNoCell);
}

// The persistent variant (a kernel of its own: the loop's state would change the resident
// kernel's register allocation): about one workgroup per resident slot, each taking the next entry
// of the largest-first queue by an atomic on *qhead until the queue is empty.
template <int MODE, bool FLD, bool P32 = false>
__global__ __launch_bounds__(192, 4) void slices_queue_kernel(const EngineTables* G, const avr_slice_desc* descs, int n,
                                                             const uint8_t* in, uint8_t* out, avr_slice_result* res,
                                                             uint16_t* est_scratch, const int* queue, uint32_t* qhead,
                                                             uint32_t flags) {
  extern __shared__ __align__(16) uint8_t smem[];
  Shared* sh = (Shared*)smem;
  // the hot tables and the walker wave's CU-board cell are set up at the first slice this
  // workgroup takes (a field-kernel workgroup that finds no field slice does neither).  The other
  // order (-DAVR_QUEUE_EAGER) hangs the first queue launch of a process in its
  // uninstrumented build only: every instrumented build of it (bounded waits with invariant checks,
  // host-mapped progress records) runs clean and sees no invariant violated, so the hang follows
  // that build's code generation, not an ordering rule of the protocol below.
  uint32_t cell = kNoCell;
  bool loaded = false;
  uint32_t qiter = 0;   // slices this workgroup drew (queue trace builds)
#ifdef AVR_WATCHDOG
  if ((threadIdx.x & 63) == 0) sh->wd_epoch[threadIdx.x >> 6] = 0;
  uint32_t wd_prev_k = 0xffffffffu;
#endif
#ifdef AVR_QUEUE_EAGER   // experiment builds: the round-5 order that hung (r05c: 1, r05e: 2)
  load_hot_tables(sh, G);
  loaded = true;
  if ((MODE == MODE_COMPRESS || MODE == MODE_DECOMPRESS) && threadIdx.x < 64) {
    cell = cu_cell();
#if AVR_QUEUE_EAGER == 1
    if (__lane_id() == 0) *(volatile __attribute__((address_space(3))) uint32_t*)&sh->qcell = cell;
#endif
  }
#endif
  for (;;) {
    if (threadIdx.x == 0) *(volatile __attribute__((address_space(3))) uint32_t*)&sh->qnext = atomicAdd(qhead, 1u);
#ifdef AVR_WATCHDOG
    if ((threadIdx.x & 63) == 0) sh->wd_epoch[threadIdx.x >> 6]++;
#endif
    __syncthreads();
    const uint32_t k = __builtin_amdgcn_readfirstlane(*(volatile __attribute__((address_space(3))) uint32_t*)&sh->qnext);
#ifdef AVR_WATCHDOG
    if (threadIdx.x == 0)
      for (uint32_t v = 1; v < blockDim.x / 64; v++)
        WD_CHECK(sh->wd_epoch[v] == sh->wd_epoch[0], WD_EPOCH, sh->wd_epoch[0], sh->wd_epoch[v], k);
    WD_CHECK(wd_prev_k == 0xffffffffu || k > wd_prev_k, WD_QORDER, wd_prev_k, k, k);
    wd_prev_k = k;
#endif
    __syncthreads();   // every thread has its entry before thread 0 draws again
    if (k >= (uint32_t)n) break;
    const int s = queue[k];
    if ((descs[s].structure != AVR_STRUCT_FRAME) != FLD) continue;
    if (!loaded) {
      load_hot_tables(sh, G);
      loaded = true;
      if ((MODE == MODE_COMPRESS || MODE == MODE_DECOMPRESS) && threadIdx.x < 64) cell = cu_cell();
    }
#if defined(AVR_QUEUE_EAGER) && AVR_QUEUE_EAGER == 1
    cell = __builtin_amdgcn_readfirstlane(*(volatile __attribute__((address_space(3))) uint32_t*)&sh->qcell);
#endif
    WD_CHECK(cell == kNoCell || cell < 4u * kCuIds, WD_CELL, cell, threadIdx.x, k);
#ifdef AVR_QTRACE
    qiter++;
    if (threadIdx.x == 0) QTRACE1(3, k);
    QTRACE(threadIdx.x >> 6, qiter << 8 | 1);
#endif
    parallel_slice<MODE, FLD, P32, true>(smem, G, descs, s, in, out, res, est_scratch + (size_t)blockIdx.x * kEstGlobal,
                                         flags, cell, qiter);
  }
  QTRACE1(threadIdx.x >> 6, qiter << 8 | 6);
}

// Host side of the parallel launches (instantiated in each kernel TU, avr_k_*.hip, with that TU's
// own CU board): the progressive kernel over the batch, then -- when the batch may hold field
// pictures / MBAFF frames -- the field-capable kernel over the same batch (its workgroups for
// progressive slices return at once).  The board starts empty on every launch (cu_cell's slot
// counter must not carry a previous launch's residue).  q.head: the persistent queue launch
// (slices_parallel_kernel) over q.grid workgroups, q.head[0] for the progressive kernel and
// q.head[1] for the field one (both zero on entry).  q.lane (FieldLane): the field kernel runs on a
// stream of its own beside the progressive one, so a mixed batch takes the longer of the two
// kernels instead of their sum.  The two kernels share the board (it ranks the slices of a CU
// whichever kernel walks them; one reset before both) and touch disjoint slices; their persistent
// workgroups take disjoint estimator scratches (the field kernel's after the q.grid progressive ones).
struct QueueLaunch {
  uint32_t* head = nullptr;
  int grid = 0, grid_fld = 0;   // persistent grids of the progressive and the field kernel
  size_t lds_fld = 0;           // LDS of the field kernel (0: the progressive kernel's)
  const FieldLane* lane = nullptr;
};
template <int MODE, bool P32>
inline hipError_t launch_parallel(const EngineTables* T, const avr_slice_desc* descs, int n, size_t lds,
                                  const uint8_t* in, uint8_t* out, avr_slice_result* res, uint16_t* est,
                                  const int* order, uint32_t flags, hipStream_t stream, QueueLaunch q = QueueLaunch()) {
  const size_t lds_fld = q.lds_fld ? q.lds_fld : lds;
  const bool fields = (flags & kFlagFields) != 0;
  const bool side = fields && q.lane && q.lane->stream;
  if (hipError_t e = reset_cu_board(stream); e != hipSuccess) return e;
  hipStream_t fs = stream;
  if (side) {
    fs = q.lane->stream;
    if (hipError_t e = hipEventRecord(q.lane->fork, stream); e != hipSuccess) return e;
    if (hipError_t e = hipStreamWaitEvent(fs, q.lane->fork, 0); e != hipSuccess) return e;
  }
  if (q.head)
    hipLaunchKernelGGL((slices_queue_kernel<MODE, false, P32>), dim3(q.grid), dim3(slice_threads<MODE>()), lds, stream,
                       T, descs, n, in, out, res, est, order, q.head, flags);
  else
    hipLaunchKernelGGL((slices_parallel_kernel<MODE, false, P32>), dim3(n), dim3(slice_threads<MODE>()), lds, stream,
                       T, descs, n, in, out, res, est, order, flags);
  if (fields) {
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    if (!side)
      if (hipError_t e = reset_cu_board(stream); e != hipSuccess) return e;
    // beside the progressive kernel, the persistent field workgroups take the scratches after its grid
    uint16_t* est_f = side && q.head ? est + (size_t)q.grid * kEstGlobal : est;
    if (q.head)
      hipLaunchKernelGGL((slices_queue_kernel<MODE, true, P32>), dim3(q.grid_fld), dim3(slice_threads<MODE>()), lds_fld,
                         fs, T, descs, n, in, out, res, est_f, order, q.head + 1, flags & ~kFlagMringGlobal);
    else
      hipLaunchKernelGGL((slices_parallel_kernel<MODE, true, P32>), dim3(n), dim3(slice_threads<MODE>()), lds_fld,
                         fs, T, descs, n, in, out, res, est_f, order, flags & ~kFlagMringGlobal);
    if (side) {
      if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
      if (hipError_t e = hipEventRecord(q.lane->join, fs); e != hipSuccess) return e;
      if (hipError_t e = hipStreamWaitEvent(stream, q.lane->join, 0); e != hipSuccess) return e;
    }
  }
  return hipGetLastError();
}

// Reference model: one workgroup (walker + coder wave) walks every slice of a file in file order
// with persistent estimators and frame metadata.  Several files at once: workgroup f walks file f,
// the slices [file_first[f], file_first[f + 1]) (file_first == nullptr: one file, all n slices),
// with its own estimator table (est_g + f kEstGlobal), frames (frames + f frame_stride) and
// frame_meta[f] -- files share nothing, as separate runs of the reference would not.
// FLD = true when the files may hold field pictures or MBAFF frames (the field-capable walker
// also walks progressive slices); FLD = false refuses such a slice (status -21)
template <int MODE, bool FLD>
__global__ __launch_bounds__(192) void slices_sequential_kernel(const EngineTables* G, const avr_slice_desc* descs, int n,
                                                                  const uint8_t* in, uint8_t* out,
                                                                  avr_slice_result* res, uint16_t* est_g,
                                                                  uint8_t* frames, int* frame_meta,
                                                                  const int* file_first, uint64_t frame_stride,
                                                                  uint32_t flags) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int file = (int)blockIdx.x;
  const int s_begin = file_first ? file_first[file] : 0;
  const int s_end = file_first ? file_first[file + 1] : n;
  est_g += (size_t)file * kEstGlobal;
  frames += (size_t)file * frame_stride;
  frame_meta += file;
  Walker<MODE, true, FLD> w;
  w.sh = (Shared*)smem;
  w.ring = (typename Walker<MODE, true, FLD>::ERec*)(smem + sizeof(Shared));
  w.mring = nullptr;   // the reference model reads its neighbours' model bytes from the frame
  w.mring_global = false;
  load_hot_tables(w.sh, G);
  w.T = &w.sh->tab;
  w.G = G;
  w.est_g = est_g;
  w.frames = frames;
  w.ring_cols = flags >> kFlagRingShift;
  // fresh global model
  {
    uint4* e4 = (uint4*)est_g;
    for (int i = tid; i < kEstGlobal / 8; i += nt) e4[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0) {
      w.sh->elog_n = 0;
      w.sh->prio = 0;
    }
    for (int i = tid; i < kEstDefault + 2; i += nt) w.sh->est[i] = 0;
    for (int i = tid; i < kEtabSize + 64; i += nt) w.sh->etab[i] = 0;
  }
  // frame_meta: [0] cur_frame.  Frame ids / sizes of the two frames, as scalars (no private arrays).
  int cur = 0, fid0 = 0, fid1 = 0, fw0 = 0, fw1 = 0, fh0 = 0, fh1 = 0;
  __syncthreads();
  for (int s = s_begin; s < s_end; s++) {
    const avr_slice_desc* d = &descs[s];
    const int W = d->mb_width, H = d->mb_height;
    // update_frame_spec (recode.cpp:824-843)
    const int fwc = cur ? fw1 : fw0, fhc = cur ? fh1 : fh0, fidc = cur ? fid1 : fid0;
    if (fwc != W || fhc != H || !(fidc == d->picture_id && fwc && fhc)) {
      cur = 1 - cur;
      const int fwn = cur ? fw1 : fw0, fhn = cur ? fh1 : fh0;   // the new current frame
      const int fwo = cur ? fw0 : fw1, fho = cur ? fh0 : fh1;   // the other one
      const bool reinit_other = (fwn != W || fhn != H) && (fwo != W || fho != H);
      // fresh/cleared current frame; a dimension change also clears the other one
      uint32_t* f32 = (uint32_t*)(frames + (size_t)cur * W * H * 52);
      for (int i = tid; i < W * H * 13; i += nt) f32[i] = 0;
      if (reinit_other) {
        uint32_t* o32 = (uint32_t*)(frames + (size_t)(1 - cur) * W * H * 52);
        for (int i = tid; i < W * H * 13; i += nt) o32[i] = 0;
        if (cur) { fw0 = W; fh0 = H; } else { fw1 = W; fh1 = H; }
      }
      if (cur) { fw1 = W; fh1 = H; fid1 = d->picture_id; } else { fw0 = W; fh0 = H; fid0 = d->picture_id; }
      __threadfence_block();
      __syncthreads();
    }
    if (!d->coded || (!FLD && d->structure != AVR_STRUCT_FRAME)) {
      if (tid == 0) {
        res[s].out_len = 0;
        res[s].status = d->coded ? -21 : 1;
        res[s].bins = 0;
        res[s].mbs = 0;
      for (int i = 0; i < 6; i++) res[s].bill[i] = 0;
      }
      continue;
    }
    w.cur_off = (int64_t)cur * W * H * 52;
    w.prev_off = (int64_t)(1 - cur) * W * H * 52;
    w.gmode = false;
    w.gsink = nullptr;
    w.gcount = 0;
    w.d = d;
    w.W = W;
    init_slice_state(w, G);
    const int wave = tid >> 6;
    if (wave == 0) walker_slice(w, d, in, &res[s]);
    else if (MODE == MODE_COMPRESS && wave == 1) model_slice(w.sh, w.est_g);
    else coder_slice<MODE, false, true>(w.sh, w.T, d, out, flags);
    __syncthreads();
    if (tid == 0) finish_slice<MODE>(w.sh, d, &res[s]);
    __syncthreads();
  }
  if (tid == 0) frame_meta[0] = cur;
}

}  // namespace avr
