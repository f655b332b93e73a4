// Device-side building blocks of the recode path (gfx950).  Included by avr_kernels.hip only.
//
//   CabacDecoder   ITU-T H.264 9.3.3.2 decoding engine (the fork's ff_get_cabac*, called at
//                  recode.cpp:1176-1188), byte-refilled 64-bit window, exact bit position.
//   CabacEncoder   exact re-encoder with the output bytes of cabac_code.h:27-80 (the generic
//                  arithmetic_code<uint32_t,uint16_t,0x200> coder): 9-bit range, carry cache.
//   RecodedEncoder arithmetic_code<uint64_t,uint8_t> encoder (arithmetic_code.h:89-203,
//                  recode.cpp:315-316): same bytes, carry handled with a cache + 0xFF run.
//   RecodedDecoder its decoder (arithmetic_code.h:211-298), 1-bit misaligned byte digits.
//   Estimators     recode.cpp:816-820 / 1030-1047: p1 = (range/(pos+neg))*pos with an exact
//                  per-divisor reciprocal instead of a 64-bit divide.
//
// Every function here runs redundantly on all 64 lanes of the wavefront that owns a slice
// (the values are wave-uniform); only the staging helpers use the lanes cooperatively.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace avr {

constexpr int kStage = 1024;  // bytes per LDS staging window

// The serial state is wave-uniform and lives in SGPRs.  LLVM folds a compare of the high word of
// a 64-bit value back into a 64-bit compare, which the scalar unit lacks (it becomes a VALU
// compare + a VCC round trip); readfirstlane on the high word (free on a uniform value) keeps
// the compare 32-bit scalar.
__device__ __forceinline__ uint32_t opaque_u32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return opaque_u32((uint32_t)(x >> 32)); }

// Tables read on every bin: copied into each workgroup's LDS at kernel start.
struct HotTables {
  uint64_t div[128][2];     // [d] = {m, shift}: floor(n/d) = umulhi(n, m) >> shift for n <= 2^63,
                            //   m = ceil(2^(63+l)/d), l = ceil(log2 d), shift = l - 1 (one 16-B read)
  uint32_t rcp32[128];      // [d] = floor(2^32 / d): the P-format coder's r1 = umulhi(range, rcp32[tot]) * pos
  uint64_t cabac[128];      // [state]: LPS range for q = (range >> 6) & 3 in byte q, successor state
                            //   after an MPS in byte 4, after an LPS in byte 5 (one 8-B read per bin)
  uint8_t nb_left[48];      // get_neighbor_sub_mb: block left of n (| 128 if in the left macroblock)
  uint8_t nb_up[48];        //                      block above n (| 128 if in the upper macroblock)
  uint8_t sig8x8[64];       // significant_coeff_flag ctxIdxInc of 8x8 blocks (frame coded)
  uint8_t last8x8[64];      // last_significant_coeff_flag ctxIdxInc of 8x8 blocks
  int16_t cbf_base[16];     // ctxIdxOffset + ctxBlockCatOffset per ctxBlockCat, 9.3.3.1.1.9
  int16_t sig_base[16];
  int16_t last_base[16];
  int16_t abs_base[16];
  int32_t sig_est_base[16]; // first dense SIG estimator of each ctxBlockCat
};
static_assert(sizeof(HotTables) % 16 == 0, "HotTables is copied in 16-byte units");

struct EngineTables {
  HotTables hot;
  // field-coded macroblocks (field pictures, MBAFF field pairs): Table 9-34's field ctxIdxOffsets of
  // significant / last_significant_coeff_flag per ctxBlockCat and Table 9-43's 8x8 field ctxIdxInc
  // of significant_coeff_flag (last is shared); patched into the walker's LDS copy of `hot`
  int16_t sig_base_fld[16], last_base_fld[16];
  uint8_t sig8x8_fld[64];
  int8_t mn[4][1024][2];  // init (m,n): [0] I, [1..3] cabac_init_idc 0..2
  uint16_t gen_plps[64];  // generator: p_LPS(pStateIdx) * 65536
};

// ------------------------------------------------------------------------- byte staging (LDS)
// The refill / flush paths run once per kStage bytes.  They are real calls (__noinline__), so
// their code exists once in the kernel instead of at every bin site: with everything inlined
// the compress kernel was 1 MB of code and instruction fetch dominated.  They take and return
// plain values, never a pointer to the caller's walker, so the caller's state stays in registers.
struct InStream {
  const uint8_t* g;     // global base (payload start)
  uint32_t limit;       // readable bytes; beyond -> 0
  uint32_t win;         // window start (relative)
  uint8_t* lds;         // kStage bytes
};

// Load the window [at, at + kStage) into LDS, bytes at or past `limit` as 0.  Returns `at`.
__device__ __noinline__ uint32_t in_fill_call(uint8_t* lds, const uint8_t* g, uint32_t limit, uint32_t at) {
  // one wave fills and reads the window: its LDS operations execute in order, so only the
  // compiler needs fencing (the other wave of the workgroup never touches the window)
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  const int lane = __lane_id();
  constexpr int per = kStage / 64;   // bytes per lane
  const uint32_t base = at + (uint32_t)per * lane;
#pragma unroll
  for (int k = 0; k < per; k++) {
    uint32_t i = base + k;
#ifdef AVR_NT_IN
    lds[per * lane + k] = i < limit ? __builtin_nontemporal_load(&g[i]) : 0;
#else
    lds[per * lane + k] = i < limit ? g[i] : 0;
#endif
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  return at;
}
// byte i of the stream (0 at or past limit: the window is zero-filled there)
__device__ __forceinline__ uint32_t in_byte(InStream& s, uint32_t i) {
  if (i - s.win >= (uint32_t)kStage) s.win = in_fill_call(s.lds, s.g, s.limit, i);
  return s.lds[i - s.win];
}
// big-endian 32 bits at i..i+3 with a single window check
__device__ __forceinline__ uint32_t in_be32(InStream& s, uint32_t i) {
  if (i - s.win > (uint32_t)kStage - 4) s.win = in_fill_call(s.lds, s.g, s.limit, i);
  const uint8_t* p = s.lds + (i - s.win);
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// Output bytes go straight to global memory from lane 0 (fire-and-forget stores: nothing in
// the serial chain waits on them, and no staging buffer needs a flush path at every bin site).
struct OutStream {
  uint8_t* g;          // global base (slice output region)
  uint32_t cap;        // capacity
  uint32_t n;          // bytes emitted (written while n < cap)
  uint32_t last;       // last byte emitted
};
__device__ __forceinline__ void out_byte(OutStream& o, uint32_t v) {
#ifdef AVR_NT_OUT
  if (o.n < o.cap && __lane_id() == 0) __builtin_nontemporal_store((uint8_t)v, &o.g[o.n]);
#else
  if (o.n < o.cap && __lane_id() == 0) o.g[o.n] = (uint8_t)v;
#endif
  o.n++;
  o.last = v & 0xff;
}
// k copies of byte v at g[n..n+k) (the deferred 0xFF runs of the carry handling).  Rare: a real
// call, so the loop exists once (inlined, the compiler unrolls it at every bin site).
__device__ __noinline__ void out_run_call(uint8_t* g, uint32_t cap, uint32_t n, uint32_t v, uint32_t k) {
  for (uint32_t i = __lane_id(); i < k; i += 64)
    if (n + i < cap) g[n + i] = (uint8_t)v;
}
__device__ __forceinline__ void out_repeat(OutStream& o, uint32_t v, uint32_t k) {
  out_run_call(o.g, o.cap, o.n, v, k);
  o.n += k;
  if (k) o.last = v & 0xff;
}
__device__ __forceinline__ uint32_t out_total(const OutStream& o) { return o.n; }
__device__ __forceinline__ bool out_overflow(const OutStream& o) { return o.n > o.cap; }

// ------------------------------------------------------------- CABAC state records in VGPRs
// Per pStateIdx p (state byte s = 2p + valMPS): the four LPS ranges (byte q for
// q = (range >> 6) & 3) and the successor states of both state bytes of p: byte
// (s & 1) + 2 is_lps of `nxt` (MPS -> s + 2 while p < 62; LPS -> 2 transIdxLPS[p] + (valMPS ^
// (p == 0))), so the successor is one shift and mask of a record read with the LPS ranges.
struct CabacRec {
  uint32_t lps4, nxt;
};
__device__ __forceinline__ CabacRec rec_of(uint64_t packed) {  // from HotTables::cabac[s]
  CabacRec r;
  r.lps4 = (uint32_t)packed;
  const uint32_t mps = (uint32_t)(packed >> 32) & 0xff, lps = (uint32_t)(packed >> 40) & 0xff;
  r.nxt = (mps | lps << 16) * 0x101u;   // this state's successors in both byte slots
  return r;
}
// The table in two VGPRs (lane p); a lookup with a wave-uniform state is two independent
// v_readlane, no LDS round trip and no branch.
struct VTab {
  uint32_t lps4, nxt;
};
__device__ __forceinline__ void vtab_load(VTab& v, const HotTables* T) {
  const uint64_t p0 = T->cabac[2 * __lane_id()], p1 = T->cabac[2 * __lane_id() + 1];
  v.lps4 = (uint32_t)p0;
  v.nxt = ((uint32_t)(p0 >> 32) & 0xff) | ((uint32_t)(p1 >> 32) & 0xff) << 8 |
          ((uint32_t)(p0 >> 40) & 0xff) << 16 | ((uint32_t)(p1 >> 40) & 0xff) << 24;
}
__device__ __forceinline__ CabacRec vtab_rec(const VTab& v, uint32_t s) {
  CabacRec r;
  r.lps4 = __builtin_amdgcn_readlane(v.lps4, s >> 1);
  r.nxt = __builtin_amdgcn_readlane(v.nxt, s >> 1);
  return r;
}
// Shared by the decoder and the encoder: the LPS range for the current range and the successor
// state for either outcome (is_lps is 0 or 1).
__device__ __forceinline__ uint32_t cabac_lps(uint32_t range, CabacRec r) { return (r.lps4 >> ((range >> 3) & 0x18)) & 0xff; }
__device__ __forceinline__ uint32_t cabac_next(uint32_t s, CabacRec r, uint32_t is_lps) {
  return (r.nxt >> (((s & 1) | is_lps << 1) << 3)) & 0xff;
}

// ---------------------------------------------------------------------- CABAC decoding engine
// 32-bit form of the 9.3.3.2 engine: low = codIOffset << k | the next k stream bits, k >= 8 at
// the start of every operation (one operation consumes at most 7 bits), refilled 16 bits at a
// time so low stays below 2^32.  Every quantity fits a scalar register.
struct CabacDecoder {
  uint32_t low;        // offset << k | lookahead bits
  uint32_t range;      // 9-bit codIRange
  int k;               // lookahead bits below the 9-bit offset
  uint32_t next;       // next byte to load
};

__device__ __forceinline__ void cd_refill(CabacDecoder& d, InStream& in) {
  if (d.k < 8) {
    d.low = (d.low << 16) | (in_be32(in, d.next) >> 16);
    d.next += 2;
    d.k += 16;
  }
}
__device__ __forceinline__ void cd_init(CabacDecoder& d, InStream& in) {  // 9.3.1.2
  d.low = in_be32(in, 0) >> 8;   // 9 offset bits + 15 lookahead bits
  d.k = 15;
  d.next = 3;
  d.range = 510;
}
// bits consumed by the spec decoder so far (9 + renormalisation shifts)
__device__ __forceinline__ uint32_t cd_bitpos(const CabacDecoder& d) { return 8u * d.next - (uint32_t)d.k; }

// One decision given the context's state byte s (2*pStateIdx + valMPS, FFmpeg's cabac_state
// layout) and its record; *ns receives the successor state.  No memory access, so the caller can
// issue the context read of the model side at the same time.
__device__ __forceinline__ int cd_decide(CabacDecoder& d, InStream& in, uint32_t s, CabacRec r, uint32_t* ns) {
  const uint32_t lps = cabac_lps(d.range, r);
  const uint32_t rmps = d.range - lps;
  const uint32_t scaled = rmps << d.k;
  // low >= scaled  <=>  no borrow out of the 64-bit difference (scalar sub + subb)
  const uint32_t is_lps = ~(uint32_t)(((uint64_t)d.low - scaled) >> 32) & 1u;
  const uint32_t m = 0u - is_lps;
  d.low -= scaled & m;
  d.range = rmps ^ ((lps ^ rmps) & m);
  *ns = cabac_next(s, r, is_lps);
  const int n = __builtin_clz(d.range) - 23;   // range >= 2 here: no zero case (one s_flbit, no clamp)
  d.range <<= n;
  d.k -= n;
  cd_refill(d, in);
  return (int)((s & 1) ^ is_lps);
}
__device__ __forceinline__ int cd_decision_v(CabacDecoder& d, InStream& in, uint8_t* state, const VTab& v) {
  const uint32_t s = *state;
  uint32_t ns;
  const int b = cd_decide(d, in, s, vtab_rec(v, s), &ns);
  *state = (uint8_t)ns;
  return b;
}
__device__ __forceinline__ int cd_decision(CabacDecoder& d, InStream& in, uint8_t* state, const HotTables* T) {
  const uint32_t s = *state;
  uint32_t ns;
  const int b = cd_decide(d, in, s, rec_of(T->cabac[s]), &ns);
  *state = (uint8_t)ns;
  return b;
}
__device__ __forceinline__ int cd_bypass(CabacDecoder& d, InStream& in) {
  d.k -= 1;
  const uint32_t scaled = d.range << d.k;
  const bool one = d.low >= scaled;
  d.low -= one ? scaled : 0;
  cd_refill(d, in);
  return one;
}
__device__ __forceinline__ int cd_terminate(CabacDecoder& d, InStream& in) {
  d.range -= 2;
  const uint32_t scaled = d.range << d.k;
  if (d.low >= scaled) return 1;  // no renormalisation: the last bit read is rbsp_stop_one_bit
  if (d.range < 256) {
    d.range <<= 1;
    d.k -= 1;
    cd_refill(d, in);
  }
  return 0;
}

// ---------------------------------------------------------------------- CABAC re-encoder
// Interval arithmetic identical to the spec encoder; the flush writes x = (low' | 1) through its
// last set bit, which is the value arithmetic_code::finish() selects for cabac_code.h.
// low holds the pending bits plus a 10-bit window; queue <= 7 keeps it below 2^25.
struct CabacEncoder {
  uint32_t low;        // pending bits + 10-bit window (bit 9 = carry into the window)
  uint32_t range;      // 9-bit
  int queue;           // (pending bits above the window) - 8
  uint32_t outstanding;
  int have_cache;
  uint32_t cache;
  int err;
};
__device__ __forceinline__ void ce_init(CabacEncoder& e) {
  e.low = 0;
  e.range = 510;
  e.queue = -9;
  e.outstanding = 0;
  e.have_cache = 0;
  e.cache = 0;
  e.err = 0;
}
// one byte out of the window (called with queue >= 0)
__device__ __forceinline__ void ce_putbyte1(CabacEncoder& e, OutStream& o) {
  const uint32_t out = e.low >> (e.queue + 10);
  e.low &= (0x400u << e.queue) - 1;
  e.queue -= 8;
  const uint32_t carry = out >> 8, byte = out & 0xff;
  if (byte == 0xff && !carry) {
    e.outstanding++;
  } else {
    if (e.have_cache) {
      if (e.cache + carry > 0xff) e.err = 1;
      out_byte(o, e.cache + carry);
    } else if (carry) {
      e.err = 1;
    }
    if (e.outstanding) out_repeat(o, (0xff + carry) & 0xff, e.outstanding);
    e.outstanding = 0;
    e.cache = byte;
    e.have_cache = 1;
  }
}
__device__ __forceinline__ void ce_encode(CabacEncoder& e, OutStream& o, int bin, uint32_t s, CabacRec r, uint32_t* ns) {
  const uint32_t lps = cabac_lps(e.range, r);
  const uint32_t rmps = e.range - lps;
  const uint32_t is_lps = ((uint32_t)bin ^ s) & 1u;
  const uint32_t m = 0u - is_lps;
  e.low += rmps & m;
  e.range = rmps ^ ((lps ^ rmps) & m);
  *ns = cabac_next(s, r, is_lps);
  const int n = __builtin_clz(e.range) - 23;   // <= 6: at most one byte per decision
  e.range <<= n;
  e.low <<= n;
  e.queue += n;
  if (e.queue >= 0) ce_putbyte1(e, o);
}
__device__ __forceinline__ void ce_decision(CabacEncoder& e, OutStream& o, int bin, uint8_t* state,
                                            const HotTables* T) {
  const uint32_t s = *state;
  uint32_t ns;
  ce_encode(e, o, bin, s, rec_of(T->cabac[s]), &ns);
  *state = (uint8_t)ns;
}
__device__ __forceinline__ void ce_decision_v(CabacEncoder& e, OutStream& o, int bin, uint8_t* state, const VTab& v) {
  const uint32_t s = *state;
  uint32_t ns;
  ce_encode(e, o, bin, s, vtab_rec(v, s), &ns);
  *state = (uint8_t)ns;
}
__device__ __forceinline__ void ce_bypass(CabacEncoder& e, OutStream& o, int bin) {
  e.low = (e.low << 1) + (bin ? e.range : 0);
  e.queue += 1;
  if (e.queue >= 0) ce_putbyte1(e, o);
}
__device__ __forceinline__ void ce_terminate(CabacEncoder& e, OutStream& o, int bin) {
  e.range -= 2;
  if (!bin) {
    const int n = __clz(e.range) - 23;
    e.range <<= n;
    e.low <<= n;
    e.queue += n;
    if (e.queue >= 0) ce_putbyte1(e, o);
    return;
  }
  // flush: x = (low + range - 2) | 1 in units of the window LSB, written through that bit.
  // Up to 25 pending bits + 10 + 7 pad: done in 64 bits, once per slice.
  uint64_t low = (uint64_t)((e.low + e.range) | 1) << 10;
  int queue = e.queue + 10;
  const int total = queue + 8;  // bits still pending
  const int pad = (8 - (total & 7)) & 7;
  low <<= pad;
  queue += pad;
  #pragma clang loop unroll(disable)
  while (queue >= 0) {
    const uint32_t out = (uint32_t)(low >> (queue + 10));
    low &= (0x400ull << queue) - 1;
    queue -= 8;
    const uint32_t carry = out >> 8, byte = out & 0xff;
    if (byte == 0xff && !carry) {
      e.outstanding++;
    } else {
      if (e.have_cache) {
        if (e.cache + carry > 0xff) e.err = 1;
        out_byte(o, e.cache + carry);
      } else if (carry) {
        e.err = 1;
      }
      if (e.outstanding) out_repeat(o, (0xff + carry) & 0xff, e.outstanding);
      e.outstanding = 0;
      e.cache = byte;
      e.have_cache = 1;
    }
  }
  e.low = 0;
  e.queue = queue;
  if (e.have_cache) out_byte(o, e.cache);
  if (e.outstanding) out_repeat(o, 0xff, e.outstanding);
  e.outstanding = 0;
  e.have_cache = 0;
}

// ----------------------------------------------------------------- recoded coder (u64 / u8)
// p1 = floor(range / (pos + neg)) * pos (recode.cpp:819), est = (pos - 1) | (neg - 1) << 8: the
// walkers divide with HotTables::div (floor(n/d) = umulhi(n, m) >> shift, exact for n <= 2^63:
// check_reciprocals in avr_api.cpp) -- by scalar load in the decompress walker (Walker::p1), by a
// per-lane gather in the compress coder.
// update_state_for_model_key (recode.cpp:1036-1045)
// On the packed form: with p = pos - 1 and n = neg - 1 in the two bytes, the count goes up in its
// byte (no carry: pos + neg <= 0x60 after every update, so p <= 0x5e before one), the test
// pos + neg > thresh is p + n > thresh - 2, and ((x + 1) >> 1) - 1 = (x - 1) >> 1 halves both
// bytes at once: p >> 1 and n >> 1, i.e. (x >> 1) & 0x7f7f.  Nine scalar instructions instead of
// about twenty for the unpacked form.
// The test is made on the counts before the update, (p + n) + 1 > thresh - 2: their sum is the
// one the decision's probability already formed (tot = p + n + 2, Walker::p1), so the compiler
// shares it and the update costs six scalar instructions.
__device__ __forceinline__ uint32_t est_update(uint32_t est, int bin, uint32_t thresh) {
  const uint32_t sum = (est & 0xff) + (est >> 8);
  const uint32_t x = est + (bin ? 1u : 0x100u);
  return sum > thresh - 3 ? (x >> 1) & 0x7f7fu : x;
}

struct RecodedEncoder {
  uint64_t low, range;
  uint32_t pending;     // deferred 0xFF digits
  int have_cache;
  uint32_t cache;
  int err;
};
__device__ __forceinline__ void re_init(RecodedEncoder& e) {
  e.low = 0;
  e.range = 1ull << 63;
  e.pending = 0;
  e.have_cache = 0;
  e.cache = 0;
  e.err = 0;
}
__device__ __forceinline__ void re_shift(RecodedEncoder& e, OutStream& o) {
  const uint32_t h = hi32(e.low);
  const uint32_t carry = h >> 31;
  const uint32_t digit = (h >> 23) & 0xff;
  if (digit != 0xff || carry) {
    if (e.have_cache) {
      if (e.cache + carry > 0xff) e.err = 1;
      out_byte(o, e.cache + carry);
    } else if (carry) {
      e.err = 1;
    }
    if (e.pending) out_repeat(o, (0xff + carry) & 0xff, e.pending);
    e.pending = 0;
    e.cache = digit;
    e.have_cache = 1;
  } else {
    e.pending++;
  }
  e.low = (e.low & ((1ull << 55) - 1)) << 8;
}
__device__ __forceinline__ void re_put(RecodedEncoder& e, OutStream& o, int bin, uint64_t r1) {
  const uint64_t r0 = e.range - r1;
  e.low += bin ? r0 : 0;
  e.range = bin ? r1 : r0;
  if (hi32(e.range) < (1u << 19)) {  // range < min_range = (fixed_one/digit_base)/16 = 2^51
    if (e.range == 0) e.err = 1;
    #pragma clang loop unroll(disable)
    do {  // at most twice: r1, r0 >= range/96 and range >= 2^51 before the put
      re_shift(e, o);
      e.range <<= 8;
    } while (hi32(e.range) < (1u << 23) && e.range != 0);  // until range >= 2^55
  }
}
// Billing (h264_model::billable_bytes, recode.cpp:656-658, 1074-1078): encoder::put returns the
// bytes its renormalisation emitted (arithmetic_code.h:106-126, 147-190), and the reference emits a
// digit only once its top digit cannot change (deferring it, and every digit after it, while
// low and low + range - 1 disagree on it), so its count per put differs from the bytes this
// encoder's cache scheme writes at that put.  re_put_billed runs re_put and returns the
// reference's count: at each renormalisation step the reference's low is this low without the
// carry bit (bit 63), its range is this range; *pend counts the reference's deferred digits.
__device__ __forceinline__ uint32_t re_put_billed(RecodedEncoder& e, OutStream& o, int bin, uint64_t r1,
                                                  uint32_t* pend) {
  const uint64_t r0 = e.range - r1;
  e.low += bin ? r0 : 0;
  e.range = bin ? r1 : r0;
  uint32_t bytes = 0;
  if (hi32(e.range) < (1u << 19)) {
    if (e.range == 0) e.err = 1;
    #pragma clang loop unroll(disable)
    do {
      const uint64_t lo = e.low & ((1ull << 63) - 1);
      const bool deferred = ((lo >> 55) & 0xff) != (((lo + e.range - 1) >> 55) & 0xff);
      bytes += deferred ? 0u : *pend + 1;
      *pend = deferred ? *pend + 1 : 0u;
      re_shift(e, o);
      e.range <<= 8;
    } while (hi32(e.range) < (1u << 23) && e.range != 0);
  }
  return bytes;
}

// The generic coder behind cabac_code.h (arithmetic_code<uint32_t, uint16_t, 0x200>: fixed_one
// 2^31, 16-bit digits of 2 bytes, min_range 0x200, renormalised while range < 2^15), tracked only
// for its billing (h264_model::billable_cabac_bytes, recode.cpp:659-661, 1443-1468): the CABAC
// encoder above writes the same bytes, but at other moments.
struct CabacBill {
  uint32_t low, range, pend;
};
__device__ __forceinline__ void cb_init(CabacBill& b) {
  b.low = 0;
  b.range = (0x80000000u / 0x200u) * 0x1FEu;   // cabac_code.h:30
  b.pend = 0;
}
// encoder::put(symbol, range_of_1): the bytes it reports
__device__ __forceinline__ uint32_t cb_put(CabacBill& b, int sym, uint32_t r1) {
  const uint32_t r0 = b.range - r1;
  b.low += sym ? r0 : 0u;
  b.range = sym ? r1 : r0;
  uint32_t bytes = 0;
  if (b.range < 0x200u) {
    #pragma clang loop unroll(disable)
    while (b.range < 0x8000u && b.range != 0) {
      if (b.low >= 0x80000000u) b.low -= 0x80000000u;   // carry into the deferred digits
      const uint32_t d = b.low >> 15, dhi = ((b.low + b.range - 1) >> 15) & 0xffffu;
      bytes += d != dhi ? 0u : 2u * (b.pend + 1);
      b.pend = d != dhi ? b.pend + 1 : 0u;
      b.low = (b.low - (d << 15)) << 16;
      b.range <<= 16;
    }
  }
  return bytes;
}
// normalize = log2(range / 0x100) (cabac_code.h:39, 70-79): range >> normalize is 9 bits
__device__ __forceinline__ uint32_t cb_norm(uint32_t range) { return 23u - (uint32_t)__clz(range); }
// cabac::encoder::put (cabac_code.h:33-49): state s before the bin
__device__ __forceinline__ uint32_t cb_decision(CabacBill& b, int bin, uint32_t s, CabacRec r) {
  const uint32_t nrm = cb_norm(b.range);
  const uint32_t lps = cabac_lps(b.range >> nrm, r) << nrm;
  return cb_put(b, ((uint32_t)bin ^ s) & 1u, lps);
}
__device__ __forceinline__ uint32_t cb_bypass(CabacBill& b, int bin) { return cb_put(b, bin, b.range >> 1); }
__device__ __forceinline__ uint32_t cb_terminate(CabacBill& b, int bin) {
  return cb_put(b, bin, 2u << cb_norm(b.range));
}

__device__ __forceinline__ void re_finish(RecodedEncoder& e, OutStream& o) {  // arith:128-144
  #pragma clang loop unroll(disable)
  for (uint64_t sb = 1ull << 62; sb; sb >>= 1) {
    uint64_t x = (e.low | sb) & ~(sb - 1);
    if (sb < e.range && e.low <= x && x < e.low + e.range) {
      e.low = x;
      break;
    }
  }
  #pragma clang loop unroll(disable)
  while (e.low != 0) re_shift(e, o);
  if (e.have_cache) out_byte(o, e.cache);
  if (e.pending) out_repeat(o, 0xff, e.pending);
  e.pending = 0;
  e.have_cache = 0;
}

struct RecodedDecoder {
  uint64_t low, range;
  uint32_t next_digit;  // last aligned digit read
  uint32_t next;        // next byte index
};
__device__ __forceinline__ void rd_consume(RecodedDecoder& d, InStream& in) {
  // the byte comes from LDS in a vector register: move it to a scalar one so that low stays a
  // scalar register (otherwise every bin pays vector<->scalar transfers on low)
  uint32_t b = __builtin_amdgcn_readfirstlane(in_byte(in, d.next++));
  uint32_t digit = ((d.next_digit & 1) << 7) | (b >> 1);
  d.next_digit = b;
  d.low = (d.low << 8) | digit;
  d.range <<= 8;
}
__device__ __forceinline__ void rd_init(RecodedDecoder& d, InStream& in) {  // arith:218-230
  d.next = 0;
  d.next_digit = in_byte(in, d.next++);
  d.low = d.next_digit >> 1;
  d.range = 128;
  #pragma clang loop unroll(disable)
  while (d.range < (1ull << 63)) rd_consume(d, in);
}
// low < range <= 2^63, so low - r0 fits a signed 64-bit value: its sign bit is the decision
// (two scalar subtracts and a 32-bit shift instead of a vector 64-bit compare).
__device__ __forceinline__ int rd_get(RecodedDecoder& d, InStream& in, uint64_t r1) {
  const uint64_t r0 = d.range - r1;
  const uint64_t diff = d.low - r0;
  const bool bin = (hi32(diff) >> 31) == 0;
  d.low = bin ? diff : d.low;
  d.range = bin ? r1 : r0;
  // below min_range (2^51) the encoder shifts until range >= 2^55 (re_put).  A decision starts
  // from range >= 2^51 and both outcomes keep at least range / 97 > 2^44 (pos, neg >= 1,
  // pos + neg <= 97), never 0: one or two digits, straight-line instead of a loop
  if (hi32(d.range) < (1u << 19)) {
    rd_consume(d, in);
    if (hi32(d.range) < (1u << 23)) rd_consume(d, in);
  }
  return bin;
}

// ------------------------------------------------------------ P-format coder (u32 / u8 digits)
// The parallel model's container (avrecode-amd:P32) is this library's own format, not bound to the
// reference's arithmetic_code<uint64_t, uint8_t>: a 32-bit range coder with byte digits, the same
// estimators and the same decision rule (bin 1 takes the top r1 of the range).
//   range in [2^24, 2^32) between decisions (0xFFFFFFFF at the start);
//   r1 = umulhi(range, rcp32[tot]) * pos, rcp32[tot] = floor(2^32 / tot), tot = pos + neg <= 97:
//   r1 <= range * pos / tot, so both parts keep >= range / tot - 1 > 2^17 and ONE 8-bit
//   renormalisation step always restores range >= 2^24.
// Per decision that is one 32-bit multiply-high and one multiply instead of the 64-bit
// reciprocal product (~15 scalar instructions), and 32-bit compares and selects; the coding
// loss of the truncated quotient is below 97 / 2^24 of the range (1e-5 of a bit per decision).
// Encoder: low holds the window (bits 0-31) and the carry (bit 32); digits are bits 24-31 at each
// renormalisation, with the cache + 0xFF-run carry scheme of RecodedEncoder.
struct PEncoder {
  uint64_t low;
  uint32_t range;
  uint32_t pending;     // deferred 0xFF digits
  int have_cache;
  uint32_t cache;
  int err;
};
__device__ __forceinline__ void re_init(PEncoder& e) {
  e.low = 0;
  e.range = 0xffffffffu;
  e.pending = 0;
  e.have_cache = 0;
  e.cache = 0;
  e.err = 0;
}
__device__ __forceinline__ void pe_shift(PEncoder& e, OutStream& o) {
  const uint32_t carry = (uint32_t)(e.low >> 32) & 1u;
  const uint32_t digit = (uint32_t)(e.low >> 24) & 0xff;
  if (digit != 0xff || carry) {
    if (e.have_cache) {
      if (e.cache + carry > 0xff) e.err = 1;
      out_byte(o, e.cache + carry);
    } else if (carry) {
      e.err = 1;
    }
    if (e.pending) out_repeat(o, (0xff + carry) & 0xff, e.pending);
    e.pending = 0;
    e.cache = digit;
    e.have_cache = 1;
  } else {
    e.pending++;
  }
  e.low = (e.low & 0xffffffu) << 8;
}
__device__ __forceinline__ void re_put(PEncoder& e, OutStream& o, int bin, uint32_t r1) {
  const uint32_t r0 = e.range - r1;
  e.low += bin ? r0 : 0u;
  e.range = bin ? r1 : r0;
  if (e.range < (1u << 24)) {
    pe_shift(e, o);
    e.range <<= 8;
  }
}
// billing (as re_put_billed): a digit counts when its value is final, deferred digits with it
__device__ __forceinline__ uint32_t re_put_billed(PEncoder& e, OutStream& o, int bin, uint32_t r1, uint32_t* pend) {
  const uint32_t r0 = e.range - r1;
  e.low += bin ? r0 : 0u;
  e.range = bin ? r1 : r0;
  uint32_t bytes = 0;
  if (e.range < (1u << 24)) {
    const uint32_t lo = (uint32_t)e.low;
    const bool deferred = (lo >> 24) != (uint32_t)(((uint64_t)lo + e.range - 1) >> 24);   // a carry may still come
    bytes = deferred ? 0u : *pend + 1;
    *pend = deferred ? *pend + 1 : 0u;
    pe_shift(e, o);
    e.range <<= 8;
  }
  return bytes;
}
// flush: the value in [low, low + range) with the most trailing zero bits, through its last
// non-zero digit (the decoder reads zeros past the end)
__device__ __forceinline__ void re_finish(PEncoder& e, OutStream& o) {
  #pragma clang loop unroll(disable)
  for (uint64_t sb = 1ull << 32; sb; sb >>= 1) {
    const uint64_t x = (e.low | sb) & ~(sb - 1);
    if (sb < e.range && e.low <= x && x < e.low + e.range) {
      e.low = x;
      break;
    }
  }
  #pragma clang loop unroll(disable)
  while (e.low != 0) pe_shift(e, o);
  if (e.have_cache) out_byte(o, e.cache);
  if (e.pending) out_repeat(o, 0xff, e.pending);
  e.pending = 0;
  e.have_cache = 0;
}
// Decoder: low = (stream value - encoder low) in the 32-bit window, always < range.
struct PDecoder {
  uint32_t low, range;
  uint32_t next;        // next byte index
  uint32_t pf;          // byte next, read from LDS one renormalisation ahead (its latency off the chain)
};
__device__ __forceinline__ void rd_init(PDecoder& d, InStream& in) {
  d.low = __builtin_amdgcn_readfirstlane(in_be32(in, 0));
  d.next = 4;
  d.range = 0xffffffffu;
  d.pf = in_byte(in, 4);
}
__device__ __forceinline__ int rd_get(PDecoder& d, InStream& in, uint32_t r1) {
  const uint32_t r0 = d.range - r1;
  const bool bin = d.low >= r0;
  d.low = bin ? d.low - r0 : d.low;
  d.range = bin ? r1 : r0;
  if (d.range < (1u << 24)) {
    d.low = (d.low << 8) | __builtin_amdgcn_readfirstlane(d.pf);
    d.pf = in_byte(in, ++d.next);
    d.range <<= 8;
  }
  return bin;
}

}  // namespace avr
