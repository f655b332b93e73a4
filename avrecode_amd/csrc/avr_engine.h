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

// Tables read on every bin: copied into each workgroup's LDS at kernel start.
struct HotTables {
  uint64_t div_m[128];    // ceil(2^(63+l)/d), l = ceil(log2 d)
  uint64_t div_top[128];  // floor(2^63 / d)
  uint8_t lps[512];       // [q*128 + state]
  uint8_t mlps[256];      // [128+s] after MPS, [127-s] after LPS
  uint8_t div_s[128];     // l - 1
  uint8_t nb_left[48];    // get_neighbor_sub_mb: block left of n (| 128 if in the left macroblock)
  uint8_t nb_up[48];      //                      block above n (| 128 if in the upper macroblock)
};
static_assert(sizeof(HotTables) % 16 == 0, "HotTables is copied in 16-byte units");

struct EngineTables {
  HotTables hot;
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
  __syncthreads();
  const int lane = threadIdx.x;
  const uint32_t base = at + 16u * lane;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    uint32_t i = base + k;
    lds[16 * lane + k] = i < limit ? g[i] : 0;
  }
  __syncthreads();
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
  if (o.n < o.cap && threadIdx.x == 0) o.g[o.n] = (uint8_t)v;
  o.n++;
  o.last = v & 0xff;
}
// k copies of byte v at g[n..n+k) (the deferred 0xFF runs of the carry handling).  Rare: a real
// call, so the loop exists once (inlined, the compiler unrolls it at every bin site).
__device__ __noinline__ void out_run_call(uint8_t* g, uint32_t cap, uint32_t n, uint32_t v, uint32_t k) {
  for (uint32_t i = threadIdx.x; i < k; i += 64)
    if (n + i < cap) g[n + i] = (uint8_t)v;
}
__device__ __forceinline__ void out_repeat(OutStream& o, uint32_t v, uint32_t k) {
  out_run_call(o.g, o.cap, o.n, v, k);
  o.n += k;
  if (k) o.last = v & 0xff;
}
__device__ __forceinline__ uint32_t out_total(const OutStream& o) { return o.n; }
__device__ __forceinline__ bool out_overflow(const OutStream& o) { return o.n > o.cap; }

// ---------------------------------------------------------------------- CABAC decoding engine
struct CabacDecoder {
  uint64_t value;      // offset << avail | lookahead bits
  uint32_t range;      // 9-bit codIRange
  int avail;           // lookahead bits below the 9-bit offset
  uint32_t next;       // next byte to load
};

__device__ __forceinline__ void cd_refill(CabacDecoder& d, InStream& in) {
  uint32_t w = in_be32(in, d.next);
  d.next += 4;
  d.value = (d.value << 32) | w;
  d.avail += 32;
}
__device__ __forceinline__ void cd_init(CabacDecoder& d, InStream& in) {  // 9.3.1.2
  d.value = 0;
  d.avail = -9;
  d.next = 0;
  d.range = 510;
  cd_refill(d, in);
}
// bits consumed by the spec decoder so far (9 + renormalisation shifts)
__device__ __forceinline__ uint32_t cd_bitpos(const CabacDecoder& d) { return 8u * d.next - (uint32_t)d.avail; }

__device__ __forceinline__ int cd_decision(CabacDecoder& d, InStream& in, uint8_t* state, const HotTables* T) {
  uint32_t s = *state;
  uint32_t lps = T->lps[((d.range >> 6) & 3) * 128 + s];
  d.range -= lps;
  uint64_t scaled = (uint64_t)d.range << d.avail;
  int bin;
  if (d.value >= scaled) {
    bin = !(s & 1);
    d.value -= scaled;
    d.range = lps;
    *state = T->mlps[127 - s];
  } else {
    bin = s & 1;
    *state = T->mlps[128 + s];
  }
  int n = __clz(d.range) - 23;
  d.range <<= n;
  d.avail -= n;
  if (d.avail < 16) cd_refill(d, in);
  return bin;
}
__device__ __forceinline__ int cd_bypass(CabacDecoder& d, InStream& in) {
  d.avail -= 1;
  uint64_t scaled = (uint64_t)d.range << d.avail;
  int bin = 0;
  if (d.value >= scaled) {
    d.value -= scaled;
    bin = 1;
  }
  if (d.avail < 16) cd_refill(d, in);
  return bin;
}
__device__ __forceinline__ int cd_terminate(CabacDecoder& d, InStream& in) {
  d.range -= 2;
  uint64_t scaled = (uint64_t)d.range << d.avail;
  if (d.value >= scaled) return 1;  // no renormalisation: the last bit read is rbsp_stop_one_bit
  if (d.range < 256) {
    d.range <<= 1;
    d.avail -= 1;
    if (d.avail < 16) cd_refill(d, in);
  }
  return 0;
}

// ---------------------------------------------------------------------- CABAC re-encoder
// Interval arithmetic identical to the spec encoder; the flush writes x = (low' | 1) through its
// last set bit, which is the value arithmetic_code::finish() selects for cabac_code.h.
struct CabacEncoder {
  uint64_t low;        // pending bits + 10-bit window (bit 9 = carry into the window)
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
__device__ __forceinline__ void ce_putbyte(CabacEncoder& e, OutStream& o) {
  #pragma clang loop unroll(disable)
  while (e.queue >= 0) {
    uint32_t out = (uint32_t)(e.low >> (e.queue + 10));
    e.low &= (0x400ull << e.queue) - 1;
    e.queue -= 8;
    uint32_t carry = out >> 8, byte = out & 0xff;
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
}
__device__ __forceinline__ void ce_renorm(CabacEncoder& e, OutStream& o) {
  int n = __clz(e.range) - 23;
  e.range <<= n;
  e.low <<= n;
  e.queue += n;
  if (e.queue >= 0) ce_putbyte(e, o);
}
__device__ __forceinline__ void ce_decision(CabacEncoder& e, OutStream& o, int bin, uint8_t* state,
                                            const HotTables* T) {
  uint32_t s = *state;
  uint32_t lps = T->lps[((e.range >> 6) & 3) * 128 + s];
  e.range -= lps;
  if (bin != (int)(s & 1)) {
    e.low += e.range;
    e.range = lps;
    *state = T->mlps[127 - s];
  } else {
    *state = T->mlps[128 + s];
  }
  ce_renorm(e, o);
}
__device__ __forceinline__ void ce_bypass(CabacEncoder& e, OutStream& o, int bin) {
  e.low = (e.low << 1) + (bin ? e.range : 0);
  e.queue += 1;
  if (e.queue >= 0) ce_putbyte(e, o);
}
__device__ __forceinline__ void ce_terminate(CabacEncoder& e, OutStream& o, int bin) {
  e.range -= 2;
  if (!bin) {
    ce_renorm(e, o);
    return;
  }
  // flush: x = (low + range - 2) | 1 in units of the window LSB, written through that bit
  e.low = (e.low + e.range) | 1;
  e.low <<= 10;
  e.queue += 10;
  int total = e.queue + 8;  // bits still pending
  int pad = (8 - (total & 7)) & 7;
  e.low <<= pad;
  e.queue += pad;
  ce_putbyte(e, o);
  if (e.have_cache) out_byte(o, e.cache);
  if (e.outstanding) out_repeat(o, 0xff, e.outstanding);
  e.outstanding = 0;
  e.have_cache = 0;
}

// ----------------------------------------------------------------- recoded coder (u64 / u8)
__device__ __forceinline__ uint64_t rc_div(uint64_t range, uint32_t d, const HotTables* T) {
  if (range >> 63) return T->div_top[d];
  return __umul64hi(range, T->div_m[d]) >> T->div_s[d];
}
// p1 = (range/(pos+neg))*pos  (recode.cpp:819); est = (pos-1) | (neg-1) << 8
__device__ __forceinline__ uint64_t rc_p1(uint64_t range, uint32_t est, const HotTables* T) {
  uint32_t pos = (est & 0xff) + 1, neg = (est >> 8) + 1;
  return rc_div(range, pos + neg, T) * pos;
}
// update_state_for_model_key (recode.cpp:1036-1045)
__device__ __forceinline__ uint32_t est_update(uint32_t est, int bin, uint32_t thresh) {
  uint32_t pos = (est & 0xff) + 1 + (bin ? 1 : 0), neg = (est >> 8) + 1 + (bin ? 0 : 1);
  if (pos + neg > thresh) {
    pos = (pos + 1) >> 1;
    neg = (neg + 1) >> 1;
  }
  return (pos - 1) | ((neg - 1) << 8);
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
  uint32_t carry = (uint32_t)(e.low >> 63);
  uint32_t digit = (uint32_t)(e.low >> 55) & 0xff;
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
  if (bin) {
    e.low += e.range - r1;
    e.range = r1;
  } else {
    e.range -= r1;
  }
  if (e.range < (1ull << 51)) {  // min_range = (fixed_one/digit_base)/16
    if (e.range == 0) e.err = 1;
    #pragma clang loop unroll(disable)
    while (e.range < (1ull << 55)) {
      re_shift(e, o);
      e.range <<= 8;
    }
  }
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
  uint32_t b = in_byte(in, d.next++);
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
__device__ __forceinline__ int rd_get(RecodedDecoder& d, InStream& in, uint64_t r1) {
  uint64_t r0 = d.range - r1;
  int bin = d.low >= r0;
  if (bin) {
    d.low -= r0;
    d.range = r1;
  } else {
    d.range = r0;
  }
  if (d.range < (1ull << 51))
    #pragma clang loop unroll(disable)
    while (d.range < (1ull << 55)) rd_consume(d, in);
  return bin;
}

}  // namespace avr
