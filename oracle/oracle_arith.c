/*
 * Oracle: arithmetic coders.  TEST INFRASTRUCTURE ONLY (see avr_oracle.h).
 *
 * ac_enc_* / ac_dec_*  restate arithmetic_code.h:31-299 literally, including the unbounded
 *                      "overflow" digit vector (arith:155-174, 200) so that the restatement can be
 *                      compared against the header compiled as-is (oracle/_ref/ref_arith).
 * cabac_enc_*          restates cabac_code.h:27-80.
 * cabac_dec_*          restates the ITU-T H.264 9.3.1.2 / 9.3.3.2 decoding engine that the
 *                      libavcodec-hooks fork exposes as ff_get_cabac* (recode.cpp:1176-1188).
 */
#include <stdlib.h>
#include <string.h>

#include "avr_oracle.h"

void ob_init(obuf_t *b) { b->data = NULL; b->len = b->cap = 0; }
void ob_free(obuf_t *b) { free(b->data); ob_init(b); }
static void ob_reserve(obuf_t *b, size_t n) {
  if (b->len + n <= b->cap) return;
  size_t c = b->cap ? b->cap : 256;
  while (c < b->len + n) c *= 2;
  b->data = (uint8_t *)realloc(b->data, c);
  b->cap = c;
}
void ob_put(obuf_t *b, uint8_t v) { ob_reserve(b, 1); b->data[b->len++] = v; }
void ob_append(obuf_t *b, const uint8_t *p, size_t n) {
  if (!n) return;
  ob_reserve(b, n);
  memcpy(b->data + b->len, p, n);
  b->len += n;
}

/* ---------------------------------------------------------------- generic encoder (arith:89-203) */
void ac_enc_init(ac_enc_t *e, obuf_t *out, int fixed_bits, int digit_bits, uint64_t min_range,
                 uint64_t initial_range) {
  e->fixed_one = 1ull << (fixed_bits - 1);                   /* arith:54-55 */
  e->digit_bits = digit_bits;
  e->out_bits = 8;
  /* arith:60-61: MinRange > 0 ? MinRange : (fixed_one/digit_base)/16 */
  e->min_range = min_range ? min_range : ((e->fixed_one >> digit_bits) / 16);
  e->low = 0;
  e->range = initial_range ? initial_range : e->fixed_one;  /* arith:96-98 */
  e->overflow = NULL;
  e->novf = e->capovf = 0;
  e->bytes_emitted = 0;
  e->out = out;
}

void ac_enc_free(ac_enc_t *e) { free(e->overflow); e->overflow = NULL; e->novf = e->capovf = 0; }

/* emit_digit<Digit> (arith:178-184): big-endian split into OutputDigits; bills sizeof(digit) */
static void emit_digit(ac_enc_t *e, uint32_t digit, int bits) {
  for (int i = bits - 8; i >= 0; i -= 8) ob_put(e->out, (uint8_t)(digit >> i));
  e->bytes_emitted += (size_t)(bits / 8);
}

/* renormalize_and_emit_digit<Digit> (arith:146-175) */
static void renorm_emit(ac_enc_t *e, int bits) {
  const uint64_t base = 1ull << bits;
  const uint64_t msd = e->fixed_one / base;
  const uint32_t dmask = (uint32_t)(base - 1);
  const uint16_t cmask = (uint16_t)((1u << e->digit_bits) - 1);
  if (e->low >= e->fixed_one) {  /* carry cascades from the lowest overflow digit upward */
    for (long i = (long)e->novf - 1; i >= 0; i--) {
      e->overflow[i] = (uint16_t)((e->overflow[i] + 1) & cmask);
      if (e->overflow[i] != 0) break;
    }
    e->low -= e->fixed_one;
  }
  uint32_t digit = (uint32_t)(e->low / msd) & dmask;
  uint32_t top = (uint32_t)((e->low + e->range - 1) / msd) & dmask;
  if (digit != top) {
    if (e->novf == e->capovf) {
      e->capovf = e->capovf ? 2 * e->capovf : 16;
      e->overflow = (uint16_t *)realloc(e->overflow, e->capovf * sizeof(uint16_t));
    }
    e->overflow[e->novf++] = (uint16_t)digit;
  } else {
    for (size_t i = 0; i < e->novf; i++) emit_digit(e, e->overflow[i], e->digit_bits);
    e->novf = 0;
    emit_digit(e, digit, bits);
  }
  e->low -= (uint64_t)digit * msd;
  e->low *= base;
  e->range *= base;
}

/* encoder::put (arith:106-126) */
size_t ac_enc_put(ac_enc_t *e, int symbol, uint64_t range_of_1) {
  uint64_t range_of_0 = e->range - range_of_1;
  if (symbol != 0) {
    e->low += range_of_0;
    e->range = range_of_1;
  } else {
    e->range = range_of_0;
  }
  if (e->range < e->min_range) {
    if (e->range == 0) abort(); /* "Encoder error: emitted a zero-probability symbol." */
    size_t before = e->bytes_emitted;
    while (e->range < e->fixed_one / (1ull << e->digit_bits)) renorm_emit(e, e->digit_bits);
    return e->bytes_emitted - before;
  }
  return 0;
}

/* encoder::finish (arith:128-144) */
void ac_enc_finish(ac_enc_t *e) {
  if (e->range == 0) return; /* already finished (destructor's second call is a no-op) */
  for (uint64_t stop_bit = e->fixed_one >> 1; stop_bit > 0; stop_bit >>= 1) {
    uint64_t x = (e->low | stop_bit) & ~(stop_bit - 1);
    if (stop_bit < e->range && e->low <= x && x < e->low + e->range) {
      e->low = x;
      break;
    }
  }
  while (e->low != 0) {
    e->range = 1;
    renorm_emit(e, e->out_bits);
  }
  e->range = 0;
}

/* ---------------------------------------------------------------- generic decoder (arith:211-298) */
static uint64_t consume_aligned(ac_dec_t *d) {
  uint64_t digit = 0;
  for (int i = 0; i < d->digit_bytes; i++) {
    digit <<= 8;
    if (d->in != d->end) digit |= *d->in++;  /* reads past the end return 0 */
  }
  return digit;
}
static uint64_t consume_digit(ac_dec_t *d) {
  uint64_t in = consume_aligned(d);
  uint64_t digit = ((d->next_digit * (d->digit_base / d->digit_alignment)) |
                    (in / d->digit_alignment)) & (d->digit_base - 1);
  d->next_digit = in;
  return digit;
}
static void renorm_consume(ac_dec_t *d) {
  uint64_t digit = consume_digit(d);
  d->low = d->low * d->digit_base + digit;
  d->range *= d->digit_base;
}

void ac_dec_init(ac_dec_t *d, const uint8_t *in, const uint8_t *end, int fixed_bits, int digit_bits,
                 uint64_t min_range) {
  d->fixed_one = 1ull << (fixed_bits - 1);
  d->digit_base = 1ull << digit_bits;
  d->digit_bytes = digit_bits / 8;
  d->min_range = min_range ? min_range : ((d->fixed_one >> digit_bits) / 16);
  /* digit_alignment = max/fixed_one + 1 (arith:252) */
  uint64_t maxv = fixed_bits == 64 ? ~0ull : ((1ull << fixed_bits) - 1);
  d->digit_alignment = maxv / d->fixed_one + 1;
  d->in = in;
  d->end = end;
  d->next_digit = consume_aligned(d);
  d->low = d->next_digit / d->digit_alignment;
  d->range = d->digit_base / d->digit_alignment;
  while (d->range < d->fixed_one) renorm_consume(d);
}

int ac_dec_get(ac_dec_t *d, uint64_t range_of_1) {
  uint64_t range_of_0 = d->range - range_of_1;
  int symbol = d->low >= range_of_0;
  if (symbol) {
    d->low -= range_of_0;
    d->range = range_of_1;
  } else {
    d->range = range_of_0;
  }
  if (d->range < d->min_range) {
    while (d->range < d->fixed_one / d->digit_base) renorm_consume(d);
  }
  return symbol;
}

/* recoded_code = arithmetic_code<uint64_t, uint8_t> (recode.cpp:315-316) */
void rc_enc_init(ac_enc_t *e, obuf_t *out) { ac_enc_init(e, out, 64, 8, 0, 0); }
void rc_dec_init(ac_dec_t *d, const uint8_t *in, size_t n) { ac_dec_init(d, in, in + n, 64, 8, 0); }

/* ---------------------------------------------------------------- P-format coder (avr_oracle.h) */
void pc_enc_init(pc_enc_t *e, obuf_t *out) {
  memset(e, 0, sizeof(*e));
  e->range = 0xffffffffu;
  e->out = out;
}
static void pc_shift(pc_enc_t *e) {
  const uint32_t carry = (uint32_t)(e->low >> 32) & 1u, digit = (uint32_t)(e->low >> 24) & 0xff;
  if (digit != 0xff || carry) {
    if (e->have_cache) {
      if (e->cache + carry > 0xff) e->err = 1;
      ob_put(e->out, (uint8_t)(e->cache + carry));
    } else if (carry) {
      e->err = 1;
    }
    for (; e->pending; e->pending--) ob_put(e->out, (uint8_t)(0xff + carry));
    e->cache = digit;
    e->have_cache = 1;
  } else {
    e->pending++;
  }
  e->low = (e->low & 0xffffffu) << 8;
}
size_t pc_enc_put(pc_enc_t *e, int symbol, uint32_t r1) {
  const uint32_t r0 = e->range - r1;
  if (symbol) e->low += r0;
  e->range = symbol ? r1 : r0;
  size_t billed = 0;
  if (e->range < (1u << 24)) {
    const uint64_t lo = e->low & 0xffffffffu;
    if ((lo >> 24) != ((lo + e->range - 1) >> 24)) {
      e->bill_pend++;
    } else {
      billed = e->bill_pend + 1;
      e->bill_pend = 0;
    }
    pc_shift(e);
    e->range <<= 8;
  }
  return billed;
}
void pc_enc_finish(pc_enc_t *e) {
  for (uint64_t sb = 1ull << 32; sb; sb >>= 1) {
    const uint64_t x = (e->low | sb) & ~(sb - 1);
    if (sb < e->range && e->low <= x && x < e->low + e->range) {
      e->low = x;
      break;
    }
  }
  while (e->low != 0) pc_shift(e);
  if (e->have_cache) ob_put(e->out, (uint8_t)e->cache);
  for (; e->pending; e->pending--) ob_put(e->out, 0xff);
  e->have_cache = 0;
}
static uint32_t pc_byte(pc_dec_t *d) { return d->in < d->end ? *d->in++ : 0u; }   /* zeros past the end */
void pc_dec_init(pc_dec_t *d, const uint8_t *in, size_t n) {
  d->in = in;
  d->end = in + n;
  d->low = 0;
  for (int i = 0; i < 4; i++) d->low = d->low << 8 | pc_byte(d);
  d->range = 0xffffffffu;
}
int pc_dec_get(pc_dec_t *d, uint32_t r1) {
  const uint32_t r0 = d->range - r1;
  const int bin = d->low >= r0;
  if (bin) d->low -= r0;
  d->range = bin ? r1 : r0;
  if (d->range < (1u << 24)) {
    d->low = d->low << 8 | pc_byte(d);
    d->range <<= 8;
  }
  return bin;
}

/* ---------------------------------------------------------------- CABAC re-encoder (cabac_code.h) */
static int ilog2_u64(uint64_t x) { /* cabac_code.h:70-79 */
  int i = 0;
  if (x >> 32) { x >>= 32; i += 32; }
  if (x >> 16) { x >>= 16; i += 16; }
  if (x >> 8) { x >>= 8; i += 8; }
  if (x >> 4) { x >>= 4; i += 4; }
  if (x >> 2) { x >>= 2; i += 2; }
  if (x >> 1) { i += 1; }
  return i;
}

void cabac_enc_init(cabac_enc_t *c, obuf_t *out) {
  /* arithmetic_code<uint32_t, uint16_t, 0x200>, initial range (fixed_one/0x200)*0x1FE (cabac_code.h:30) */
  ac_enc_init(&c->e, out, 32, 16, 0x200, ((1ull << 31) / 0x200) * 0x1FE);
}
void cabac_enc_free(cabac_enc_t *c) { ac_enc_free(&c->e); }

size_t cabac_enc_put(cabac_enc_t *c, int symbol, uint8_t *state) { /* cabac_code.h:33-49 */
  int lps = symbol != (*state & 1);
  uint64_t range = c->e.range;
  int normalize = ilog2_u64(range / 0x100);
  int range_approx = (int)(range >> (normalize - 1));
  uint64_t r1 = (uint64_t)avr_lps_range[(range_approx & 0x180) + *state] << normalize;
  size_t ret = ac_enc_put(&c->e, lps, r1);
  *state = lps ? avr_mlps_state[127 - *state] : avr_mlps_state[128 + *state];
  return ret;
}
size_t cabac_enc_put_bypass(cabac_enc_t *c, int symbol) { /* cabac_code.h:52-54 */
  return ac_enc_put(&c->e, symbol, c->e.range / 2);
}
size_t cabac_enc_put_terminate(cabac_enc_t *c, int symbol) { /* cabac_code.h:57-67 */
  int normalize = ilog2_u64(c->e.range / 0x100);
  size_t ret = ac_enc_put(&c->e, symbol, 2ull << normalize);
  if (symbol) ac_enc_finish(&c->e);
  return ret;
}

/* ---------------------------------------------------------------- CABAC decoding engine (9.3) */
static inline uint32_t rd_bit(cabac_dec_t *d) {
  uint32_t b = 0;
  if (d->pos < d->nbits) b = (d->buf[d->pos >> 3] >> (7 - (d->pos & 7))) & 1;
  else d->overrun++;
  d->pos++;
  return b;
}
void cabac_dec_init(cabac_dec_t *d, const uint8_t *buf, size_t n) { /* 9.3.1.2 */
  d->buf = buf;
  d->nbits = n * 8;
  d->pos = 0;
  d->overrun = 0;
  d->range = 510;
  d->offset = 0;
  for (int i = 0; i < 9; i++) d->offset = (d->offset << 1) | rd_bit(d);
}
int cabac_dec_decision(cabac_dec_t *d, uint8_t *state) { /* 9.3.3.2.1 */
  uint32_t s = *state;
  uint32_t lps = avr_lps_range[((d->range >> 6) & 3) * 128 + s];
  int bin;
  d->range -= lps;
  if (d->offset >= d->range) {
    bin = !(s & 1);
    d->offset -= d->range;
    d->range = lps;
    *state = avr_mlps_state[127 - s];
  } else {
    bin = s & 1;
    *state = avr_mlps_state[128 + s];
  }
  while (d->range < 256) {
    d->range <<= 1;
    d->offset = (d->offset << 1) | rd_bit(d);
  }
  return bin;
}
int cabac_dec_bypass(cabac_dec_t *d) { /* 9.3.3.2.3 */
  d->offset = (d->offset << 1) | rd_bit(d);
  if (d->offset >= d->range) {
    d->offset -= d->range;
    return 1;
  }
  return 0;
}
int cabac_dec_terminate(cabac_dec_t *d) { /* 9.3.3.2.2.3 */
  d->range -= 2;
  if (d->offset >= d->range) return 1; /* no renormalisation; last bit read = rbsp_stop_one_bit */
  while (d->range < 256) {
    d->range <<= 1;
    d->offset = (d->offset << 1) | rd_bit(d);
  }
  return 0;
}

/* ---------------------------------------------------------------- op scripts (tests) */
/* Runs the same op scripts as oracle/ref_arith_driver.cpp.  ops = quads (op, a, b, c):
 *   's' sym pos neg (recoded), 'd' sym state (cabac), 'b' sym, 't' sym, 'f' finish.
 * kind 0 = recoded coder, 1 = CABAC coder, 2 = P-format coder.  Returns bytes written (or -1 if cap
 * too small). */
long avr_script_run(int kind, const int32_t *ops, size_t nops, uint8_t *out, size_t cap) {
  obuf_t o;
  ob_init(&o);
  if (kind == 2) { /* the P-format coder: 's' ops, 'f' ends the stream */
    pc_enc_t pc;
    pc_enc_init(&pc, &o);
    for (size_t i = 0; i < nops; i++) {
      const int32_t *q = ops + 4 * i;
      if (q[0] == 's') pc_enc_put(&pc, q[1], pc_p1(pc.range, q[2], q[3]));
    }
    pc_enc_finish(&pc);
    long n = pc.err ? -2 : (long)o.len;
    if (n >= 0 && o.len > cap) n = -1;
    else if (n >= 0) memcpy(out, o.data, o.len);
    ob_free(&o);
    return n;
  }
  ac_enc_t rc;
  cabac_enc_t cb;
  if (kind == 0) rc_enc_init(&rc, &o);
  else cabac_enc_init(&cb, &o);
  for (size_t i = 0; i < nops; i++) {
    const int32_t *q = ops + 4 * i;
    switch (q[0]) {
      case 's': ac_enc_put(&rc, q[1], rc_p1(rc.range, q[2], q[3])); break;
      case 'd': { uint8_t st = (uint8_t)q[2]; cabac_enc_put(&cb, q[1], &st); break; }
      case 'b': cabac_enc_put_bypass(&cb, q[1]); break;
      case 't': cabac_enc_put_terminate(&cb, q[1]); break;
      case 'f': if (kind == 0) ac_enc_finish(&rc); else ac_enc_finish(&cb.e); break;
      default: break;
    }
  }
  if (kind == 0) { ac_enc_finish(&rc); ac_enc_free(&rc); }
  else { ac_enc_finish(&cb.e); cabac_enc_free(&cb); }
  long n = (long)o.len;
  if (o.len > cap) n = -1;
  else memcpy(out, o.data, o.len);
  ob_free(&o);
  return n;
}

/* decode a recoded stream with the given (pos, neg) sequence; returns #symbols matching */
long avr_script_decode_recoded(const uint8_t *in, size_t n, const int32_t *ops, size_t nops) {
  ac_dec_t d;
  rc_dec_init(&d, in, n);
  long ok = 0;
  for (size_t i = 0; i < nops; i++) {
    const int32_t *q = ops + 4 * i;
    if (q[0] != 's') continue;
    if (ac_dec_get(&d, rc_p1(d.range, q[2], q[3])) != q[1]) return ok;
    ok++;
  }
  return ok;
}

/* decode a P-format stream with the given (pos, neg) sequence; returns #symbols matching */
long avr_script_decode_p(const uint8_t *in, size_t n, const int32_t *ops, size_t nops) {
  pc_dec_t d;
  pc_dec_init(&d, in, n);
  long ok = 0;
  for (size_t i = 0; i < nops; i++) {
    const int32_t *q = ops + 4 * i;
    if (q[0] != 's') continue;
    if (pc_dec_get(&d, pc_p1(d.range, q[2], q[3])) != q[1]) return ok;
    ok++;
  }
  return ok;
}

/* decode a CABAC stream produced from 'd'/'b'/'t' ops with the spec engine; returns #ops matching */
long avr_script_decode_cabac(const uint8_t *in, size_t n, const int32_t *ops, size_t nops) {
  cabac_dec_t d;
  cabac_dec_init(&d, in, n);
  long ok = 0;
  for (size_t i = 0; i < nops; i++) {
    const int32_t *q = ops + 4 * i;
    int s;
    if (q[0] == 'd') { uint8_t st = (uint8_t)q[2]; s = cabac_dec_decision(&d, &st); }
    else if (q[0] == 'b') s = cabac_dec_bypass(&d);
    else if (q[0] == 't') s = cabac_dec_terminate(&d) != 0;
    else continue;
    if (s != q[1]) return ok;
    ok++;
  }
  return ok;
}
