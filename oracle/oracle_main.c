/*
 * Oracle CLI (mirrors recode.cpp:1627-1659 main).  TEST INFRASTRUCTURE ONLY.
 *
 *   recode_oracle compress   [-p|-p32|-c] <input> [output]
 *   recode_oracle decompress           <input> [output]
 *   recode_oracle roundtrip  [-p|-p32|-c] <input> [output]
 *   recode_oracle slices          <input>          per-slice parse / regeneration report
 *   recode_oracle pieces          <input>          the parallel model's split slices (AVR_SPLIT_BYTES),
 *                                                  each piece decompressed on its own, compared
 *
 * -p selects the parallel model (fresh model per slice) on arithmetic_code<uint64_t, uint8_t>, -p32 the
 * parallel model on the P-format coder, -c the reference model in chains of 16 coded slices (a
 * fresh model before every 16th: avrecode-amd:R16); default is the reference model.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "avr_oracle.h"

static uint8_t *read_file(const char *path, size_t *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *b = (uint8_t *)malloc((size_t)sz + 1);
  if (fread(b, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); free(b); return NULL; }
  fclose(f);
  *n = (size_t)sz;
  return b;
}
static int write_out(const char *path, const uint8_t *p, size_t n) {
  FILE *f = path ? fopen(path, "wb") : stdout;
  if (!f) return -1;
  fwrite(p, 1, n, f);
  if (path) fclose(f);
  return 0;
}
static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static int cmd_slices(const uint8_t *file, size_t n) {
  avr_nal_t *nals;
  int nn = avr_demux(file, n, &nals);
  if (nn < 0) { fprintf(stderr, "demux failed\n"); return 1; }
  avr_param_sets_t *ps = (avr_param_sets_t *)calloc(1, sizeof(*ps));
  int ok = 0, bad = 0, idx = 0, x264_build = -1;
  for (int i = 0; i < nn; i++) {
    const uint8_t *nal = file + nals[i].offset;
    size_t sz = nals[i].size;
    int type = nal[0] & 0x1f;
    uint8_t *rbsp = (uint8_t *)malloc(sz);
    size_t rl = avr_nal_unescape(nal + 1, sz - 1, rbsp);
    if (type == 6) { int b = avr_parse_sei_x264_build(rbsp, rl); if (b > 0) x264_build = b; }
    if (type == 7) avr_parse_sps(ps, rbsp, rl);
    else if (type == 8) avr_parse_pps(ps, rbsp, rl);
    else if (type == 1 || type == 5) {
      avr_slice_hdr_t h;
      if (avr_parse_slice_header(ps, rbsp, rl, type, (nal[0] >> 5) & 3, &h) == 0) {
        h.x264_build = x264_build;
        size_t bits = avr_rbsp_bit_length(rbsp, rl);
        size_t size = (bits + 7) / 8 - h.cabac_start;
        obuf_t regen;
        size_t bins = 0, endpos = 0;
        int r = avr_cabac_regenerate(&h, rbsp + h.cabac_start, rl - h.cabac_start, &regen, &bins, &endpos);
        /* the stop bit must be the last bit read, i.e. bit (bits) of the RBSP = the rbsp_stop_one_bit */
        size_t stop_bit = bits - 8 * h.cabac_start;
        int match = r == 0 && endpos - 1 == stop_bit;
        size_t cmp = regen.len < size ? regen.len : size;
        int prefix_ok = r == 0 && cmp > 1 && memcmp(regen.data, rbsp + h.cabac_start, cmp - 1) == 0;
        /* what the decompressor would restore (recode.cpp:1345-1356, 1503-1505) */
        int restored = 0;
        if (r == 0 && size > 1) {
          if (regen.len && regen.data[regen.len - 1] == 0x80) regen.len--;
          if ((int)(size & 1) != (int)(regen.len & 1)) ob_put(&regen, rbsp[h.cabac_start + size - 1]);
          else if (regen.len) regen.data[regen.len - 1] = rbsp[h.cabac_start + size - 1];
          restored = regen.len == size && !memcmp(regen.data, rbsp + h.cabac_start, size);
        }
        printf("slice %d type %d first_mb %d qp %d idc %d size %zu bins %zu walk %d stop %s(%ld) prefix %s restored %s escaped %d\n",
               idx, h.slice_type, h.first_mb, h.slice_qp, h.cabac_init_idc, size, bins, r,
               match ? "ok" : "off", (long)(endpos - 1) - (long)stop_bit, prefix_ok ? "ok" : "BAD",
               restored ? "ok" : "BAD", sz - 1 != rl);
        if (restored) ok++;
        else bad++;
        ob_free(&regen);
        idx++;
      }
    }
    free(rbsp);
  }
  printf("slices ok %d bad %d\n", ok, bad);
  free(ps);
  free(nals);
  return bad != 0;
}

/* ~h264_model (recode.cpp:634-655): the bills to stderr, nonzero entries only, by CodingType
 * name; once for the compressor's model(s) (re-coded bytes), once for the decompressor's (CABAC
 * bytes), summed over the fresh per-slice models in the parallel mode. */
static const char *const billing_names[6] = {"PIP_UNKNOWN", "PIP_UNREACHABLE", "PIP_SIGNIFICANCE_MAP",
                                            "PIP_SIGNIFICANCE_EOB", "PIP_SIGNIFICANCE_NZ", "PIP_RESIDUALS"};
static void print_bill(const char *title, const size_t *b) {
  int first = 1;
  for (int i = 0; i < 6; i++) {
    if (!b[i]) continue;
    if (first) fprintf(stderr, "%s\n=============\n", title);
    first = 0;
    fprintf(stderr, "%s : %ld\n", billing_names[i], (long)b[i]);
  }
}
static void print_bills(const size_t *bill, const size_t *cabac_bill) {
  print_bill("Avrecode Bill", bill);
  print_bill("CABAC Bill", cabac_bill);
}

int main(int argc, char **argv) {
  int mode = AVR_MODE_R;
  int a = 1;
  if (argc < 3) {
    fprintf(stderr, "Usage: %s [compress|decompress|roundtrip|slices] [-p|-p32|-c] <input> [output]\n", argv[0]);
    return 1;
  }
  const char *cmd = argv[a++];
  if (a < argc && !strcmp(argv[a], "-p")) { mode = AVR_MODE_P; a++; }
  else if (a < argc && !strcmp(argv[a], "-p32")) { mode = AVR_MODE_P32; a++; }
  else if (a < argc && !strcmp(argv[a], "-c")) { mode = AVR_MODE_C; a++; }
  if (a >= argc) return 1;
  const char *in = argv[a++];
  const char *outp = a < argc ? argv[a] : NULL;
  size_t n;
  uint8_t *file = read_file(in, &n);
  if (!file) { fprintf(stderr, "Failed to open file: %s\n", in); return 1; }
  if (!strcmp(cmd, "slices")) return cmd_slices(file, n);
  if (!strcmp(cmd, "pieces")) {   /* the parallel model's long-slice split, piece by piece */
    int ns = 0, np = 0;
    int bad = avr_check_pieces(file, n, avr_oracle_split_bytes(), &ns, &np);
    printf("split slices %d pieces %d mismatches %d\n", ns, np, bad);
    return bad != 0;
  }
  if (!strcmp(cmd, "compress")) {
    uint8_t *o; size_t on;
    if (avr_compress(file, n, mode, &o, &on)) { fprintf(stderr, "compress failed\n"); return 1; }
    return write_out(outp, o, on);
  }
  if (!strcmp(cmd, "decompress")) {
    uint8_t *o; size_t on;
    int r = avr_decompress(file, n, &o, &on);
    if (r) { fprintf(stderr, "decompress failed (%d)\n", r); return 1; }
    return write_out(outp, o, on);
  }
  if (!strcmp(cmd, "roundtrip")) { /* recode.cpp:1594-1624 */
    uint8_t *c, *d;
    size_t cn, dn;
    double t0 = now_s();
    if (avr_compress(file, n, mode, &c, &cn)) { fprintf(stderr, "compress failed\n"); return 1; }
    double t1 = now_s();
    avr_stats_t st = avr_last_stats;
    size_t bill[8];
    memcpy(bill, avr_last_bill, sizeof(bill));
    int r = avr_decompress(c, cn, &d, &dn);
    double t2 = now_s();
    if (r || dn != n || memcmp(d, file, n)) {
      fprintf(stderr, "Compress-decompress roundtrip failed. (%d)\n", r);
      return 1;
    }
    if (outp) write_out(outp, c, cn);
    avr_pb_block_t *blocks;
    int nb = avr_pb_parse(c, cn, &blocks);
    size_t block_bytes = 0;
    for (int i = 0; i < nb; i++) block_bytes += blocks[i].literal_len + blocks[i].cabac_len;
    printf("Compress-decompress roundtrip succeeded:\n");
    printf(" compression ratio: %g%%\n", cn * 100.0 / n);
    printf(" protobuf overhead: %g%%\n", (cn - block_bytes) * 100.0 / cn);
    printf(" slices %zu coded %zu skipped %zu payload %zu recoded %zu bins %zu\n", st.slices, st.coded_slices,
           st.skipped_slices, st.payload_bytes, st.recoded_bytes, st.bins);
    printf(" compress %.3fs decompress %.3fs (%.2f MB/s roundtrip)\n", t1 - t0, t2 - t1, n / 1e6 / (t2 - t0));
    print_bills(bill, avr_last_cabac_bill);
    return 0;
  }
  fprintf(stderr, "Unknown command: %s\n", cmd);
  return 1;
}
