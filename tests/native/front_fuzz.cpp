// Host-only mutation harness for the recode path's front end (avr_front.cpp): the demuxer (MP4 /
// Annex-B), the parameter-set / slice-header walk (StreamParser) and the recode.proto reader
// (pb_parse), built with AddressSanitizer + UndefinedBehaviorSanitizer by
// tests/test_front_sanitizers.py.  The reference reads these through libavformat / libavcodec and
// protobuf (recode.cpp:73-135, 1312-1336); every caller of this build runs them before any device
// work, on bytes it does not control.
//
//   front_fuzz <iterations> <seed> <file>...
//
// Each iteration takes one input, applies 1-8 random mutations (byte flips, overwrites with
// boundary values, truncation, duplication of a span, insertion of a start code) and runs the
// three readers on the result.  Whatever a reader accepts must describe bytes inside its input.
// Exit status 0 = no sanitizer report and no broken invariant.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "../../avrecode_amd/csrc/avr_front.h"

namespace {

std::vector<uint8_t> read_file(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

void mutate(std::vector<uint8_t>* d, std::mt19937_64& rng) {
  const int n = 1 + (int)(rng() % 8);
  for (int k = 0; k < n && !d->empty(); k++) {
    const size_t at = rng() % d->size();
    switch (rng() % 6) {
      case 0: (*d)[at] ^= (uint8_t)(1u << (rng() % 8)); break;
      case 1: {
        static const uint8_t v[] = {0x00, 0x01, 0x7f, 0x80, 0xff};
        (*d)[at] = v[rng() % 5];
        break;
      }
      case 2: d->resize(at); break;
      case 3: {  // a 32-bit field set to a boundary value (box sizes, counts, offsets)
        static const uint32_t v[] = {0u, 1u, 7u, 8u, 0x7fffffffu, 0x80000000u, 0xffffffffu};
        const uint32_t x = v[rng() % 7];
        for (int b = 0; b < 4 && at + b < d->size(); b++) (*d)[at + b] = (uint8_t)(x >> (24 - 8 * b));
        break;
      }
      case 4: {  // duplicate a span in place
        const size_t len = std::min<size_t>(1 + rng() % 64, d->size() - at);
        std::vector<uint8_t> span(d->begin() + at, d->begin() + at + len);
        d->insert(d->begin() + at, span.begin(), span.end());
        break;
      }
      default: {  // an Annex-B start code
        static const uint8_t sc[] = {0, 0, 1};
        d->insert(d->begin() + at, sc, sc + 3);
        break;
      }
    }
  }
}

int check(const std::vector<uint8_t>& d) {
  const uint8_t* p = d.data();
  const size_t n = d.size();
  std::vector<avr::NalRef> nals;
  if (avr::demux(p, n, &nals)) {
    avr::StreamParser sp;
    for (const avr::NalRef& r : nals) {
      if (r.offset > n || r.size > n - r.offset) {
        fprintf(stderr, "demux: NAL [%zu, +%zu) outside %zu bytes\n", r.offset, r.size, n);
        return 1;
      }
      avr::SliceInfo s;
      if (sp.next(p + r.offset, r.size, &s)) {
        if (s.h.cabac_start > s.rbsp.size() || s.size > s.rbsp.size() - s.h.cabac_start ||
            s.read_limit < s.size) {
          fprintf(stderr, "parser: slice payload [%zu, +%zu) limit %zu outside rbsp %zu\n", s.h.cabac_start,
                  s.size, s.read_limit, s.rbsp.size());
          return 1;
        }
        volatile uint8_t sink = 0;
        for (size_t i = 0; i < s.size; i++) sink ^= s.payload()[i];
        (void)sink;
      }
    }
  }
  std::vector<avr::PbBlock> blocks;
  std::string version;
  if (avr::pb_parse(p, n, &blocks, &version)) {
    std::vector<uint8_t> again;
    for (const avr::PbBlock& b : blocks) {
      if ((b.has_literal && (b.literal < p || b.literal + b.literal_len > p + n)) ||
          (b.has_cabac && (b.cabac < p || b.cabac + b.cabac_len > p + n))) {
        fprintf(stderr, "pb_parse: block bytes outside the input\n");
        return 1;
      }
      avr::pb_put_block(&again, b);
    }
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <iterations> <seed> <file>...\n", argv[0]);
    return 2;
  }
  const long iters = strtol(argv[1], nullptr, 10);
  std::mt19937_64 rng(strtoull(argv[2], nullptr, 10));
  std::vector<std::vector<uint8_t>> inputs;
  for (int i = 3; i < argc; i++) {
    inputs.push_back(read_file(argv[i]));
    if (inputs.back().empty()) {
      fprintf(stderr, "cannot read %s\n", argv[i]);
      return 2;
    }
    if (check(inputs.back())) return 1;   // the unmutated input first
  }
  for (long it = 0; it < iters; it++) {
    std::vector<uint8_t> d = inputs[rng() % inputs.size()];
    mutate(&d, rng);
    if (check(d)) {
      fprintf(stderr, "iteration %ld\n", it);
      return 1;
    }
  }
  printf("front_fuzz: %ld mutated inputs, no finding\n", iters);
  return 0;
}
