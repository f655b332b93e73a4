// Drives the reference's generic arithmetic coder, compiled as-is from
// /root/reference/arithmetic_code.h (nothing copied), to produce golden vectors for the oracle.
// TEST INFRASTRUCTURE ONLY: built into oracle/_ref/ by `make -C oracle ref`.
//
// stdin:  line 1  "recoded" | "cabac"
//         cabac:  line 2 = 512 LPS-range bytes (FFmpeg layout [q*128 + state]) used to form r1 the
//                 way cabac_code.h:35-45 does; the state byte of each op is given explicitly.
//         ops, one per line:
//           recoded: "s <symbol> <pos> <neg>"          put(symbol, (range/(pos+neg))*pos)  (recode.cpp:816-820)
//           cabac:   "d <symbol> <state>"               CABAC decision (cabac_code.h:33-49 translation)
//                    "b <symbol>"                       bypass (range/2, cabac_code.h:52-54)
//                    "t <symbol>"                       terminate (2<<normalize, cabac_code.h:57-67)
//         "f" = finish
// stdout: the emitted bytes as hex, then (recoded only) a decode check line "decode ok|mismatch".
#include <cstdint>
#include <cstdio>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "arithmetic_code.h"

static int log2_u64(uint64_t x) {
  int i = 0;
  while (x >>= 1) i++;
  return i;
}

int main() {
  std::string kind;
  std::cin >> kind;
  std::vector<uint8_t> out;
  if (kind == "recoded") {
    typedef arithmetic_code<uint64_t, uint8_t> recoded_code;  // recode.cpp:315-316
    std::vector<int> syms, poss, negs;
    {
      auto enc = make_encoder<recoded_code>(&out);
      std::string op;
      while (std::cin >> op) {
        if (op == "s") {
          int s, p, n;
          std::cin >> s >> p >> n;
          enc.put(s, [p, n](uint64_t range) { return (range / (uint64_t)(p + n)) * (uint64_t)p; });
          syms.push_back(s);
          poss.push_back(p);
          negs.push_back(n);
        } else if (op == "f") {
          enc.finish();
        }
      }
    }
    for (uint8_t b : out) printf("%02x", b);
    printf("\n");
    auto dec = make_decoder<recoded_code>(out);
    for (size_t i = 0; i < syms.size(); i++) {
      int p = poss[i], n = negs[i];
      int s = dec.get([p, n](uint64_t range) { return (range / (uint64_t)(p + n)) * (uint64_t)p; });
      if (s != syms[i]) {
        printf("decode mismatch %zu\n", i);
        return 1;
      }
    }
    printf("decode ok\n");
    return 0;
  }
  if (kind == "cabac") {
    std::vector<int> lps(512);
    for (int i = 0; i < 512; i++) std::cin >> lps[i];
    typedef arithmetic_code<uint32_t, uint16_t, 0x200> cabac_code;  // cabac_code.h:18-24
    auto it = std::back_inserter(out);
    cabac_code::encoder<decltype(it), uint8_t> e(it, (cabac_code::fixed_one / 0x200) * 0x1FE);
    std::string op;
    while (std::cin >> op) {
      if (op == "d") {
        int s, state;
        std::cin >> s >> state;
        bool is_lps = (s != (state & 1));
        e.put(is_lps, [&](uint32_t range) {
          int normalize = log2_u64(range / 0x100);
          int range_approx = int(range >> (normalize - 1));
          uint32_t r = (uint32_t)lps[(range_approx & 0x180) + state];
          return r << normalize;
        });
      } else if (op == "b") {
        int s;
        std::cin >> s;
        e.put(s, [](uint32_t range) { return range / 2; });
      } else if (op == "t") {
        int s;
        std::cin >> s;
        e.put(s, [](uint32_t range) { return uint32_t(2) << log2_u64(range / 0x100); });
        if (s) e.finish();
      } else if (op == "f") {
        e.finish();
      }
    }
    e.finish();
    for (uint8_t b : out) printf("%02x", b);
    printf("\n");
    return 0;
  }
  return 2;
}
