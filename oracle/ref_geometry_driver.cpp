// Drives the reference's scan geometry (recode.cpp:233-471: r_scan8, scan_8, reverse_scan_8, the
// zigzag tables, test_reverse_scan8, get_neighbor_sub_mb), compiled from the reference's own source
// where it lies: `make -C oracle ref` cuts those lines out of /root/reference/recode.cpp into
// oracle/_ref/recode_geometry.inc (git-ignored; nothing is copied into the repository) and this
// file includes them behind the standard headers and the reference's arithmetic_code.h, which is
// all they need (no fork header, no stand-in).
// TEST INFRASTRUCTURE ONLY: output feeds tests/golden/make_geometry_golden.py.
//
// stdout: one JSON object
//   {"test_reverse_scan8": r, "scan_8": [...], "zigzag16": [...], "unzigzag16": [...],
//    "zigzag64": [...], "unzigzag64": [...],
//    "neighbors": [[above, size, scan8_index, mb_x, mb_y, ok, out_mb_x, out_mb_y, out_scan8], ...]}
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <stdexcept>
#include <tuple>
#include <vector>

#include "arithmetic_code.h"
#include "_ref/recode_geometry.inc"

template <size_t N>
static void dump(const char* name, const uint8_t (&t)[N]) {
  printf("\"%s\": [", name);
  for (size_t i = 0; i < N; i++) printf("%s%d", i ? ", " : "", t[i]);
  printf("],\n");
}

int main() {
  printf("{\"test_reverse_scan8\": %d,\n", test_reverse_scan8());
  dump("scan_8", scan_8);
  dump("zigzag16", zigzag16);
  dump("unzigzag16", unzigzag16);
  dump("zigzag64", zigzag64);
  dump("unzigzag64", unzigzag64);
  printf("\"neighbors\": [");
  static const int sizes[] = {4, 8, 15, 16, 64};
  bool first = true;
  for (int above = 0; above < 2; above++)
    for (int size : sizes)
      for (int idx = 0; idx < 51; idx++)
        for (int y = 0; y < 2; y++)
          for (int x = 0; x < 2; x++) {
            CoefficientCoord in{x, y, idx, 0}, out{-1, -1, -1, -1};
            const bool ok = get_neighbor_sub_mb(above != 0, size, in, &out);
            printf("%s\n [%d, %d, %d, %d, %d, %d, %d, %d, %d]", first ? "" : ",", above, size, idx, x, y, ok ? 1 : 0,
                   out.mb_x, out.mb_y, out.scan8_index);
            first = false;
          }
  printf("\n]}\n");
  return 0;
}
