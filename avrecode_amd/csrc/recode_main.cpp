// recode CLI (recode.cpp:1627-1659): recode [compress|decompress|roundtrip] [-p|-p32|-c] <input> [output]
//   -p    parallel model (fresh model per slice; slices independent) on the reference's
//         arithmetic_code<uint64_t, uint8_t>; default = reference model.
//   -p32  parallel model on the optional 32-bit P32 coder (avrecode-amd:P32 containers).
//   -c    the reference model in chains of 16 coded slices (avrecode-amd:R16 containers).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "../../include/avrecode.h"

static bool read_file(const char* p, std::vector<uint8_t>* v) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return false;
  v->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

// ~h264_model (recode.cpp:634-655): the bills to stderr, nonzero entries by CodingType name -- the
// compressor's (re-coded bytes) and the decompressor's (CABAC bytes), summed over the file.
static const char* const kBillingNames[6] = {"PIP_UNKNOWN", "PIP_UNREACHABLE", "PIP_SIGNIFICANCE_MAP",
                                             "PIP_SIGNIFICANCE_EOB", "PIP_SIGNIFICANCE_NZ", "PIP_RESIDUALS"};
static void print_bill(const char* title, const uint64_t* b) {
  bool first = true;
  for (int i = 0; i < 6; i++) {
    if (!b[i]) continue;
    if (first) std::cerr << title << "\n=============\n";
    first = false;
    std::cerr << kBillingNames[i] << " : " << b[i] << "\n";
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "Usage: " << argv[0] << " [compress|decompress|roundtrip] [-p|-p32|-c] <input> [output]" << std::endl;
    return 1;
  }
  std::string cmd = argv[1];
  int a = 2, model = AVR_MODEL_REFERENCE;
  if (!strcmp(argv[a], "-p")) model = AVR_MODEL_PARALLEL, a++;
  else if (!strcmp(argv[a], "-p32")) model = AVR_MODEL_PARALLEL32, a++;
  else if (!strcmp(argv[a], "-c")) model = AVR_MODEL_CHAINED, a++;
  if (a >= argc) return 1;
  const char* input = argv[a++];
  const char* output = a < argc ? argv[a] : nullptr;
  std::vector<uint8_t> in;
  if (!read_file(input, &in)) {
    std::cerr << "Failed to open file: " << input << std::endl;
    return 1;
  }
  avr_ctx* ctx = nullptr;
  if (avr_create(0, &ctx) != AVR_OK) {
    std::cerr << "No usable MI355X / HIP device" << std::endl;
    return 1;
  }
  uint8_t* out = nullptr;
  size_t out_len = 0;
  int r;
  if (cmd == "compress") {
    r = avr_compress_file(ctx, in.data(), in.size(), model, &out, &out_len);
  } else if (cmd == "decompress") {
    r = avr_decompress_file(ctx, in.data(), in.size(), &out, &out_len);
  } else if (cmd == "roundtrip") {
    avr_file_stats st;
    r = avr_roundtrip_file(ctx, in.data(), in.size(), model, &out, &out_len, &st);
    if (r == AVR_OK) {
      std::cout << "Compress-decompress roundtrip succeeded:" << std::endl;
      std::cout << " compression ratio: " << out_len * 100.0 / in.size() << "%" << std::endl;
      std::cout << " slices " << st.slices << " coded " << st.coded_slices << " skipped " << st.skipped_slices
                << " payload " << st.payload_bytes << " recoded " << st.recoded_bytes << std::endl;
      std::cout << " compress " << st.compress_s << "s decompress " << st.decompress_s << "s" << std::endl;
      print_bill("Avrecode Bill", st.bill);
      print_bill("CABAC Bill", st.cabac_bill);
    } else {
      std::cerr << "Compress-decompress roundtrip failed: " << avr_last_error(ctx) << std::endl;
      avr_destroy(ctx);
      return 1;
    }
    if (!output) {
      avr_free(out);
      avr_destroy(ctx);
      return 0;
    }
  } else {
    std::cerr << "Unknown command: " << cmd << std::endl;
    return 1;
  }
  if (r != AVR_OK) {
    std::cerr << "Exception: " << avr_last_error(ctx) << " (" << r << ")" << std::endl;
    avr_destroy(ctx);
    return 1;
  }
  if (output) {
    std::ofstream f(output, std::ios::binary);
    f.write((const char*)out, (std::streamsize)out_len);
  } else {
    fwrite(out, 1, out_len, stdout);
  }
  avr_free(out);
  avr_destroy(ctx);
  return 0;
}
