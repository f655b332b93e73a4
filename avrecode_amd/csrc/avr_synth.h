// Synthetic H.264 CABAC streams for benchmarks: the device generator (avr_kernels.hip, generate
// mode) produces slice_data(); this writes SPS/PPS and slice headers around it (Annex-B).
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/avrecode.h"

namespace avr {
void synth_write_parameter_sets(std::vector<uint8_t>* out, const avr_synth_params& p);
// slice_type: this slice's type (avr_synth_params.gop_length may make it differ from p.slice_type);
// index: the frame's number (frame_num / idr_pic_id); structure: AVR_STRUCT_* of the picture;
// second_field: the picture is the second field of its frame (of an I frame: a non-IDR I field);
// first_mb: the first macroblock's address
void synth_write_slice(std::vector<uint8_t>* out, const avr_synth_params& p, int slice_type, int index,
                       int structure, bool second_field, int first_mb, const uint8_t* payload,
                       size_t payload_len);
}  // namespace avr
