// SPS / PPS / slice header writer for synthetic streams (ITU-T H.264 7.3.2.1.1, 7.3.2.2, 7.3.3)
// and NAL emulation prevention (7.4.1).  A picture is one slice or several (equal MB runs).
#include "avr_synth.h"

namespace avr {
namespace {

class BitWriter {
 public:
  void u(uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) bit((v >> i) & 1);
  }
  void ue(uint32_t v) {
    uint32_t x = v + 1;
    int len = 0;
    while ((x >> len) > 1) len++;
    u(0, len);
    u(x, len + 1);
  }
  void se(int32_t v) { ue(v > 0 ? 2 * (uint32_t)v - 1 : 2 * (uint32_t)(-v)); }
  void bit(int b) {
    cur_ = (uint8_t)((cur_ << 1) | (b & 1));
    if (++n_ == 8) bytes.push_back(cur_), cur_ = 0, n_ = 0;
  }
  void align_ones() {
    while (n_) bit(1);
  }
  void trailing() {
    bit(1);
    while (n_) bit(0);
  }
  std::vector<uint8_t> bytes;

 private:
  uint8_t cur_ = 0;
  int n_ = 0;
};

void put_nal(std::vector<uint8_t>* out, int ref_idc, int type, const std::vector<uint8_t>& rbsp) {
  static const uint8_t sc[4] = {0, 0, 0, 1};
  out->insert(out->end(), sc, sc + 4);
  out->push_back((uint8_t)((ref_idc << 5) | type));
  int zeros = 0;
  for (uint8_t b : rbsp) {
    if (zeros >= 2 && b <= 3) {
      out->push_back(3);
      zeros = 0;
    }
    out->push_back(b);
    zeros = b == 0 ? zeros + 1 : 0;
  }
}

}  // namespace

void synth_write_parameter_sets(std::vector<uint8_t>* out, const avr_synth_params& p) {
  BitWriter s;
  const int profile = p.chroma_format_idc == 3 ? 244 : p.chroma_format_idc == 2 ? 122 : 100;
  s.u(profile, 8);
  s.u(0, 8);
  s.u(51, 8);            // level 5.1
  s.ue(0);               // sps id
  s.ue(p.chroma_format_idc);
  if (p.chroma_format_idc == 3) s.u(0, 1);
  s.ue(0);
  s.ue(0);               // 8-bit
  s.u(0, 1);
  s.u(0, 1);             // no scaling matrices
  s.ue(12);              // log2_max_frame_num = 16
  s.ue(2);               // pic_order_cnt_type 2
  s.ue(4);               // max_num_ref_frames
  s.u(0, 1);
  s.ue(p.mb_width - 1);
  const bool frames_only = p.structure == 0;
  s.ue((frames_only ? p.mb_height : p.mb_height / 2) - 1);   // pic_height_in_map_units_minus1
  s.u(frames_only ? 1 : 0, 1);                              // frame_mbs_only
  if (!frames_only) s.u(p.structure == 2 ? 1 : 0, 1);        // mb_adaptive_frame_field_flag
  s.u(1, 1);             // direct_8x8_inference (required without frame_mbs_only)
  s.u(0, 1);             // no cropping
  s.u(0, 1);             // no VUI
  s.trailing();
  put_nal(out, 3, 7, s.bytes);
  BitWriter q;
  q.ue(0);
  q.ue(0);
  q.u(1, 1);             // CABAC
  q.u(0, 1);
  q.ue(0);               // one slice group
  q.ue((uint32_t)(p.num_ref_idx_l0 > 0 ? p.num_ref_idx_l0 - 1 : 0));
  q.ue((uint32_t)(p.num_ref_idx_l1 > 0 ? p.num_ref_idx_l1 - 1 : 0));
  q.u(0, 1);
  q.u(0, 2);
  q.se(0);               // pic_init_qp 26
  q.se(0);
  q.se(0);
  q.u(1, 1);             // deblocking_filter_control_present
  q.u(0, 1);
  q.u(0, 1);
  q.u(p.transform_8x8_mode ? 1 : 0, 1);
  q.u(0, 1);
  q.se(0);
  q.trailing();
  put_nal(out, 3, 8, q.bytes);
}

void synth_write_slice(std::vector<uint8_t>* out, const avr_synth_params& p, int slice_type, int index,
                       int structure, bool second_field, int first_mb, const uint8_t* payload,
                       size_t payload_len) {
  // every I picture is an IDR picture; the second field of an IDR frame is a non-IDR I field
  const bool idr = slice_type == 2 && !second_field;
  const bool field = structure == AVR_STRUCT_TOP_FIELD || structure == AVR_STRUCT_BOTTOM_FIELD;
  BitWriter h;
  h.ue((uint32_t)(structure == AVR_STRUCT_MBAFF ? first_mb / 2 : first_mb));   // first_mb_in_slice (pairs in MBAFF)
  h.ue((uint32_t)slice_type + 5);
  h.ue(0);                       // pps id
  // frame_num: an IDR frame's is 0, and both fields of a frame carry the same one
  h.u(slice_type == 2 ? 0 : (uint32_t)(index & 0xffff), 16);
  if (p.structure != 0) {
    h.u(field ? 1 : 0, 1);       // field_pic_flag
    if (field) h.u(structure == AVR_STRUCT_BOTTOM_FIELD ? 1 : 0, 1);   // bottom_field_flag
  }
  if (idr) h.ue((uint32_t)(index & 0xffff));
  if (slice_type == 1) h.u(1, 1);           // direct_spatial_mv_pred_flag
  if (slice_type != 2) {
    h.u(1, 1);                                // num_ref_idx_active_override_flag
    h.ue((uint32_t)(p.num_ref_idx_l0 > 0 ? p.num_ref_idx_l0 - 1 : 0));
    if (slice_type == 1) h.ue((uint32_t)(p.num_ref_idx_l1 > 0 ? p.num_ref_idx_l1 - 1 : 0));
    h.u(0, 1);                                // ref_pic_list_modification_flag_l0
    if (slice_type == 1) h.u(0, 1);
  }
  if (idr) {
    h.u(0, 1);
    h.u(0, 1);
  } else {
    h.u(0, 1);                                // adaptive_ref_pic_marking_mode_flag
  }
  if (slice_type != 2) h.ue(0);             // cabac_init_idc
  h.se(p.slice_qp - 26);
  h.ue(1);                                    // disable_deblocking_filter_idc
  h.align_ones();                             // cabac_alignment_one_bit
  std::vector<uint8_t> rbsp = h.bytes;
  rbsp.insert(rbsp.end(), payload, payload + payload_len);  // ends with the stop bit + zero bits
  put_nal(out, 2, idr ? 5 : 1, rbsp);
}

}  // namespace avr
