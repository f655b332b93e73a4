// Host front end of the recode path: what recode.cpp obtains from FFmpeg's demuxer and H.264
// headers parser (av_decoder, recode.cpp:73-135), the block segmentation
// (find_next_coded_block_and_emit_literal, recode.cpp:1275-1297) and the recode.proto container.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace avr {

struct Sps {
  bool valid = false;
  int profile_idc = 0, chroma_format_idc = 1, separate_colour_plane = 0;
  int log2_max_frame_num = 4, poc_type = 0, log2_max_poc_lsb = 4, delta_pic_order_always_zero = 0;
  int frame_mbs_only = 1, mb_aff = 0, direct_8x8_inference = 0, mb_width = 0, mb_height = 0;
};
struct Pps {
  bool valid = false;
  int sps_id = 0, entropy_coding_mode = 0, bottom_field_pic_order_present = 0, num_slice_groups = 1;
  int num_ref_idx_default[2] = {1, 1}, weighted_pred = 0, weighted_bipred_idc = 0, pic_init_qp = 26;
  int deblocking_filter_control_present = 0, redundant_pic_cnt_present = 0, transform_8x8_mode = 0;
};

struct SliceHeader {
  int nal_unit_type = 0, nal_ref_idc = 0, first_mb = 0, slice_type = 0, pps_id = 0, frame_num = 0;
  int field_pic = 0, bottom_field = 0, mbaff = 0, idr_pic_id = 0, poc_lsb = 0, num_ref_idx[2] = {0, 0}, cabac_init_idc = -1;
  int slice_qp = 26, chroma_array_type = 1, transform_8x8_mode = 0, direct_8x8_inference = 0;
  int mb_width = 0, mb_height = 0, x264_build = -1, entropy_coding_mode = 0;
  size_t cabac_start = 0;   // byte offset of slice_data() in the RBSP
  bool supported = false;
};

// A CABAC slice as FFmpeg would hand it to init_decoder (recode.cpp:143).
struct SliceInfo {
  SliceHeader h;
  int picture_id = 0;
  size_t nal_offset = 0, nal_size = 0;   // escaped NAL in the file
  std::vector<uint8_t> rbsp;             // unescaped NAL payload after the header byte (owned), or
  const uint8_t* view = nullptr;         //   these view_len bytes of the parsed buffer when the NAL
  size_t view_len = 0;                   //   has no emulation-prevention bytes (StreamParser views)
  size_t size = 0;                       // init_decoder size
  size_t read_limit = 0;                 // bytes a decoder may read from the payload start
  bool verbatim = false;                 // the NAL has no emulation-prevention bytes: the payload
                                         //   is the file's bytes at file_payload_offset()
  const uint8_t* rbsp_data() const { return view ? view : rbsp.data(); }
  size_t rbsp_size() const { return view ? view_len : rbsp.size(); }
  const uint8_t* payload() const { return rbsp_data() + h.cabac_start; }
  void own() {   // copy a view (before writing to rbsp)
    if (view) rbsp.assign(view, view + view_len), view = nullptr, view_len = 0;
  }
  uint64_t file_payload_offset() const { return verbatim ? nal_offset + 1 + h.cabac_start : ~(uint64_t)0; }
};

struct NalRef {
  size_t offset, size;
};

// MP4 (avcC) or Annex-B; returns false on a malformed container.
// Byte ranges [first, second) of a buffer, sorted, known to hold no 0x00 and no 0x03 byte (the
// decompressor's surrogate fill, read_packet's stream): no start code and no emulation-prevention
// byte can begin, end or lie in them, so the Annex-B scan and the emulation-prevention check step
// over them instead of reading them.
typedef std::vector<std::pair<size_t, size_t>> SkipRanges;
bool demux(const uint8_t* file, size_t n, std::vector<NalRef>* nals, const SkipRanges* skips = nullptr);
bool is_mp4(const uint8_t* file, size_t n);
// The video track's layout in an MP4 file: the avcC parameter sets and every sample's (offset,
// size) in decode order, from the moov box's sample tables -- what the mov demuxer knows before
// its first packet.  Returns 1, 0 when no complete moov box lies within [0, n) (a prefix of a
// moov-last file), -1 for a malformed one.  Samples may lie past n (a moov-first file's prefix).
struct Mp4Layout {
  std::vector<NalRef> param_sets, samples;
  int len_size = 4;
};
int mp4_layout(const uint8_t* file, size_t n, Mp4Layout* layout);
// the length-prefixed NAL units of one sample
void mp4_sample_nals(const uint8_t* file, const NalRef& sample, int len_size, std::vector<NalRef>* nals);

// Stateful walk over a NAL sequence (parameter sets, x264 SEI, picture boundaries).
class StreamParser {
 public:
  // Returns true and fills *s when the NAL is a CABAC slice FFmpeg would decode.  views: a slice
  // NAL without emulation-prevention bytes is not copied (SliceInfo::view points into nal, which
  // must outlive *s).
  bool next(const uint8_t* nal, size_t n, SliceInfo* s, bool views = false);
  // the NALs passed to next() lie in base[...] with these skip ranges (demux's)
  void set_skips(const uint8_t* base, const SkipRanges* skips) { skip_base_ = base, skips_ = skips; }

 private:
  bool nal_has_epb(const uint8_t* nal, size_t n) const;
  const uint8_t* skip_base_ = nullptr;
  const SkipRanges* skips_ = nullptr;
  Sps sps_[32];
  Pps pps_[256];
  int x264_build_ = -1;
  bool have_prev_ = false;
  SliceHeader prev_;
  int picture_id_ = 0;
  bool second_field_ = false;   // the current picture is the second field of a pair
};

// recode.proto
struct PbBlock {
  bool has_size = false, has_literal = false, has_skip = false, has_cabac = false, has_parity = false,
       has_last_byte = false;
  int64_t size = 0;
  bool skip_coded = false, length_parity = false;
  const uint8_t* literal = nullptr;
  size_t literal_len = 0;
  const uint8_t* cabac = nullptr;
  size_t cabac_len = 0;
  std::string last_byte;
  // field 16, this library's own (not in recode.proto): the parallel model's long-slice split of a
  // coded block (avr_api.cpp "seams"; zlib, the layout oracle/avr_oracle.h avr_seams_encode names)
  bool has_seams = false;
  const uint8_t* seams = nullptr;
  size_t seams_len = 0;
};
void pb_put_block(std::vector<uint8_t>* o, const PbBlock& b);
// The same bytes written into a buffer sized beforehand: pb_block_size(b) bytes at o + at (returns
// at + that).  The literal and cabac fields' bytes are left to the caller as copy jobs (dst offset
// in o, source, length) when copies is given, else copied here.
struct PbCopy {
  size_t dst;
  const uint8_t* src;
  size_t len;
};
size_t pb_block_size(const PbBlock& b);
size_t pb_write_block(uint8_t* o, size_t at, const PbBlock& b, std::vector<PbCopy>* copies);
void pb_put_metadata_version(std::vector<uint8_t>* o, const std::string& version);
bool pb_parse(const uint8_t* in, size_t n, std::vector<PbBlock>* blocks, std::string* version,
              bool* has_metadata = nullptr);
// Recoded.Metadata.version only (empty without Metadata); false for bytes that are not a Recoded
// message at the top level.  No block list is built.
bool pb_read_version(const uint8_t* in, size_t n, std::string* version);

// Recoded.Metadata.version of the parallel model's containers (the reference model writes none, as
// the reference does): its decisions through the reference's arithmetic_code<uint64_t, uint8_t>, or
// through the optional 32-bit P32 coder
extern const char* const kParallelModelTag;     // "avrecode-amd:P64"
extern const char* const kParallel32ModelTag;   // "avrecode-amd:P32"
extern const char* const kChainedModelTag;      // "avrecode-amd:R16"
// The model a container's Metadata.version names: 0 reference (no tag, or any foreign one), 1
// parallel / u64 coder, 2 parallel / P32 coder (AVR_MODEL_*); -1 another avrecode-amd format (the
// round-2 "avrecode-amd:P", ...), which must be refused rather than read as a reference container.
int model_of_version(const std::string& version);
const char* version_of_model(int model);   // nullptr for the reference model
constexpr int kSurrogateMarkerBytes = 8;      // recode.cpp:27
void surrogate_marker(uint64_t seq, uint8_t out[8]);

}  // namespace avr
