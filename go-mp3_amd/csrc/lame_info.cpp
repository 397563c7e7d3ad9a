// lame_info.cpp -- Xing/Info/LAME tag of the first frame (SURVEY.md 8f row
// f4): the reference's lameinfo package (lameinfo/lameinfo.go), which the
// decoder itself never calls (decode.go decodes the tag frame as audio).  Host
// code: one frame of bytes, no device work.
#include <cstring>

#include "../../include/mp3g.h"
#include "abi_util.h"

namespace {

uint32_t be32(const uint8_t* p) {  // binary.BigEndian.Uint32
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// isLAMEVersion (lameinfo.go:273-281): the first 4 of the 9 version bytes
bool is_lame_version(const uint8_t* s) {
  return !std::memcmp(s, "LAME", 4) || !std::memcmp(s, "L3.9", 4) || !std::memcmp(s, "Gogo", 4) ||
         !std::memcmp(s, "GOGO", 4);
}

// calculateFrameSize (lameinfo.go:364-384) with its tables (:331-362);
// version / layer are the raw header fields (version 1 = reserved, layer 3 = I)
int frame_size(uint32_t version, uint32_t layer, uint32_t br_index, uint32_t sr_index, uint32_t padding) {
  static const int kBr[2][16] = {
      {0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160, 0},        // MPEG 2 / 2.5, layer II/III
      {0, 32, 48, 56, 64, 80, 96, 112, 128, 144, 160, 176, 192, 224, 256, 0}};  // MPEG 2 / 2.5, layer I
  static const int kBr1[3][16] = {
      {0, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 0},    // MPEG 1 layer III
      {0, 32, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384, 0},   // MPEG 1 layer II
      {0, 32, 64, 96, 128, 160, 192, 224, 256, 288, 320, 352, 384, 416, 448, 0}};  // MPEG 1 layer I
  static const int kSr[4][4] = {{11025, 12000, 8000, 0}, {0, 0, 0, 0}, {22050, 24000, 16000, 0}, {44100, 48000, 32000, 0}};
  if (version == 1 || layer == 0) return 0;  // the reference's empty table rows
  int kbps;
  if (version == 3) kbps = kBr1[layer - 1][br_index];
  else kbps = layer == 3 ? kBr[1][br_index] : kBr[0][br_index];
  const int bitrate = kbps * 1000, rate = kSr[version][sr_index];
  if (bitrate == 0 || rate == 0) return 0;
  if (layer == 3) return (12 * bitrate / rate + (int)padding) * 4;  // layer I
  return (version == 3 ? 144 : 72) * bitrate / rate + (int)padding;
}

}  // namespace

extern "C" {

// Parse (lameinfo.go:139-270)
int mp3g_lame_parse(const uint8_t* frame, size_t len, mp3g_lame_info* out) {
  if (!out || (len && !frame)) return mp3g::abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  std::memset(out, 0, sizeof *out);
  const int kNo = MP3G_ERR_NO_XING_HEADER;
  if (len < 4) return kNo;
  const uint32_t h = be32(frame);
  if ((h & 0xFFE00000u) != 0xFFE00000u) return kNo;  // sync
  const uint32_t version = (h >> 19) & 3u;
  if (version == 1) return kNo;  // reserved
  const bool mono = ((h >> 6) & 3u) == 3u;
  // sideInfoSize (lameinfo.go:118-130)
  const size_t side = version == 3 ? (mono ? 17 : 32) : (mono ? 9 : 17);
  const size_t offset = 4 + side;
  if (len < offset + 4) return kNo;
  const bool xing = !std::memcmp(frame + offset, "Xing", 4);
  if (!xing && std::memcmp(frame + offset, "Info", 4)) return kNo;
  mp3g_lame_info info;
  std::memset(&info, 0, sizeof info);
  info.is_xing = xing;
  size_t pos = offset + 4;
  if (len < pos + 4) return kNo;
  info.flags = be32(frame + pos);
  pos += 4;
  if (info.flags & MP3G_XING_FRAME_COUNT) {
    if (len < pos + 4) return kNo;
    info.frame_count = be32(frame + pos);
    pos += 4;
  }
  if (info.flags & MP3G_XING_BYTE_COUNT) {
    if (len < pos + 4) return kNo;
    info.byte_count = be32(frame + pos);
    pos += 4;
  }
  if (info.flags & MP3G_XING_TOC) {
    if (len < pos + 100) return kNo;
    std::memcpy(info.toc, frame + pos, 100);
    pos += 100;
  }
  if (info.flags & MP3G_XING_VBR_SCALE) {
    if (len < pos + 4) return kNo;
    info.vbr_scale = be32(frame + pos);
    pos += 4;
  }
  // LAME extension: 9-byte version, 12 bytes of fields, then the 3 bytes of
  // 12-bit delay + 12-bit padding (lameinfo.go:238-267)
  if (len >= pos + 9 && is_lame_version(frame + pos)) {
    info.has_lame = 1;
    std::memcpy(info.lame_version, frame + pos, 9);
    pos += 9;
    const size_t d = pos + 12;
    if (len >= d + 3) {
      info.encoder_delay = (uint16_t)((uint16_t)frame[d] << 4 | frame[d + 1] >> 4);
      info.encoder_padding = (uint16_t)((uint16_t)(frame[d + 1] & 0x0F) << 8 | frame[d + 2]);
    }
  }
  *out = info;
  return MP3G_OK;
}

// ParseFromReader (lameinfo.go:288-328) over a byte buffer (a bytes.Reader):
// io.ReadFull's io.EOF / io.ErrUnexpectedEOF become MP3G_EOF /
// MP3G_ERR_UNEXPECTED_EOF.  *consumed = the bytes the reader took.
int mp3g_lame_parse_reader(const uint8_t* data, size_t len, mp3g_lame_info* out, size_t* consumed) {
  if (!out || (len && !data)) return mp3g::abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  std::memset(out, 0, sizeof *out);
  size_t used = 0;
  auto done = [&](int st) {
    if (consumed) *consumed = used;
    return st;
  };
  if (len < 4) {  // io.ReadFull(r, header)
    used = len;
    return done(len == 0 ? MP3G_EOF : MP3G_ERR_UNEXPECTED_EOF);
  }
  used = 4;
  const uint32_t h = be32(data);
  if ((h & 0xFFE00000u) != 0xFFE00000u) return done(MP3G_ERR_NO_XING_HEADER);
  const uint32_t version = (h >> 19) & 3u, layer = (h >> 17) & 3u, br = (h >> 12) & 15u, sr = (h >> 10) & 3u,
                 padding = (h >> 9) & 1u;
  if (version == 1 || layer == 0 || br == 0 || br == 15 || sr == 3) return done(MP3G_ERR_NO_XING_HEADER);
  const int fsize = frame_size(version, layer, br, sr, padding);
  if (fsize < 4) return done(MP3G_ERR_NO_XING_HEADER);
  const size_t need = (size_t)fsize - 4;  // io.ReadFull(r, frame[4:])
  if (len - 4 < need) {
    used = len;
    return done(len == 4 ? MP3G_EOF : MP3G_ERR_UNEXPECTED_EOF);
  }
  used = (size_t)fsize;
  return done(mp3g_lame_parse(data, (size_t)fsize, out));
}

// Info.TotalDelay / TotalPadding (lameinfo.go:92-111), DecoderDelay = 529
int mp3g_lame_total_delay(const mp3g_lame_info* info) {
  if (!info || !info->has_lame) return MP3G_LAME_DECODER_DELAY;
  return (int)info->encoder_delay + MP3G_LAME_DECODER_DELAY;
}

int mp3g_lame_total_padding(const mp3g_lame_info* info) {
  if (!info || !info->has_lame) return 0;
  const int p = (int)info->encoder_padding - MP3G_LAME_DECODER_DELAY;
  return p < 0 ? 0 : p;
}

// Gapless trim of a decoded stream (the use the reference documents for the
// two totals, lameinfo.go:86-111; it never applies them itself): go-mp3
// decodes the tag frame as silence (decode.go), so the caller passes the
// samples that frame produced (1152 MPEG-1, 576 MPEG-2) and gets the range of
// the n_samples to keep.
int mp3g_lame_trim(const mp3g_lame_info* info, uint64_t n_samples, uint32_t tag_frame_samples, uint64_t* first,
                   uint64_t* count) {
  if (!info || !first || !count) return mp3g::abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  const uint64_t skip = (uint64_t)tag_frame_samples + (uint64_t)mp3g_lame_total_delay(info);
  const uint64_t drop = (uint64_t)mp3g_lame_total_padding(info);
  *first = skip < n_samples ? skip : n_samples;
  *count = n_samples > skip + drop ? n_samples - skip - drop : 0;
  return MP3G_OK;
}

// Xing TOC seek: the byte offset of `percent` (0..100) of the playback time,
// TOC[i] / 256 of the byte count, interpolated between entries (the table
// Info.TOC holds, lameinfo.go:33-35).  The byte count is the tag's own
// (flag 0x2) or, when the tag has none, `stream_bytes` from the caller; without
// a TOC the offset is linear in that count.  *offset = 0 and
// MP3G_ERR_INVALID_ARGUMENT when neither count is known (stream_bytes = 0).
int mp3g_lame_toc_offset(const mp3g_lame_info* info, double percent, uint64_t stream_bytes, uint64_t* offset) {
  if (!info || !offset) return mp3g::abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *offset = 0;
  const bool own = info->flags & MP3G_XING_BYTE_COUNT;
  if (!own && stream_bytes == 0) return mp3g::abi_fail(MP3G_ERR_INVALID_ARGUMENT, "no byte count in the tag or from the caller");
  const double p = percent < 0.0 ? 0.0 : percent > 100.0 ? 100.0 : percent;
  const double bytes = own ? (double)info->byte_count : (double)stream_bytes;
  if (!(info->flags & MP3G_XING_TOC)) {
    *offset = (uint64_t)(p / 100.0 * bytes);
    return MP3G_OK;
  }
  int i = (int)p;
  if (i > 99) i = 99;
  const double a = info->toc[i], b = i < 99 ? info->toc[i + 1] : 256.0;
  *offset = (uint64_t)((a + (b - a) * (p - i)) / 256.0 * bytes);
  return MP3G_OK;
}

}  // extern "C"
