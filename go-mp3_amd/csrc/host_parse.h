// host_parse.h -- product host-side bitstream parse of an MP3 byte stream into
// the granule boundary input of the GPU path.
//
// This is the part of go-mp3's per-frame pipeline that stays on the CPU:
// source/tag handling (source.go:42-122), frame header + sync search
// (frameheader.go:279-328), side info (sideinfo.go:33-156), bit reservoir
// (maindata.go:290-323), scale factors (maindata.go:119-288) and Huffman
// decoding (maindata/huffman.go:27-138, huffman/huffman.go:348-419).  The
// semantics (including the reference's quirks: reservoir underflow, zero
// reads past the end of the main data, count1 back-off) are the reference's;
// the implementation is table driven: Huffman codewords are decoded with
// two-level lookup tables built from ISO 11172-3 Table B.7 instead of a
// bit-serial tree walk, and the output is written straight into
// mp3g_granule descriptors + int16 coefficients.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/mp3g.h"

namespace mp3g {
namespace host {

// Error classes the reference's decode.go distinguishes.  kRead: the
// caller's io.Reader failed (decode.go:48-63 passes its error through).
enum class St { kOk = 0, kEof = 1, kErr = 2, kPanic = 3, kRead = 4 };

// source.go (source.go:22-122) over one of two byte sources:
//  * in memory (data, len): a bytes.Reader; seekable = implements io.Seeker;
//  * reader mode (rd != nullptr): the caller's io.Reader / io.Seeker as
//    callbacks (mp3g_reader).  Bytes are pulled into a window of the stream,
//    [base, base + win.size()); rpos is the absolute stream position of the
//    next byte.  A read past the window calls rd->read (io.Reader.Read: any
//    count >= 1, 0 = io.EOF, < 0 = error) unless may_fetch is off, in which
//    case the read stops short and sets `starved` -- the decoder's read-ahead
//    uses that to scan only bytes that have already arrived (a live stream's
//    Read may block).  Seeks inside the window move rpos; others go to
//    rd->seek and empty the window.
struct Source {
  const uint8_t* data = nullptr;
  int64_t len = 0;
  int64_t rpos = 0;  // reader position
  bool seekable = true;
  uint8_t unread[16];
  int n_unread = 0;
  int64_t pos = 0;  // source.pos

  // ---- reader mode ----
  const mp3g_reader* rd = nullptr;
  std::vector<uint8_t> win;
  int64_t base = 0;
  int64_t keep_from = 0;   // a fetch may drop window bytes before min(keep_from, rpos)
  bool may_fetch = true;   // reads past the window may call rd->read
  bool starved = false;    // a read stopped short because may_fetch was off
  bool read_failed = false;  // rd->read returned an error (cleared by the caller)
  size_t fetch_bytes = 64 << 10;  // bytes asked of one rd->read

  int64_t read_full(uint8_t* buf, int64_t n, bool* short_read);
  void unread_bytes(const uint8_t* b, int n);
  bool seek(int64_t off, int whence, int64_t* res);
  St skip_tags();

  // Position state for a rollback (reader mode: the window keeps the bytes
  // from keep_from on, so a restore never needs the reader again).
  struct Mark {
    int64_t rpos, pos;
    int n_unread;
    uint8_t unread[16];
  };
  Mark mark() const;
  void restore(const Mark& m);

 private:
  bool fill(int64_t end);  // reader mode: grow the window towards `end`
};

// One parsed frame: its header, start offset and the boundary input of its
// granules (2 for MPEG-1, 1 for MPEG-2 LSF).
struct ParsedFrame {
  uint32_t header = 0;
  int64_t start = 0;
  int n_granules = 0;
  mp3g_granule gran[2];
  int16_t coef[2][MP3G_COEF_PER_GRANULE];
};

// Carries the bit reservoir between frames (frame.Read's `prev`).
class FrameParser {
 public:
  // Parses the next frame at the source's position (frame.go:67-115).
  // prev_frame = false reproduces frame.Read(source, pos, nil) -- after a
  // seek the reservoir is empty.
  St next(Source& src, ParsedFrame* out);
  void reset() { have_prev_ = false; prev_md_.clear(); }

 private:
  bool have_prev_ = false;
  std::vector<uint8_t> prev_md_;  // previous frame's main-data bytes
  std::vector<uint8_t> md_;       // scratch
};

// frame.Read split at the bit reservoir: everything
// but the scale factors and Huffman codes, which the device decodes
// (huffman_dev.hip) from one job per (granule, channel).
struct ScannedFrame {
  uint32_t header = 0;
  int64_t start = 0;
  int n_granules = 0;
  mp3g_granule gran[2];  // side-info fields; scale factors and count1 zero
  mp3g_hjob job[2][2];   // [gr][ch]; bit positions in the scanner's main-data buffer
};

// A main-data sink over caller memory: bytes [0, n) are in use, appends may
// grow n up to cap (mp3g_scan_streams writes every stream's main data
// straight into its place in the concatenation).  `overflow` records an
// append that did not fit.
struct RawMd {
  uint8_t* base = nullptr;
  size_t n = 0, cap = 0;
  bool overflow = false;
  size_t size() const { return n; }
  uint8_t* data() const { return base; }
};

class FrameScanner {
 public:
  // Parses the next frame's header and side info and appends its main-data
  // bytes to *md; the same statuses, at the same source positions, as
  // FrameParser::next on the same input.  (RawMd: a frame that does not fit
  // ends the scan with kErr and sets md->overflow.)
  St next(Source& src, ScannedFrame* out, std::vector<uint8_t>* md);
  St next(Source& src, ScannedFrame* out, RawMd* md);
  void reset() { have_prev_ = false; }  // frame.Read(source, pos, nil)
  // First byte of *md the next frame's bit buffer can reach back to.
  int64_t live_start(const std::vector<uint8_t>& md) const { return have_prev_ ? prev_start_ : (int64_t)md.size(); }
  // Rebases after the caller dropped the first n bytes of *md.
  void drop(int64_t n) { prev_start_ -= n; }

 private:
  bool have_prev_ = false;
  int64_t prev_start_ = 0;  // byte offset in *md of the previous frame's bit buffer
  template <class Md>
  St next_impl(Source& src, ScannedFrame* out, Md* md);
};

// One read-ahead step of the decoder (decode.go:45-67 repeated): up to
// max_frames frames from the source's position, each handed to `emit` with
// the source position after it.  Returns the status that ended the scan
// (kOk: max_frames reached, or -- reader mode -- the next frame is not fully
// buffered and may not be fetched).  Fetch rule: an in-memory or seekable
// source always reads; a non-seekable reader is read only while `must` is set
// and no frame has been scanned in this call, i.e. only when the decoder holds
// no complete frame it has not decoded -- where the reference's Decoder.Read
// would block too.  A frame cut short by that rule is rolled back: the
// scanner state, *md and the source position are as before it.
St scan_some(Source& src, FrameScanner& sc, std::vector<uint8_t>* md, size_t max_frames, bool must,
             void (*emit)(void* ctx, const ScannedFrame& f, int64_t src_pos), void* ctx);
St parse_some(Source& src, FrameParser& fp, size_t max_frames, bool must,
              void (*emit)(void* ctx, const ParsedFrame& f, int64_t src_pos), void* ctx);

// frameheader.Read: sync search from the source position.
St read_header(Source& s, int64_t* pos_io, uint32_t* out);

// Header-only walk of a whole stream (tags, sync search, sizes): the granules
// and main-data bytes of the frames FrameScanner would accept if no frame's
// side info ended the stream early (an upper bound; equal for every stream
// that scans to EOF).
void prescan(const uint8_t* data, size_t len, uint64_t* n_granules, uint64_t* md_bytes);

// frameheader accessors used by the decoder
int header_bytes_per_frame(uint32_t h);
int header_frame_size(uint32_t h);
int header_sample_rate(uint32_t h);
int header_granules(uint32_t h);

}  // namespace host
}  // namespace mp3g
