// reader_driver.cpp -- the decoder's streaming input (mp3g_reader, reader mode
// of host::Source, host::scan_some) against the in-memory source, on the CPU.
//
// Built by tests/test_reader_cpu.py with g++ from go-mp3_amd/csrc/host_parse.cpp
// (no GPU code).  For one input file and seed it scans every frame
//   (a) in memory (the bytes.Reader the other decoder entry wraps),
//   (b) through a read callback that hands out 1..4096-byte pieces, with and
//       without a seek callback, in the decoder's pattern: read-ahead scans of
//       random length that may only use arrived bytes (non-seekable), and a
//       "must" scan whenever the previous one produced nothing,
//   (c) through a reader that delivers the bytes of the first N frames and
//       then blocks (here: records that it was asked and reports EOF) --
//       every one of those N frames must have been delivered before the
//       reader is asked for more (the reference's Decoder.Read blocks only
//       for the frame it is about to decode, decode.go:70-80),
// and checks that (b) and (c) produce the same frames (descriptors, Huffman
// jobs, main-data bytes, end status) as (a), plus a seek into the middle
// through the seek callback.  Exit 0 and "ok ..." when every check holds.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../go-mp3_amd/csrc/host_parse.h"

using namespace mp3g::host;

struct Rec {
  uint32_t header;
  int64_t start, src_pos;
  int n_granules;
  mp3g_granule gran[2];
  mp3g_hjob job[2][2];
};

static bool same(const Rec& a, const Rec& b) {
  return a.header == b.header && a.start == b.start && a.src_pos == b.src_pos && a.n_granules == b.n_granules &&
         std::memcmp(a.gran, b.gran, sizeof a.gran) == 0 && std::memcmp(a.job, b.job, sizeof a.job) == 0;
}

struct Run {
  std::vector<Rec> frames;
  std::vector<uint8_t> md;
  St end = St::kOk;
};

static void emit(void* ctx, const ScannedFrame& f, int64_t sp) {
  Rec r;
  std::memset(&r, 0, sizeof r);
  r.header = f.header;
  r.start = f.start;
  r.src_pos = sp;
  r.n_granules = f.n_granules;
  std::memcpy(r.gran, f.gran, sizeof r.gran);
  std::memcpy(r.job, f.job, sizeof r.job);
  static_cast<Run*>(ctx)->frames.push_back(r);
}

struct Feed {  // the caller's io.Reader (+ io.Seeker)
  const std::vector<uint8_t>* data;
  size_t off = 0;
  uint64_t rng;
  size_t block_at = (size_t)-1;  // (c): bytes delivered before the reader "blocks"
  size_t fail_at = (size_t)-1;   // (d): bytes delivered before the reader fails
  bool blocked = false;
  size_t frames_when_blocked = 0;
  const Run* run = nullptr;
  long calls = 0;
  uint32_t next() {
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(rng >> 33);
  }
};

static int64_t feed_read(void* user, uint8_t* buf, size_t cap) {
  Feed& f = *static_cast<Feed*>(user);
  f.calls++;
  if (f.off >= f.fail_at) return -1;
  const size_t lim = std::min({f.data->size(), f.block_at, f.fail_at});
  if (f.off >= lim) {
    if (f.off < f.data->size() && !f.blocked) {  // a live stream would block here
      f.blocked = true;
      f.frames_when_blocked = f.run->frames.size();
    }
    return 0;
  }
  size_t k = 1 + f.next() % 4096;
  k = std::min({k, cap, lim - f.off});
  std::memcpy(buf, f.data->data() + f.off, k);
  f.off += k;
  return (int64_t)k;
}

static int64_t feed_seek(void* user, int64_t off, int whence) {
  Feed& f = *static_cast<Feed*>(user);
  const int64_t a = whence == 0 ? off : whence == 1 ? (int64_t)f.off + off : (int64_t)f.data->size() + off;
  if (a < 0) return -1;
  f.off = (size_t)a;
  return a;
}

// The decoder's pattern of scans (host_decoder.cpp refill / scan_batch).
static Run scan_all(Source& src, Feed* feed) {
  Run r;
  FrameScanner sc;
  St st = src.skip_tags();
  if (st != St::kOk) {
    r.end = st;
    return r;
  }
  bool must = true;
  for (int guard = 0; guard < 10000000; guard++) {
    const size_t before = r.frames.size();
    const size_t max_frames = feed ? 1 + feed->next() % 40 : 1000000;
    st = scan_some(src, sc, &r.md, max_frames, must, emit, &r);
    if (st != St::kOk) break;
    must = r.frames.size() == before;
  }
  r.end = st;
  return r;
}

static int fail(const char* what, size_t i) {
  std::printf("FAIL %s at %zu\n", what, i);
  return 1;
}

static int compare(const Run& a, const Run& b, const char* what) {
  if (a.frames.size() != b.frames.size()) {
    std::printf("FAIL %s: %zu frames vs %zu\n", what, b.frames.size(), a.frames.size());
    return 1;
  }
  for (size_t i = 0; i < a.frames.size(); i++)
    if (!same(a.frames[i], b.frames[i])) return fail(what, i);
  if (a.md != b.md) return fail(what, (size_t)-1);
  if (a.end != b.end) {
    std::printf("FAIL %s: end %d vs %d\n", what, (int)b.end, (int)a.end);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  std::vector<uint8_t> d;
  {
    FILE* fp = std::fopen(argv[1], "rb");
    if (!fp) return 2;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) d.insert(d.end(), buf, buf + n);
    std::fclose(fp);
  }
  const uint64_t seed = std::strtoull(argv[2], nullptr, 10);
  // (a) in memory
  Source mem;
  mem.data = d.data();
  mem.len = (int64_t)d.size();
  const Run ref = scan_all(mem, nullptr);
  long calls = 0;
  // (b) pieces, seekable and not
  for (int seekable = 0; seekable < 2; seekable++) {
    Feed f;
    f.data = &d;
    f.rng = seed * 2 + seekable + 1;
    Run* live = nullptr;
    mp3g_reader rd{feed_read, seekable ? feed_seek : nullptr, &f};
    Source src;
    src.rd = &rd;
    src.seekable = seekable != 0;
    Run r = scan_all(src, &f);
    (void)live;
    calls += f.calls;
    if (compare(ref, r, seekable ? "pieces+seek" : "pieces")) return 1;
    if (seekable && ref.frames.size() > 4) {
      // seek to the middle frame through the callback, rescan a few frames
      const size_t k = ref.frames.size() / 2;
      const int64_t at = ref.frames[k].start;
      Source m2 = mem;
      m2.n_unread = 0;
      FrameScanner s1, s2;
      Run a, b;
      if (!m2.seek(at, 0, nullptr) || !src.seek(at, 0, nullptr)) return fail("seek", k);
      const St e1 = scan_some(m2, s1, &a.md, 6, true, emit, &a);
      const St e2 = scan_some(src, s2, &b.md, 6, true, emit, &b);
      a.end = e1;
      b.end = e2;
      if (compare(a, b, "after seek")) return 1;
    }
  }
  // (c) a live stream that stops after the first N frames' bytes (non-seekable)
  size_t checked = 0;
  for (size_t n : {(size_t)1, (size_t)2, ref.frames.size() / 3, ref.frames.size() - 1}) {
    if (ref.frames.size() < 2 || n == 0 || n >= ref.frames.size()) continue;
    Feed f;
    f.data = &d;
    f.rng = seed * 7 + n;
    // frames 0..n-1 have fully arrived.  (source.pos, hence a frame's start,
    // runs 3 bytes behind the reader after skipTags: its Unread lowers pos and
    // ReadFull counts only the reader's bytes, source.go:94-97, :99-122.)
    f.block_at = (size_t)ref.frames[n].start + 3;
    Run r;
    f.run = &r;
    mp3g_reader rd{feed_read, nullptr, &f};
    Source src;
    src.rd = &rd;
    src.seekable = false;
    FrameScanner sc;
    St st = src.skip_tags();
    bool must = true;
    while (st == St::kOk) {
      const size_t before = r.frames.size();
      st = scan_some(src, sc, &r.md, 1 + f.next() % 40, must, emit, &r);
      must = r.frames.size() == before;
    }
    if (!f.blocked) return fail("live: the reader was never asked past the arrived frames", n);
    if (f.frames_when_blocked != n) {
      std::printf("FAIL live: %zu of %zu arrived frames delivered before the reader was asked for more\n",
                  f.frames_when_blocked, n);
      return 1;
    }
    for (size_t i = 0; i < n; i++)
      if (!same(ref.frames[i], r.frames[i])) return fail("live frame", i);
    checked++;
  }
  // (d) a reader that fails part-way: every frame that arrived before the
  // failure is delivered, then the scan ends with the reader's error (kRead)
  for (size_t n : {(size_t)1, ref.frames.size() / 2}) {
    if (ref.frames.size() < 2 || n == 0 || n >= ref.frames.size()) continue;
    for (int seekable = 0; seekable < 2; seekable++) {
      Feed f;
      f.data = &d;
      f.rng = seed * 11 + n + seekable;
      f.fail_at = (size_t)ref.frames[n].start + 3;
      mp3g_reader rd{feed_read, seekable ? feed_seek : nullptr, &f};
      Source src;
      src.rd = &rd;
      src.seekable = seekable != 0;
      Run r = scan_all(src, &f);
      if (r.end != St::kRead) {
        std::printf("FAIL reader error: end %d\n", (int)r.end);
        return 1;
      }
      if (r.frames.size() != n) return fail("reader error: frames before it", r.frames.size());
      for (size_t i = 0; i < n; i++)
        if (!same(ref.frames[i], r.frames[i])) return fail("reader error frame", i);
    }
  }
  std::printf("ok frames=%zu end=%d reader_calls=%ld live_cases=%zu\n", ref.frames.size(), (int)ref.end, calls,
              checked);
  return 0;
}
