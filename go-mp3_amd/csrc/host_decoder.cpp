// host_decoder.cpp -- mp3.Decoder semantics on top of the GPU granule path
// (SURVEY.md 8f rows f2/f3): NewDecoder / Read / Seek / Length / time API of
// reference decode.go:27-388, with read-ahead: frames are parsed on the host
// in batches and each batch is decoded by one plan launch on the device,
// carrying Frame.store / Frame.vVec across batches through the plan's state
// buffers.  Error classes and their timing follow the reference: PCM of the
// frames before a failing frame is delivered first, the error is returned
// once the buffer is empty, and the next Read resumes parsing where the
// failed frame left the source, with no reservoir and zero DSP state
// (d.frame = nil, decode.go:45-67).
//
// Also the host-only batch parse entry points (mp3g_parse_*), which need no
// GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../../include/mp3g.h"
#include "abi_util.h"
#include "host_parse.h"

using namespace mp3g;
using host::St;

namespace {

int to_status(St s) {
  switch (s) {
    case St::kOk: return MP3G_OK;
    case St::kEof: return MP3G_EOF;
    case St::kErr: return MP3G_ERR_PARSE;
    case St::kPanic: return MP3G_ERR_UNSUPPORTED;
  }
  return MP3G_ERR_PARSE;
}

// Parses a whole stream (NewDecoder + reading to the end): tags skipped,
// reservoir carried, stops at EOF or at the first failing frame.
St parse_all(const uint8_t* data, size_t len, std::vector<mp3g_granule>* g, std::vector<int16_t>* c) {
  host::Source src;
  src.data = data;
  src.len = (int64_t)len;
  St st = src.skip_tags();
  if (st != St::kOk) return st;
  host::FrameParser parser;
  host::ParsedFrame f;
  for (;;) {
    st = parser.next(src, &f);
    if (st != St::kOk) return st;
    for (int gr = 0; gr < f.n_granules; gr++) {
      g->push_back(f.gran[gr]);
      c->insert(c->end(), f.coef[gr], f.coef[gr] + MP3G_COEF_PER_GRANULE);
    }
  }
}

}  // namespace

// PCM read-ahead bytes in page-locked memory: the batch's PCM is copied from
// the device straight into it (no pageable bounce, no second host copy).
struct PinnedBytes {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  bool pinned = false;
  PinnedBytes() = default;
  PinnedBytes(const PinnedBytes&) = delete;
  PinnedBytes& operator=(const PinnedBytes&) = delete;
  ~PinnedBytes() { release(); }
  void release() {
    if (p) {
      if (pinned) (void)hipHostFree(p);
      else std::free(p);
    }
    p = nullptr;
    n = cap = 0;
  }
  size_t size() const { return n; }
  const uint8_t* data() const { return p; }
  void clear() { n = 0; }
  // room for `more` bytes past n (contents kept)
  bool reserve_more(size_t more) {
    if (n + more <= cap) return true;
    const size_t c = std::max(n + more, 2 * cap);
    void* q = nullptr;
    bool pin = hipHostMalloc(&q, c, hipHostMallocDefault) == hipSuccess;
    if (!pin) q = std::malloc(c);
    if (!q) return false;
    if (n) std::memcpy(q, p, n);
    const size_t keep = n;
    release();
    p = static_cast<uint8_t*>(q);
    n = keep;
    cap = c;
    pinned = pin;
    return true;
  }
};

// Read-ahead batches start at 16 frames and double up to this.  A small
// batch is latency-bound on the device (the main-data kernel's lanes each walk
// one granule-channel's Huffman codes: ~0.2 ms for any batch that fits one
// round of waves), so the cap is set by that, not by the host scan (~0.2 us
// per frame): 8,192 frames = 32,768 jobs is still one round.
constexpr size_t kMaxBatchFrames = 8192;

// One read-ahead batch of frames as the host scan (or full parse) left it:
// everything its device leg needs, so that the next batch can be scanned
// while this one is on the device.
struct Batch {
  std::vector<mp3g_granule> gran;
  std::vector<int16_t> coef;   // MP3G_FLAG_HOST_HUFFMAN
  std::vector<mp3g_hjob> jobs;  // default: jobs into `md`
  std::vector<uint8_t> md;      // the main data the jobs address (a snapshot)
  std::vector<uint32_t> frame_pcm_bytes;  // PCM bytes of each frame
  std::vector<int64_t> frame_src;         // source position after each frame
  int err = MP3G_OK;  // status that ended the batch (EOF / parse error), after its frames
  bool fresh = true;  // starts from zero DSP state (frame = nil)
  size_t n() const { return gran.size(); }
  void clear() {
    gran.clear();
    coef.clear();
    jobs.clear();
    md.clear();
    frame_pcm_bytes.clear();
    frame_src.clear();
    err = MP3G_OK;
  }
};

// ---------------------------------------------------------------------------
struct mp3g_decoder {
  std::vector<uint8_t> data;  // own copy: no caller pointer is retained
  host::Source src;
  host::FrameParser parser;    // MP3G_FLAG_HOST_HUFFMAN: full host parse
  host::FrameScanner scanner;  // default: host scan + GPU main-data kernel
  std::vector<uint8_t> md;     // main-data concatenation the scanner's jobs address
  int device = 0;
  uint32_t mode = 0;
  int sample_rate = 0;
  int64_t length = -1;  // invalidLength
  int64_t bytes_per_frame = 0;
  std::vector<int64_t> frame_starts;
  int64_t pos = 0;
  // PCM being served (one batch) and the PCM of the batch on the device
  PinnedBytes buf, ahead;
  size_t buf_off = 0;
  int pending = MP3G_OK;  // parse error to report once buf runs dry
  bool scan_fresh = true;  // the next scanned batch starts from zero DSP state
  size_t batch_frames = 16;
  // Read-ahead pipeline: bat[fl] is on the device (its PCM lands in `ahead`),
  // bat[sc] is scanned and waits for the device; one slot each.
  Batch bat[2];
  bool inflight = false, scanned = false;
  int fl = 0, sc = 1;
  uint32_t first_header = 0;  // header of the first granule served (SampleRate)
  // device resources (grown on demand)
  hipStream_t stream = nullptr;
  mp3g_granule* d_gran = nullptr;
  int16_t* d_coef = nullptr;
  int16_t* d_pcm = nullptr;
  mp3g_state* d_state = nullptr;  // [0] = carried in, [1] = out
  mp3g_hjob* d_jobs = nullptr;
  uint8_t* d_md = nullptr;
  size_t cap_granules = 0, cap_md = 0;
  // the last plan (batches of the same length and state flags reuse it)
  mp3g_plan* plan = nullptr;
  uint64_t plan_n = 0;
  uint32_t plan_flags = 0;
  std::vector<size_t> frame_ends;         // end offset in buf of each buffered frame
  std::vector<int64_t> frame_src_ends;    // source position after each buffered frame
  // index into frame_ends of the frame the reference read last: Decoder.Read
  // reads one frame once its d.buf is empty (decode.go:70-80), so this is the
  // frame being served, advanced lazily at the next Read like the reference
  size_t next_end = 0;

  ~mp3g_decoder() {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (plan) mp3g_plan_destroy(plan);
    buf.release();
    ahead.release();
    for (void* p : {(void*)d_gran, (void*)d_coef, (void*)d_pcm, (void*)d_state, (void*)d_jobs, (void*)d_md})
      if (p) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
    if (prev >= 0) (void)hipSetDevice(prev);
  }

  int ensure_capacity(size_t n) {
    if (n <= cap_granules) return MP3G_OK;
    size_t cap = std::max<size_t>(n, cap_granules * 2);
    for (void** p : {(void**)&d_gran, (void**)&d_coef, (void**)&d_pcm, (void**)&d_jobs})
      if (*p) { (void)hipFree(*p); *p = nullptr; }
    if (hipMalloc(&d_gran, cap * sizeof(mp3g_granule)) != hipSuccess ||
        hipMalloc(&d_coef, cap * MP3G_COEF_PER_GRANULE * sizeof(int16_t)) != hipSuccess ||
        hipMalloc(&d_pcm, cap * MP3G_PCM_BYTES_PER_GRANULE) != hipSuccess ||
        hipMalloc(&d_jobs, 2 * cap * sizeof(mp3g_hjob)) != hipSuccess) {
      cap_granules = 0;
      return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder device buffers");
    }
    cap_granules = cap;
    return MP3G_OK;
  }

  bool gpu_huffman() const { return (mode & MP3G_FLAG_HOST_HUFFMAN) == 0; }

  // Scans (or parses) up to `max_frames` frames into b.  A failing frame ends
  // the batch: b.err, the reservoir is dropped and the next batch starts from
  // zero DSP state (d.frame = nil after a failed frame.Read).
  void scan_batch(Batch& b, size_t max_frames) {
    b.clear();
    b.fresh = scan_fresh;
    St st = St::kOk;
    if (gpu_huffman()) {
      // drop main data no later frame can reach (the reservoir is < 2 KB)
      const int64_t dead = scanner.live_start(md);
      if (dead > 0) {
        md.erase(md.begin(), md.begin() + dead);
        scanner.drop(dead);
      }
      host::ScannedFrame f;
      for (size_t i = 0; i < max_frames; i++) {
        st = scanner.next(src, &f, &md);
        if (st != St::kOk) break;
        for (int gr = 0; gr < f.n_granules; gr++) {
          b.gran.push_back(f.gran[gr]);
          b.jobs.push_back(f.job[gr][0]);
          b.jobs.push_back(f.job[gr][1]);
        }
        b.frame_pcm_bytes.push_back((uint32_t)(f.n_granules * MP3G_PCM_BYTES_PER_GRANULE));
        b.frame_src.push_back(src.pos);
      }
      if (!b.gran.empty()) b.md.assign(md.begin(), md.end());  // the scanner keeps editing md
    } else {
      host::ParsedFrame f;
      for (size_t i = 0; i < max_frames; i++) {
        st = parser.next(src, &f);
        if (st != St::kOk) break;
        for (int gr = 0; gr < f.n_granules; gr++) {
          b.gran.push_back(f.gran[gr]);
          b.coef.insert(b.coef.end(), f.coef[gr], f.coef[gr] + MP3G_COEF_PER_GRANULE);
        }
        b.frame_pcm_bytes.push_back((uint32_t)(f.n_granules * MP3G_PCM_BYTES_PER_GRANULE));
        b.frame_src.push_back(src.pos);
      }
    }
    b.err = st == St::kOk ? MP3G_OK : to_status(st);
    if (b.err != MP3G_OK) reset_reservoir();
    scan_fresh = b.gran.empty() || b.err != MP3G_OK;
    batch_frames = std::min<size_t>(batch_frames * 2, kMaxBatchFrames);
  }

  void reset_reservoir() {
    parser.reset();
    scanner.reset();
  }

  // Enqueues batch b (n() > 0) on the decoder's stream: H2D, Huffman kernel,
  // DSP plan (state carried on the device), PCM D2H into `ahead`.
  int submit(const Batch& b) {
    const size_t n = b.n();
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return abi_fail(MP3G_ERR_NO_DEVICE, "hipSetDevice");
    struct Restore {
      int p;
      ~Restore() { if (p >= 0) (void)hipSetDevice(p); }
    } restore{prev};
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess)
      return abi_fail(MP3G_ERR_DEVICE, "hipStreamCreate");
    if (!d_state && hipMalloc(&d_state, 2 * sizeof(mp3g_state)) != hipSuccess)
      return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder state");
    int rc = ensure_capacity(n);
    if (rc) return rc;
    mp3g_stream s{0, (uint32_t)n, (b.fresh ? 0u : (uint32_t)MP3G_STREAM_STATE_IN) | MP3G_STREAM_STATE_OUT};
    if (!plan || plan_n != n || plan_flags != s.flags) {
      if (plan) mp3g_plan_destroy(plan);
      plan = nullptr;
      rc = mp3g_plan_create(device, &s, 1, 0, mode & ~(uint32_t)MP3G_FLAG_HOST_HUFFMAN, &plan);
      if (rc) return rc;
      plan_n = n;
      plan_flags = s.flags;
    }
    const size_t pcm_bytes = n * MP3G_PCM_BYTES_PER_GRANULE;
    ahead.clear();
    if (!ahead.reserve_more(pcm_bytes)) return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder PCM buffer");
    hipError_t e = hipMemcpyAsync(d_gran, b.gran.data(), n * sizeof(mp3g_granule), hipMemcpyHostToDevice, stream);
    if (gpu_huffman()) {
      // main data + jobs up, then scale factors / Huffman codes on the device
      const size_t mdb = b.md.size() + 16;  // + padding for the 32-bit window loads
      if (e == hipSuccess && mdb > cap_md) {
        if (d_md) (void)hipFree(d_md);
        d_md = nullptr;
        cap_md = std::max(mdb, 2 * cap_md);
        e = hipMalloc(&d_md, cap_md);
        if (e != hipSuccess) cap_md = 0;
      }
      if (e == hipSuccess && !b.md.empty())
        e = hipMemcpyAsync(d_md, b.md.data(), b.md.size(), hipMemcpyHostToDevice, stream);
      if (e == hipSuccess)
        e = hipMemcpyAsync(d_jobs, b.jobs.data(), b.jobs.size() * sizeof(mp3g_hjob), hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) {
        rc = mp3g_huffman_execute(device, d_jobs, n, d_md, d_gran, d_coef, stream);
        if (rc) return rc;
      }
    } else if (e == hipSuccess) {
      e = hipMemcpyAsync(d_coef, b.coef.data(), b.coef.size() * sizeof(int16_t), hipMemcpyHostToDevice, stream);
    }
    if (e != hipSuccess) return abi_fail(MP3G_ERR_DEVICE, "decoder H2D copy");
    rc = mp3g_plan_execute(plan, d_gran, d_coef, d_state, d_state + 1, d_pcm, stream);
    if (rc) return rc;
    e = hipMemcpyAsync(ahead.p, d_pcm, pcm_bytes, hipMemcpyDeviceToHost, stream);
    // carry: out -> in for the next batch
    if (e == hipSuccess) e = hipMemcpyAsync(d_state, d_state + 1, sizeof(mp3g_state), hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return abi_fail(MP3G_ERR_DEVICE, "decoder batch");
    ahead.n = pcm_bytes;
    return MP3G_OK;
  }

  // Waits for the batch on the device and makes it the served buffer.
  int complete(const Batch& b) {
    if (hipStreamSynchronize(stream) != hipSuccess) return abi_fail(MP3G_ERR_DEVICE, "decoder batch");
    std::swap(buf.p, ahead.p);
    std::swap(buf.n, ahead.n);
    std::swap(buf.cap, ahead.cap);
    std::swap(buf.pinned, ahead.pinned);
    size_t end = 0;
    for (uint32_t x : b.frame_pcm_bytes) frame_ends.push_back(end += x);
    frame_src_ends.insert(frame_src_ends.end(), b.frame_src.begin(), b.frame_src.end());
    if (!first_header) first_header = b.gran.front().header;
    return MP3G_OK;
  }

  // Drops the read-ahead (seek): waits for the device, forgets both slots.
  void cancel_read_ahead() {
    if (inflight && stream) (void)hipStreamSynchronize(stream);
    inflight = scanned = false;
  }

  void buf_reset() {
    buf.clear();
    buf_off = 0;
    frame_ends.clear();
    frame_src_ends.clear();
    next_end = 0;
  }

  // Where the reference's source stands: right after the last frame it read.
  // The read-ahead has parsed further; a seek that reads nothing (to or past
  // the end, decode.go:110-113) must leave the source there, so that the next
  // Read decodes the frame the reference decodes.
  void rewind_read_ahead() {
    if (next_end < frame_src_ends.size()) src.seek(frame_src_ends[next_end], 0, nullptr);
  }

  // readFrame for Read: serve the next batch (read-ahead grows to
  // kMaxBatchFrames).  Pipelined: the batch served now was put on the device by the
  // previous refill; the next scanned batch goes on the device and the one
  // after it is scanned on the host while the device works.  A batch that
  // ends in an error (or EOF) is the last one read ahead; its status is
  // returned once its PCM has been read, and the refill after that resumes
  // scanning where the failed frame left the source.
  int refill() {
    if (pending != MP3G_OK) {
      const int e = pending;
      pending = MP3G_OK;
      frame_src_ends.clear();  // the reference's source now stands after the failed frame
      return e;
    }
    buf_reset();
    int served;
    if (inflight) {
      served = fl;
      inflight = false;
    } else {
      served = scanned ? sc : fl;
      if (!scanned) scan_batch(bat[served], batch_frames);
      scanned = false;
      Batch& b = bat[served];
      if (b.n() == 0) return b.err == MP3G_OK ? MP3G_EOF : b.err;
      const int rc = submit(b);
      if (rc) return rc;
    }
    Batch& b = bat[served];
    int rc = complete(b);
    if (rc) return rc;
    if (b.err != MP3G_OK) {
      pending = b.err;
      return MP3G_OK;
    }
    // read ahead: the scanned batch (or a fresh scan) goes on the device...
    const int other = served ^ 1;
    if (!scanned) scan_batch(bat[other], batch_frames);
    scanned = false;
    Batch& nb = bat[other];
    if (nb.n() == 0) {
      scanned = true;  // only a status: returned by the refill that would serve it
      sc = other;
      return MP3G_OK;
    }
    rc = submit(nb);
    if (rc) return rc;
    inflight = true;
    fl = other;
    // ...and the one after it is scanned while the device decodes
    if (nb.err == MP3G_OK) {
      scan_batch(bat[served], batch_frames);
      scanned = true;
      sc = served;
    }
    return MP3G_OK;
  }

  // ensureFrameStartsAndLength (decode.go:154-216)
  int ensure_length() {
    if (length != -1 || !src.seekable) return MP3G_OK;
    int64_t keep = 0;
    src.seek(0, 1, &keep);
    src.seek(0, 0, nullptr);  // rewind
    src.pos = 0;
    St st = src.skip_tags();
    if (st != St::kOk) return to_status(st);
    int64_t l = 0;
    for (;;) {
      uint32_t h;
      int64_t p = src.pos;
      st = host::read_header(src, &p, &h);
      if (st == St::kEof) break;
      if (st != St::kOk) return to_status(st);
      frame_starts.push_back(p);
      bytes_per_frame = host::header_bytes_per_frame(h);
      l += bytes_per_frame;
      src.seek(host::header_frame_size(h) - 4, 1, nullptr);
    }
    length = l;
    src.seek(keep, 0, nullptr);
    return MP3G_OK;
  }
};

extern "C" {

int mp3g_parse_stream(const uint8_t* data, size_t len, mp3g_granule** granules, int16_t** coeffs,
                      uint64_t* n_granules, int* end_status) {
  if (!granules || !coeffs || !n_granules || !end_status || (len && !data))
    return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *granules = nullptr;
  *coeffs = nullptr;
  *n_granules = 0;
  std::vector<mp3g_granule> g;
  std::vector<int16_t> c;
  *end_status = to_status(parse_all(data, len, &g, &c));
  *n_granules = g.size();
  *granules = static_cast<mp3g_granule*>(std::malloc(std::max<size_t>(1, g.size()) * sizeof(mp3g_granule)));
  *coeffs = static_cast<int16_t*>(std::malloc(std::max<size_t>(1, c.size()) * sizeof(int16_t)));
  if (!*granules || !*coeffs) {
    std::free(*granules);
    std::free(*coeffs);
    *granules = nullptr;
    *coeffs = nullptr;
    return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "parse output");
  }
  if (!g.empty()) std::memcpy(*granules, g.data(), g.size() * sizeof(mp3g_granule));
  if (!c.empty()) std::memcpy(*coeffs, c.data(), c.size() * sizeof(int16_t));
  return MP3G_OK;
}

int mp3g_parse_streams(uint32_t n_streams, const uint8_t* const* datas, const size_t* lens, int n_threads,
                       mp3g_granule** granules, int16_t** coeffs, uint64_t* n_granules, mp3g_stream* streams,
                       int* end_status) {
  if (n_streams && (!datas || !lens || !streams || !end_status))
    return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  if (!granules || !coeffs || !n_granules) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null output");
  std::vector<std::vector<mp3g_granule>> g(n_streams);
  std::vector<std::vector<int16_t>> c(n_streams);
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    for (uint32_t s; (s = next.fetch_add(1)) < n_streams;)
      end_status[s] = to_status(parse_all(datas[s], lens[s], &g[s], &c[s]));
  };
  const int nt = std::max(1, std::min<int>(n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency(),
                                           (int)std::max<uint32_t>(1, n_streams)));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; t++) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  uint64_t total = 0;
  for (uint32_t s = 0; s < n_streams; s++) {
    streams[s].first_granule = total;
    streams[s].n_granules = (uint32_t)g[s].size();
    streams[s].flags = 0;
    total += g[s].size();
  }
  *n_granules = total;
  *granules = static_cast<mp3g_granule*>(std::malloc(std::max<uint64_t>(1, total) * sizeof(mp3g_granule)));
  *coeffs = static_cast<int16_t*>(std::malloc(std::max<uint64_t>(1, total) * MP3G_COEF_PER_GRANULE * sizeof(int16_t)));
  if (!*granules || !*coeffs) {
    std::free(*granules);
    std::free(*coeffs);
    return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "parse output");
  }
  for (uint32_t s = 0; s < n_streams; s++) {
    if (g[s].empty()) continue;
    std::memcpy(*granules + streams[s].first_granule, g[s].data(), g[s].size() * sizeof(mp3g_granule));
    std::memcpy(*coeffs + streams[s].first_granule * MP3G_COEF_PER_GRANULE, c[s].data(),
                c[s].size() * sizeof(int16_t));
  }
  return MP3G_OK;
}

void mp3g_free(void* p) { std::free(p); }

int mp3g_decoder_new(const uint8_t* data, size_t len, int seekable, int device, uint32_t mode,
                     mp3g_decoder** out) {
  if (!out || (len && !data)) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  int ndev = 0;
  if (mp3g_device_count(&ndev) != MP3G_OK || device < 0 || device >= ndev)
    return abi_fail(MP3G_ERR_NO_DEVICE, "no gfx950 device for the decoder");
  mp3g_decoder* d = new (std::nothrow) mp3g_decoder;
  if (!d) return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder");
  d->data.assign(data, data + len);
  d->src.data = d->data.data();
  d->src.len = (int64_t)len;
  d->src.seekable = seekable != 0;
  d->device = device;
  d->mode = mode;
  // NewDecoder (decode.go:361-388): skip tags, read (here: read ahead from)
  // the first frame, take the sample rate, scan frame starts + length
  int rc = to_status(d->src.skip_tags());
  if (rc == MP3G_OK) rc = d->refill();
  if (rc == MP3G_OK) {
    d->sample_rate = host::header_sample_rate(d->first_header);
    rc = d->ensure_length();
  }
  if (rc != MP3G_OK) {
    delete d;
    return rc == MP3G_EOF ? abi_fail(MP3G_EOF, "no MP3 frame") : rc;
  }
  *out = d;
  return MP3G_OK;
}

void mp3g_decoder_free(mp3g_decoder* d) { delete d; }

int mp3g_decoder_read(mp3g_decoder* d, uint8_t* out, size_t cap, size_t* n) {  // decode.go:70-80
  if (!d || !n || (cap && !out)) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *n = 0;
  while (d->buf.size() - d->buf_off == 0) {
    const int rc = d->refill();
    if (rc != MP3G_OK) return rc;
  }
  // like Decoder.Read, never return bytes past the end of the current frame
  // (the reference's d.buf holds one frame; decode.go:70-80)
  while (d->next_end < d->frame_ends.size() && d->frame_ends[d->next_end] <= d->buf_off) d->next_end++;
  const size_t frame_end = d->next_end < d->frame_ends.size() ? d->frame_ends[d->next_end] : d->buf.size();
  const size_t k = std::min(cap, frame_end - d->buf_off);
  std::memcpy(out, d->buf.data() + d->buf_off, k);
  d->buf_off += k;
  d->pos += (int64_t)k;
  *n = k;
  return MP3G_OK;
}

int mp3g_decoder_read_full(mp3g_decoder* d, uint8_t* out, size_t cap, size_t* n) {  // io.ReadFull
  if (!d || !n || (cap && !out)) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *n = 0;
  while (*n < cap) {
    size_t k = 0;
    const int rc = mp3g_decoder_read(d, out + *n, cap - *n, &k);
    *n += k;
    if (rc != MP3G_OK) return rc;
  }
  return MP3G_OK;
}

int mp3g_decoder_seek(mp3g_decoder* d, int64_t offset, int whence, int64_t* newpos) {  // decode.go:89-145
  if (!d || !newpos) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  if (offset == 0 && whence == 1) {
    *newpos = d->pos;
    return MP3G_OK;
  }
  int64_t npos;
  switch (whence) {
    case 0: npos = offset; break;
    case 1: npos = d->pos + offset; break;
    case 2: npos = d->length + offset; break;
    default: return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "mp3: invalid whence");
  }
  d->pos = npos;
  d->cancel_read_ahead();
  d->rewind_read_ahead();
  d->buf_reset();
  d->reset_reservoir();  // d.frame = nil
  d->md.clear();
  d->scan_fresh = true;
  d->pending = MP3G_OK;
  d->batch_frames = 16;
  if (d->pos < 0) d->pos = 0;
  if (d->length != -1 && d->pos >= d->length) {
    *newpos = npos;
    return MP3G_OK;
  }
  // (a non-seekable source never learns bytesPerFrame: the reference's
  // division below panics before its source.Seek could fail)
  if (d->bytes_per_frame <= 0) return abi_fail(MP3G_ERR_UNSUPPORTED, "bytesPerFrame = 0 (the reference divides by zero)");
  if (!d->src.seekable) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "mp3: source must be io.Seeker");
  int64_t f = d->pos / d->bytes_per_frame;
  const int need = f > 0 ? 2 : 1;  // frames the reference reads here
  if (f > 0) f--;
  if (f >= (int64_t)d->frame_starts.size())
    return abi_fail(MP3G_ERR_UNSUPPORTED, "frame index out of range (the reference panics)");
  if (!d->src.seek(d->frame_starts[f], 0, nullptr)) return abi_fail(MP3G_ERR_PARSE, "seek");
  int rc = d->refill();
  if (rc != MP3G_OK) return rc;
  if ((int)d->frame_ends.size() < need) {  // the reference's 2nd readFrame failed
    rc = d->pending;
    d->pending = MP3G_OK;
    return rc;
  }
  const size_t ref_len = d->frame_ends[need - 1];  // the reference's d.buf holds exactly `need` frames here
  const int64_t off = need == 2 ? d->bytes_per_frame + d->pos % d->bytes_per_frame : d->pos;
  if (off > (int64_t)ref_len) return abi_fail(MP3G_ERR_UNSUPPORTED, "slice out of range (the reference panics)");
  d->buf_off = (size_t)off;
  d->next_end = (size_t)need - 1;  // the reference read `need` frames, the last is being served
  *newpos = npos;
  return MP3G_OK;
}

int mp3g_decoder_info(const mp3g_decoder* d, int* sample_rate, int64_t* length, int64_t* bytes_per_frame,
                      int64_t* position) {
  if (!d) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null decoder");
  if (sample_rate) *sample_rate = d->sample_rate;
  if (length) *length = d->length;
  if (bytes_per_frame) *bytes_per_frame = d->bytes_per_frame;
  if (position) *position = d->pos;
  return MP3G_OK;
}

// time API (decode.go:234-354); durations in nanoseconds (time.Duration)
static int64_t bytes_to_ns(const mp3g_decoder* d, int64_t b) {
  return (int64_t)1000000000 * b / (int64_t)(d->sample_rate * 4);
}
int64_t mp3g_decoder_duration_ns(const mp3g_decoder* d) {
  return d->length == -1 ? -1 : bytes_to_ns(d, d->length);
}
int64_t mp3g_decoder_position_ns(const mp3g_decoder* d) { return bytes_to_ns(d, d->pos); }
int64_t mp3g_decoder_remaining_ns(const mp3g_decoder* d) {
  const int64_t dur = mp3g_decoder_duration_ns(d);
  return dur < 0 ? -1 : dur - mp3g_decoder_position_ns(d);
}
double mp3g_decoder_progress(const mp3g_decoder* d) {
  if (d->length == -1) return -1.0;
  if (d->length == 0) return 0.0;
  return (double)d->pos / (double)d->length;
}
int64_t mp3g_decoder_sample_position(const mp3g_decoder* d) { return d->pos / 4; }
int64_t mp3g_decoder_sample_count(const mp3g_decoder* d) { return d->length == -1 ? -1 : d->length / 4; }
int mp3g_decoder_seek_to_sample(mp3g_decoder* d, int64_t s) {
  if (d->length == -1) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "mp3: seek not supported on non-seekable source");
  if (s < 0) s = 0;
  if (s > d->length / 4) s = d->length / 4;
  int64_t np;
  return mp3g_decoder_seek(d, s * 4, 0, &np);
}
int mp3g_decoder_seek_to_time_ns(mp3g_decoder* d, int64_t t) {
  if (d->length == -1) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "mp3: seek not supported on non-seekable source");
  if (t < 0) t = 0;
  const int64_t maxd = mp3g_decoder_duration_ns(d);
  if (t > maxd) t = maxd;
  int64_t b = t * (int64_t)(d->sample_rate * 4) / (int64_t)1000000000;
  b &= ~(int64_t)3;
  int64_t np;
  return mp3g_decoder_seek(d, b, 0, &np);
}
int mp3g_decoder_skip_ns(mp3g_decoder* d, int64_t delta) {
  return mp3g_decoder_seek_to_time_ns(d, mp3g_decoder_position_ns(d) + delta);
}

}  // extern "C"
