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
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/mp3g.h"
#include "abi_util.h"
#include "host_parse.h"
#include "kernels.h"

using namespace mp3g;
using host::St;

namespace {

int to_status(St s) {
  switch (s) {
    case St::kOk: return MP3G_OK;
    case St::kEof: return MP3G_EOF;
    case St::kErr: return MP3G_ERR_PARSE;
    case St::kPanic: return MP3G_ERR_UNSUPPORTED;
    case St::kRead: return MP3G_ERR_READ;
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

// Page-locked blocks for the decoders' PCM read-ahead, pooled per process:
// pinning is the expensive part of a decoder's life (hipHostMalloc of the
// 37 MB a full batch needs takes milliseconds), so a freed decoder's blocks
// serve the next one.  mp3g_release_cached_buffers empties the pool.
namespace {
struct PinnedBlock {
  uint8_t* p;
  size_t cap;
  bool pinned;
};
std::mutex g_pin_mu;
std::vector<PinnedBlock> g_pin_pool;
constexpr size_t kPinPoolMax = 8;

void pin_free(const PinnedBlock& b);

// Frees every idle pooled pinned block (an allocation failed: the pool's idle
// memory goes back before the caller is told it is out of memory).  Returns
// whether anything was freed.
bool pin_drain() {
  std::vector<PinnedBlock> v;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    v.swap(g_pin_pool);
  }
  for (const PinnedBlock& b : v) pin_free(b);
  return !v.empty();
}

PinnedBlock pin_take(size_t need) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    // the smallest pooled block that fits
    size_t best = g_pin_pool.size();
    for (size_t i = 0; i < g_pin_pool.size(); i++)
      if (g_pin_pool[i].cap >= need && (best == g_pin_pool.size() || g_pin_pool[i].cap < g_pin_pool[best].cap)) best = i;
    if (best < g_pin_pool.size()) {
      const PinnedBlock b = g_pin_pool[best];
      g_pin_pool.erase(g_pin_pool.begin() + best);
      return b;
    }
  }
  void* q = nullptr;
  bool pin = hipHostMalloc(&q, need, hipHostMallocDefault) == hipSuccess;
  if (!pin && pin_drain()) pin = hipHostMalloc(&q, need, hipHostMallocDefault) == hipSuccess;
  if (!pin) q = std::malloc(need);
  return {static_cast<uint8_t*>(q), q ? need : 0, pin};
}

void pin_free(const PinnedBlock& b) {
  if (b.pinned) (void)hipHostFree(b.p);
  else std::free(b.p);
}

void pin_give(const PinnedBlock& b) {
  if (!b.p) return;
  PinnedBlock drop{nullptr, 0, false};
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pin_pool.push_back(b);
    if (g_pin_pool.size() > kPinPoolMax) {  // keep the largest blocks
      size_t small = 0;
      for (size_t i = 1; i < g_pin_pool.size(); i++)
        if (g_pin_pool[i].cap < g_pin_pool[small].cap) small = i;
      drop = g_pin_pool[small];
      g_pin_pool.erase(g_pin_pool.begin() + small);
    }
  }
  if (drop.p) pin_free(drop);
}
// Device blocks of the decoders (granules, coefficients, PCM, jobs of a
// batch in one block; the main data in another), pooled per process and
// device like the pinned blocks: a decoder's first batches would otherwise
// pay a hipFree + hipMalloc every time the read-ahead doubles.
struct DevBlock {
  void* p;
  size_t cap;
  int device;
};
std::vector<DevBlock> g_dev_pool;  // guarded by g_pin_mu

DevBlock dev_take(int device, size_t need) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    size_t best = g_dev_pool.size();
    for (size_t i = 0; i < g_dev_pool.size(); i++)
      if (g_dev_pool[i].device == device && g_dev_pool[i].cap >= need &&
          (best == g_dev_pool.size() || g_dev_pool[i].cap < g_dev_pool[best].cap))
        best = i;
    if (best < g_dev_pool.size()) {
      const DevBlock b = g_dev_pool[best];
      g_dev_pool.erase(g_dev_pool.begin() + best);
      return b;
    }
  }
  void* q = nullptr;
  if (hipMalloc(&q, need) != hipSuccess) {
    // idle pooled blocks of this device (too small, or merely unused) may be
    // what the allocation lacks: free them and try once more
    std::vector<DevBlock> idle;
    {
      std::lock_guard<std::mutex> lk(g_pin_mu);
      for (size_t i = 0; i < g_dev_pool.size();)
        if (g_dev_pool[i].device == device) {
          idle.push_back(g_dev_pool[i]);
          g_dev_pool.erase(g_dev_pool.begin() + i);
        } else {
          i++;
        }
    }
    if (idle.empty()) return {nullptr, 0, device};
    for (const DevBlock& b : idle) (void)hipFree(b.p);  // the caller has `device` current
    q = nullptr;
    if (hipMalloc(&q, need) != hipSuccess) return {nullptr, 0, device};
  }
  return {q, need, device};
}

void dev_give(const DevBlock& b) {
  if (!b.p) return;
  DevBlock drop{nullptr, 0, 0};
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_dev_pool.push_back(b);
    if (g_dev_pool.size() > kPinPoolMax) {
      size_t small = 0;
      for (size_t i = 1; i < g_dev_pool.size(); i++)
        if (g_dev_pool[i].cap < g_dev_pool[small].cap) small = i;
      drop = g_dev_pool[small];
      g_dev_pool.erase(g_dev_pool.begin() + small);
    }
  }
  if (drop.p) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(drop.device);
    (void)hipFree(drop.p);
    if (prev >= 0) (void)hipSetDevice(prev);
  }
}
}  // namespace

void release_pinned_pool() {
  std::vector<PinnedBlock> v;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    v.swap(g_pin_pool);
  }
  for (const PinnedBlock& b : v) pin_free(b);
  std::vector<DevBlock> dv;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    dv.swap(g_dev_pool);
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  for (const DevBlock& b : dv) {
    (void)hipSetDevice(b.device);
    (void)hipFree(b.p);
  }
  if (prev >= 0) (void)hipSetDevice(prev);
}

// PCM read-ahead bytes in page-locked memory (from the pool): the batch's
// PCM is copied from the device straight into it (no pageable bounce).
struct PinnedBytes {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  bool pinned = false;
  PinnedBytes() = default;
  PinnedBytes(const PinnedBytes&) = delete;
  PinnedBytes& operator=(const PinnedBytes&) = delete;
  ~PinnedBytes() { release(); }
  void release() {
    if (p) pin_give({p, cap, pinned});
    p = nullptr;
    n = cap = 0;
  }
  size_t size() const { return n; }
  const uint8_t* data() const { return p; }
  void clear() { n = 0; }
  // room for `more` bytes past n (contents kept)
  bool reserve_more(size_t more) {
    if (n + more <= cap) return true;
    const PinnedBlock b = pin_take(std::max(n + more, 2 * cap));
    if (!b.p) return false;
    if (n) std::memcpy(b.p, p, n);
    const size_t keep = n;
    release();
    p = b.p;
    n = keep;
    cap = b.cap;
    pinned = b.pinned;
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
  mp3g_reader reader{};       // streaming input (mp3g_decoder_new_reader): src.rd points here
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
  // the batch's inputs in page-locked memory, so that their H2D copies are
  // asynchronous (reused: a submit follows the previous batch's completion)
  PinnedBytes stage;
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
  DevBlock blk{nullptr, 0, 0}, md_blk{nullptr, 0, 0};  // (pooled) device blocks behind the pointers above
  // the last plan (batches of the same length and state flags reuse it)
  mp3g_plan* plan = nullptr;
  uint64_t plan_n = 0;
  uint32_t plan_flags = 0;
  // diagnostics (MP3G_DEC_STATS=1: printed to stderr when the decoder is freed)
  double t_scan = 0, t_submit = 0, t_wait = 0, t_copy = 0, t_plan = 0, t_pin = 0, t_h2d = 0, t_exec = 0, t_d2h = 0;
  long n_batches = 0;
  std::vector<size_t> frame_ends;         // end offset in buf of each buffered frame
  std::vector<int64_t> frame_src_ends;    // source position after each buffered frame
  // index into frame_ends of the frame the reference read last: Decoder.Read
  // reads one frame once its d.buf is empty (decode.go:70-80), so this is the
  // frame being served, advanced lazily at the next Read like the reference
  size_t next_end = 0;

  ~mp3g_decoder() {
    if (std::getenv("MP3G_DEC_STATS"))
      std::fprintf(stderr, "mp3g_decoder: %ld batches, scan %.2f ms, submit %.2f ms (plan %.2f, pin %.2f, h2d+huffman %.2f, "
                   "dsp %.2f, d2h %.2f), wait %.2f ms, copy %.2f ms\n", n_batches, 1e3 * t_scan, 1e3 * t_submit, 1e3 * t_plan,
                   1e3 * t_pin, 1e3 * t_h2d, 1e3 * t_exec, 1e3 * t_d2h, 1e3 * t_wait, 1e3 * t_copy);
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (plan) mp3g_plan_destroy(plan);
    buf.release();
    ahead.release();
    if (d_state) (void)hipFree(d_state);
    dev_give(blk);
    dev_give(md_blk);
    if (stream) (void)hipStreamDestroy(stream);
    if (prev >= 0) (void)hipSetDevice(prev);
  }

  int ensure_capacity(size_t n) {
    if (n <= cap_granules) return MP3G_OK;
    // at least 4,096 granules: the doubling read-ahead then reallocates twice
    const size_t cap = std::max<size_t>({n, cap_granules * 2, 4096});
    constexpr size_t kPerGranule =
        sizeof(mp3g_granule) + MP3G_COEF_PER_GRANULE * sizeof(int16_t) + MP3G_PCM_BYTES_PER_GRANULE + 2 * sizeof(mp3g_hjob);
    dev_give(blk);
    blk = dev_take(device, cap * kPerGranule);
    if (!blk.p) {
      cap_granules = 0;
      d_gran = nullptr;
      d_coef = d_pcm = nullptr;
      d_jobs = nullptr;
      return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder device buffers");
    }
    const size_t have = blk.cap / kPerGranule;  // a pooled block may be larger
    uint8_t* q = static_cast<uint8_t*>(blk.p);
    d_gran = reinterpret_cast<mp3g_granule*>(q);
    q += have * sizeof(mp3g_granule);
    d_coef = reinterpret_cast<int16_t*>(q);
    q += have * MP3G_COEF_PER_GRANULE * sizeof(int16_t);
    d_pcm = reinterpret_cast<int16_t*>(q);
    q += have * MP3G_PCM_BYTES_PER_GRANULE;
    d_jobs = reinterpret_cast<mp3g_hjob*>(q);
    cap_granules = have;
    return MP3G_OK;
  }

  bool gpu_huffman() const { return (mode & MP3G_FLAG_HOST_HUFFMAN) == 0; }

  // Scans (or parses) up to `max_frames` frames into b.  A failing frame ends
  // the batch: b.err, the reservoir is dropped and the next batch starts from
  // zero DSP state (d.frame = nil after a failed frame.Read).  `must`: the
  // batch is the one Read serves next, so a streaming source without a
  // seeker may be read (it may block) until it holds one frame; otherwise
  // such a source contributes only the frames that have fully arrived, and
  // the batch may come out empty with b.err == MP3G_OK (host::scan_some).
  void scan_batch(Batch& b, size_t max_frames, bool must) {
    const auto t0 = std::chrono::steady_clock::now();
    struct Acc {
      double& t;
      std::chrono::steady_clock::time_point t0;
      ~Acc() { t += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
    } acc{t_scan, t0};
    b.clear();
    b.fresh = scan_fresh;
    St st;
    if (gpu_huffman()) {
      // drop main data no later frame can reach (the reservoir is < 2 KB)
      const int64_t dead = scanner.live_start(md);
      if (dead > 0) {
        md.erase(md.begin(), md.begin() + dead);
        scanner.drop(dead);
      }
      st = host::scan_some(src, scanner, &md, max_frames, must, [](void* ctx, const host::ScannedFrame& f, int64_t sp) {
        Batch& b = *static_cast<Batch*>(ctx);
        for (int gr = 0; gr < f.n_granules; gr++) {
          b.gran.push_back(f.gran[gr]);
          b.jobs.push_back(f.job[gr][0]);
          b.jobs.push_back(f.job[gr][1]);
        }
        b.frame_pcm_bytes.push_back((uint32_t)(f.n_granules * MP3G_PCM_BYTES_PER_GRANULE));
        b.frame_src.push_back(sp);
      }, &b);
      if (!b.gran.empty()) b.md.assign(md.begin(), md.end());  // the scanner keeps editing md
    } else {
      st = host::parse_some(src, parser, max_frames, must, [](void* ctx, const host::ParsedFrame& f, int64_t sp) {
        Batch& b = *static_cast<Batch*>(ctx);
        for (int gr = 0; gr < f.n_granules; gr++) {
          b.gran.push_back(f.gran[gr]);
          b.coef.insert(b.coef.end(), f.coef[gr], f.coef[gr] + MP3G_COEF_PER_GRANULE);
        }
        b.frame_pcm_bytes.push_back((uint32_t)(f.n_granules * MP3G_PCM_BYTES_PER_GRANULE));
        b.frame_src.push_back(sp);
      }, &b);
    }
    b.err = st == St::kOk ? MP3G_OK : to_status(st);
    if (b.err != MP3G_OK) {
      reset_reservoir();
      scan_fresh = true;
    } else if (!b.gran.empty()) {
      scan_fresh = false;
    }  // (an empty batch that has not arrived yet changes nothing)
    if (!b.gran.empty()) batch_frames = std::min<size_t>(batch_frames * 2, kMaxBatchFrames);
  }

  // A scanned batch worth keeping for the next refill: frames, or a status.
  static bool has_news(const Batch& b) { return b.n() > 0 || b.err != MP3G_OK; }

  void reset_reservoir() {
    parser.reset();
    scanner.reset();
  }

  // Enqueues batch b (n() > 0) on the decoder's stream: H2D, Huffman kernel,
  // DSP plan (state carried on the device), PCM D2H into `ahead`.
  int submit(const Batch& b) {
    struct Acc {
      double& t;
      std::chrono::steady_clock::time_point t0;
      ~Acc() { t += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
    } acc{t_submit, std::chrono::steady_clock::now()};
    n_batches++;
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
    auto tp0 = std::chrono::steady_clock::now();
    auto lap = [&](double& t) {
      const auto now = std::chrono::steady_clock::now();
      t += std::chrono::duration<double>(now - tp0).count();
      tp0 = now;
    };
    if (!plan || plan_n != n || plan_flags != s.flags) {
      if (plan) mp3g_plan_destroy(plan);
      plan = nullptr;
      rc = mp3g_plan_create(device, &s, 1, 0, mode & ~(uint32_t)MP3G_FLAG_HOST_HUFFMAN, &plan);
      if (rc) return rc;
      plan_n = n;
      plan_flags = s.flags;
    }
    lap(t_plan);
    const size_t pcm_bytes = n * MP3G_PCM_BYTES_PER_GRANULE;
    ahead.clear();
    if (!ahead.reserve_more(pcm_bytes)) return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder PCM buffer");
    lap(t_pin);
    // inputs into the pinned stage, then asynchronous H2D copies
    const size_t b_gran = n * sizeof(mp3g_granule);
    const size_t b_in = gpu_huffman() ? b.jobs.size() * sizeof(mp3g_hjob) + b.md.size()
                                      : b.coef.size() * sizeof(int16_t);
    stage.clear();
    if (!stage.reserve_more(b_gran + b_in)) return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder staging buffer");
    uint8_t* sg = stage.p;
    std::memcpy(sg, b.gran.data(), b_gran);
    hipError_t e = hipMemcpyAsync(d_gran, sg, b_gran, hipMemcpyHostToDevice, stream);
    uint8_t* si = sg + b_gran;
    if (gpu_huffman()) {
      // main data + jobs up, then scale factors / Huffman codes on the device
      const size_t mdb = b.md.size() + 16;  // + padding for the 32-bit window loads
      if (e == hipSuccess && mdb > cap_md) {
        dev_give(md_blk);
        md_blk = dev_take(device, std::max<size_t>({mdb, 2 * cap_md, size_t(1) << 20}));
        d_md = static_cast<uint8_t*>(md_blk.p);
        cap_md = md_blk.cap;
        if (!d_md) e = hipErrorOutOfMemory;
      }
      const size_t b_jobs = b.jobs.size() * sizeof(mp3g_hjob);
      std::memcpy(si, b.jobs.data(), b_jobs);
      if (!b.md.empty()) std::memcpy(si + b_jobs, b.md.data(), b.md.size());
      if (e == hipSuccess && !b.md.empty())
        e = hipMemcpyAsync(d_md, si + b_jobs, b.md.size(), hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) e = hipMemcpyAsync(d_jobs, si, b_jobs, hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) {
        rc = mp3g_huffman_execute_ex(device, d_jobs, n, d_md, d_gran, d_coef,
                                     (mode_reads_to_count1(mode) ? MP3G_HUFF_ROWS_COUNT1 : 0u) |
                                         mp3g_huffman_stage_flags(b.jobs.data(), n),
                                     stream);
        if (rc) return rc;
      }
    } else if (e == hipSuccess) {
      std::memcpy(si, b.coef.data(), b_in);
      e = hipMemcpyAsync(d_coef, si, b_in, hipMemcpyHostToDevice, stream);
    }
    if (e != hipSuccess) return abi_fail(MP3G_ERR_DEVICE, "decoder H2D copy");
    lap(t_h2d);
    rc = mp3g_plan_execute(plan, d_gran, d_coef, d_state, d_state + 1, d_pcm, stream);
    if (rc) return rc;
    lap(t_exec);
    // into the pinned read-ahead block by our copy kernel (HIP's device -> host
    // DMA copy moves ~30 GB/s, the kernel 54-55: kernels.hip launch_copy_out)
    void* ahead_dev = nullptr;
    if (ahead.pinned && hipHostGetDevicePointer(&ahead_dev, ahead.p, 0) == hipSuccess && ahead_dev)
      e = launch_copy_out(d_pcm, ahead_dev, pcm_bytes, 2048, stream);
    else
      e = hipMemcpyAsync(ahead.p, d_pcm, pcm_bytes, hipMemcpyDeviceToHost, stream);
    lap(t_d2h);
    // carry: out -> in for the next batch
    if (e == hipSuccess) e = hipMemcpyAsync(d_state, d_state + 1, sizeof(mp3g_state), hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return abi_fail(MP3G_ERR_DEVICE, "decoder batch");
    ahead.n = pcm_bytes;
    return MP3G_OK;
  }

  // Waits for the batch on the device and makes it the served buffer.
  int complete(const Batch& b) {
    const auto t0 = std::chrono::steady_clock::now();
    if (hipStreamSynchronize(stream) != hipSuccess) return abi_fail(MP3G_ERR_DEVICE, "decoder batch");
    t_wait += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
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
  // false: the source's Seek failed (the reader's error is then pending in
  // src.read_failed, for seek_status)
  bool rewind_read_ahead() {
    return next_end >= frame_src_ends.size() || src.seek(frame_src_ends[next_end], 0, nullptr);
  }

  // The status of a failed source Seek: the Seeker's own error in reader mode
  // (decode.go:164-214 and :128-133 return it), MP3G_ERR_PARSE over bytes
  // (a bytes.Reader fails only on a negative position).
  int seek_status(const char* what) {
    if (src.rd) {
      src.read_failed = true;
      return read_status(St::kErr);
    }
    return abi_fail(MP3G_ERR_PARSE, what);
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
      if (!scanned) scan_batch(bat[served], batch_frames, true);
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
    if (!scanned) scan_batch(bat[other], batch_frames, false);
    scanned = false;
    Batch& nb = bat[other];
    if (nb.n() == 0) {
      // only a status, returned by the refill that would serve it -- or
      // nothing that has arrived yet (streaming), scanned again by that refill
      scanned = nb.err != MP3G_OK;
      sc = other;
      return MP3G_OK;
    }
    rc = submit(nb);
    if (rc) return rc;
    inflight = true;
    fl = other;
    // ...and the one after it is scanned while the device decodes
    if (nb.err == MP3G_OK) {
      scan_batch(bat[served], batch_frames, false);
      scanned = has_news(bat[served]);
      sc = served;
    }
    return MP3G_OK;
  }

  // A status of a source operation outside scan_some: a reader error is the
  // reader's, whatever the short read looked like (decode.go:48-63).
  int read_status(St st) {
    const bool failed = src.read_failed;
    src.read_failed = false;
    return failed ? MP3G_ERR_READ : to_status(st);
  }

  // ensureFrameStartsAndLength (decode.go:154-216)
  int ensure_length() {
    if (length != -1 || !src.seekable) return MP3G_OK;
    int64_t keep = 0;
    if (!src.seek(0, 1, &keep)) return seek_status("seek");
    if (!src.seek(0, 0, nullptr)) return seek_status("rewind");
    src.pos = 0;
    St st = src.skip_tags();
    if (st != St::kOk) return read_status(st);
    int64_t l = 0;
    for (;;) {
      uint32_t h;
      int64_t p = src.pos;
      src.keep_from = src.rpos;  // (reader mode: the walk needs no window behind it)
      st = host::read_header(src, &p, &h);
      if (st == St::kEof && !src.read_failed) break;
      if (st != St::kOk) return read_status(st);
      frame_starts.push_back(p);
      bytes_per_frame = host::header_bytes_per_frame(h);
      l += bytes_per_frame;
      if (!src.seek(host::header_frame_size(h) - 4, 1, nullptr)) return seek_status("seek");
    }
    length = l;
    if (!src.seek(keep, 0, nullptr)) return seek_status("seek");
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

// NewDecoder (decode.go:361-388) on a prepared source: skip tags, read (here:
// read ahead from) the first frame, take the sample rate, scan frame starts +
// length (seekers only).
static int decoder_start(mp3g_decoder* d, mp3g_decoder** out) {
  int rc = d->read_status(d->src.skip_tags());
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

static mp3g_decoder* decoder_alloc(int device, uint32_t mode, int* rc) {
  int ndev = 0;
  if (mp3g_device_count(&ndev) != MP3G_OK || device < 0 || device >= ndev) {
    *rc = abi_fail(MP3G_ERR_NO_DEVICE, "no gfx950 device for the decoder");
    return nullptr;
  }
  mp3g_decoder* d = new (std::nothrow) mp3g_decoder;
  if (!d) {
    *rc = abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decoder");
    return nullptr;
  }
  d->device = device;
  d->mode = mode;
  *rc = MP3G_OK;
  return d;
}

int mp3g_decoder_new(const uint8_t* data, size_t len, int seekable, int device, uint32_t mode,
                     mp3g_decoder** out) {
  if (!out || (len && !data)) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  int rc;
  mp3g_decoder* d = decoder_alloc(device, mode, &rc);
  if (!d) return rc;
  d->data.assign(data, data + len);
  d->src.data = d->data.data();
  d->src.len = (int64_t)len;
  d->src.seekable = seekable != 0;
  return decoder_start(d, out);
}

int mp3g_decoder_new_reader(const mp3g_reader* reader, int device, uint32_t mode, mp3g_decoder** out) {
  if (!out || !reader || !reader->read) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  int rc;
  mp3g_decoder* d = decoder_alloc(device, mode, &rc);
  if (!d) return rc;
  d->reader = *reader;
  d->src.rd = &d->reader;
  d->src.seekable = reader->seek != nullptr;
  return decoder_start(d, out);
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
  // io.ReadFull loops Decoder.Read (one frame's PCM at most per call); the
  // bytes it collects are the served PCM in order, so this copies whole spans
  // of the served batch at once and leaves the frame index where the last of
  // those Reads would (the frame holding the last byte copied).
  if (!d || !n || (cap && !out)) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *n = 0;
  while (*n < cap) {
    if (d->buf.size() - d->buf_off == 0) {
      const int rc = d->refill();
      if (rc != MP3G_OK) return rc;
      continue;
    }
    const size_t k = std::min(cap - *n, d->buf.size() - d->buf_off);
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(out + *n, d->buf.data() + d->buf_off, k);
    d->t_copy += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    d->buf_off += k;
    d->pos += (int64_t)k;
    *n += k;
    while (d->next_end < d->frame_ends.size() && d->frame_ends[d->next_end] < d->buf_off) d->next_end++;
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
  if (!d->rewind_read_ahead()) return d->seek_status("seek");
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
  if (!d->src.seek(d->frame_starts[f], 0, nullptr)) return d->seek_status("seek");
  int rc = d->refill();
  if (rc != MP3G_OK) return rc;
  if ((int)d->frame_ends.size() < need) {  // the reference's 2nd readFrame failed
    rc = d->pending;
    d->pending = MP3G_OK;
    // its source now stands after the failed frame (where the scan stopped): a
    // later seek that reads nothing must not rewind it to the frame before
    d->frame_src_ends.clear();
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
