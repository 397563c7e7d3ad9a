// host_scan.cpp -- batch entry points of the GPU main-data path (SURVEY.md 8f
// row f1): mp3g_scan_streams (host: tags, headers, side info, reservoir --
// host_parse.cpp FrameScanner) and mp3g_decode_streams (bitstreams in, PCM
// out: the scan, then Huffman + DSP on the device).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
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

// An uninitialised array (the scan overwrites every byte; zeroing hundreds
// of MB first would cost as much as writing them), in transparent huge pages
// where the kernel offers them (madvise mode): the first touch of each fresh
// 4-KB page costs about as much as filling it.
template <class T>
struct Buf {
  T* p = nullptr;
  size_t n = 0, bytes = 0;
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  ~Buf() { release(); }
  void release() {
    if (p) munmap(p, bytes);
    p = nullptr;
    n = bytes = 0;
  }
  bool alloc(size_t count) {
    release();
    const size_t huge = size_t(2) << 20;
    bytes = (std::max<size_t>(count, 1) * sizeof(T) + huge - 1) & ~(huge - 1);
    void* q = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (q == MAP_FAILED) {
      bytes = 0;
      return false;
    }
    madvise(q, bytes, MADV_HUGEPAGE);  // advisory: 4-KB pages if refused
    p = static_cast<T*>(q);
    n = count;
    return true;
  }
  T* data() const { return p; }
  size_t size() const { return n; }
  T& operator[](size_t i) const { return p[i]; }
};

}  // namespace

struct mp3g_scan {
  Buf<mp3g_granule> gran;
  Buf<mp3g_hjob> jobs;
  Buf<uint8_t> md;
  std::vector<mp3g_stream> streams;
  std::vector<int> status;
};

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

struct StreamScan {
  std::vector<mp3g_granule> gran;
  std::vector<mp3g_hjob> jobs;  // positions relative to md
  std::vector<uint8_t> md;
  St end = St::kOk;
};

// NewDecoder + reading to the end (as host_decoder.cpp parse_all).
void scan_all(const uint8_t* data, size_t len, StreamScan* out) {
  host::Source src;
  src.data = data;
  src.len = (int64_t)len;
  St st = src.skip_tags();
  if (st != St::kOk) {
    out->end = st;
    return;
  }
  out->md.reserve(len);
  const size_t frames_est = len / 96 + 16;  // >= 1 frame per 96 bytes at 8 kbps... an estimate, not a bound
  out->gran.reserve(2 * frames_est);
  out->jobs.reserve(4 * frames_est);
  host::FrameScanner sc;
  host::ScannedFrame f;
  for (;;) {
    st = sc.next(src, &f, &out->md);
    if (st != St::kOk) break;
    for (int gr = 0; gr < f.n_granules; gr++) {
      out->gran.push_back(f.gran[gr]);
      out->jobs.push_back(f.job[gr][0]);
      out->jobs.push_back(f.job[gr][1]);
    }
  }
  out->end = st;
}

// The same scan written straight into the concatenation: granules from
// gran[0], jobs from jobs[0], main data appended to *md (positions in the
// jobs are then absolute).  Returns the granules written; more than `cap`
// granules or main data past md->cap stops with *overflow set.
uint64_t scan_into(const uint8_t* data, size_t len, mp3g_granule* gran, mp3g_hjob* jobs, uint64_t cap,
                   host::RawMd* md, St* end, bool* overflow) {
  host::Source src;
  src.data = data;
  src.len = (int64_t)len;
  *overflow = false;
  St st = src.skip_tags();
  if (st != St::kOk) {
    *end = st;
    return 0;
  }
  host::FrameScanner sc;
  host::ScannedFrame f;
  uint64_t n = 0;
  for (;;) {
    st = sc.next(src, &f, md);
    if (st != St::kOk) break;
    if (n + (uint64_t)f.n_granules > cap) {
      *overflow = true;
      break;
    }
    for (int gr = 0; gr < f.n_granules; gr++, n++) {
      gran[n] = f.gran[gr];
      jobs[2 * n] = f.job[gr][0];
      jobs[2 * n + 1] = f.job[gr][1];
    }
  }
  *overflow = *overflow || md->overflow;
  *end = st;
  return n;
}

// fn(k) for k in [k0, k1) on up to nt threads (the calling thread included)
template <class Fn>
void parallel_for(uint32_t k0, uint32_t k1, int nt, Fn&& fn) {
  std::atomic<uint32_t> next{k0};
  auto work = [&]() {
    for (uint32_t k; (k = next.fetch_add(1)) < k1;) fn(k);
  };
  nt = std::max(1, std::min<int>(nt, (int)(k1 - k0)));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; t++) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
}

// page-locked host memory and device memory that grow on demand
struct Pinned {
  void* p = nullptr;
  size_t bytes = 0;
  ~Pinned() {
    if (p) (void)hipHostFree(p);
  }
  bool reserve(size_t b) {
    if (b <= bytes) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    if (hipHostMalloc(&p, b, hipHostMallocDefault) != hipSuccess) return false;
    bytes = b;
    return true;
  }
};
struct DevMem {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
  bool reserve(size_t b) {
    if (b <= bytes) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, b) != hipSuccess) return false;
    bytes = b;
    return true;
  }
};

// Staging and device buffers of mp3g_decode_streams_into, kept per device
// between calls (grow-only; mp3g_release_cached_buffers frees them): a
// multi-GB batch otherwise spends tens of ms pinning host memory and
// allocating device memory in every call.  A call that finds its device's
// set in use by another thread allocates its own.
struct PipeBufs {
  Pinned arena[2];
  DevMem d_gran[2], d_jobs[2], d_md[2], d_chunks[2], d_pcm[2], d_coef;
  // the fast kernel's deferred hot zones (kernels.h ZoneScratch), used by the
  // launches on `comp` in order
  DevMem d_zones;
  uint32_t zone_cap = 0;
  // the pipeline's streams and per-slot events (created once per device)
  hipStream_t up = nullptr, comp = nullptr, down = nullptr;
  hipEvent_t h2d[2] = {}, kern[2] = {}, d2h[2] = {};
  bool ensure_sync() {
    if (!down && !create_down()) return false;
    for (hipStream_t* q : {&up, &comp})
      if (!*q && hipStreamCreateWithFlags(q, hipStreamNonBlocking) != hipSuccess) return false;
    for (int i = 0; i < 2; i++)
      for (hipEvent_t* ev : {&h2d[i], &kern[i], &d2h[i]})
        if (!*ev && hipEventCreateWithFlags(ev, hipEventDisableTiming) != hipSuccess) return false;
    return true;
  }
  // The PCM copy-out's stream, limited to a few CUs spread over the XCDs
  // (MP3G_PIPE_DOWN_CUS: that many, 0 = unrestricted).  Into pinned memory the
  // copy-out is a kernel of ours (launch_copy_out: 54-55 GB/s from 16 CUs,
  // where hipMemcpyAsync's DMA engine moved 30 GB/s without a profiler and a
  // blit kernel under one: tools/copy_exp.hip); restricted, it leaves the
  // decode kernels the other CUs (an unrestricted blit had stretched the
  // main-data kernel 0.14 -> 5.9 ms per group, the r05i timeline).
  int down_cus = 0;
  bool create_down() {
    int dev = 0, ncu = 0;
    const char* env = std::getenv("MP3G_PIPE_DOWN_CUS");
    int want = env ? std::atoi(env) : 16;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 0;
    down_cus = want > 0 && want < ncu ? want : ncu > 0 ? ncu : 256;
    if (want <= 0 || ncu <= 0 || want >= ncu) return hipStreamCreateWithFlags(&down, hipStreamNonBlocking) == hipSuccess;
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    for (int i = 0; i < want; i++) {
      const int cu = (int)((int64_t)i * ncu / want);
      mask[(size_t)cu / 32] |= 1u << (cu % 32);
    }
    return hipExtStreamCreateWithCUMask(&down, (uint32_t)mask.size(), mask.data()) == hipSuccess;
  }
  ~PipeBufs() {
    for (hipStream_t q : {up, comp, down})
      if (q) (void)hipStreamDestroy(q);
    for (int i = 0; i < 2; i++)
      for (hipEvent_t ev : {h2d[i], kern[i], d2h[i]})
        if (ev) (void)hipEventDestroy(ev);
  }
};

// MP3G_PIPE_TRACE=1: host timestamps of mp3g_decode_streams_into's stages on
// stderr (diagnostic; tools/pipe_time.py)
struct PipeTrace {
  bool on;
  std::chrono::steady_clock::time_point t0;
  PipeTrace() : on(std::getenv("MP3G_PIPE_TRACE") != nullptr), t0(std::chrono::steady_clock::now()) {}
  void mark(const char* what, long group = -1) const {
    if (!on) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (group >= 0)
      std::fprintf(stderr, "mp3g pipe %9.3f ms %s %ld\n", ms, what, group);
    else
      std::fprintf(stderr, "mp3g pipe %9.3f ms %s\n", ms, what);
  }
};
std::mutex g_pipe_mu;
std::vector<std::unique_ptr<PipeBufs>> g_pipe;  // [device]
std::vector<bool> g_pipe_busy;

}  // namespace

void release_pinned_pool();  // host_decoder.cpp: the decoders' pinned PCM pool

extern "C" {

void mp3g_release_cached_buffers(void) {
  release_pinned_pool();
  std::lock_guard<std::mutex> lk(g_pipe_mu);
  int prev = -1;
  (void)hipGetDevice(&prev);
  for (size_t d = 0; d < g_pipe.size(); d++)
    if (g_pipe[d] && !g_pipe_busy[d]) {
      (void)hipSetDevice((int)d);
      g_pipe[d].reset();
    }
  if (prev >= 0) (void)hipSetDevice(prev);
}

int mp3g_scan_streams(uint32_t n_streams, const uint8_t* const* datas, const size_t* lens, int n_threads,
                      mp3g_scan** out) {
  if (!out || (n_streams && (!datas || !lens))) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  mp3g_scan* s = new (std::nothrow) mp3g_scan;
  if (!s) return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "scan");
  std::vector<StreamScan> per(n_streams);
  const int nt = std::max(1, std::min<int>(n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency(),
                                           (int)std::max<uint32_t>(1, n_streams)));
  auto parallel = [&](auto&& fn) {  // fn(k) for every stream, on nt threads
    std::atomic<uint32_t> next{0};
    auto work = [&]() {
      for (uint32_t k; (k = next.fetch_add(1)) < n_streams;) fn(k);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
  };
  // Direct path: a header-only pre-pass sizes every stream, then each stream
  // is scanned straight into its place in the concatenation (no per-stream
  // buffers, no merge copy).  A stream whose side info ends it before the
  // pre-pass's count (a parse error or a reference panic mid-stream) sends the
  // batch to the two-step path below.
  {
    std::vector<uint64_t> pg(n_streams), pm(n_streams);
    parallel([&](uint32_t k) { host::prescan(datas[k], lens[k], &pg[k], &pm[k]); });
    std::vector<uint64_t> g_at(n_streams + 1), m_at(n_streams + 1);
    for (uint32_t k = 0; k < n_streams; k++) {
      g_at[k + 1] = g_at[k] + pg[k];
      m_at[k + 1] = m_at[k] + ((pm[k] + 15) & ~(uint64_t)15);
    }
    const uint64_t ng = g_at[n_streams], nmd = m_at[n_streams];
    if (!s->gran.alloc(ng) || !s->jobs.alloc(2 * ng) || !s->md.alloc(nmd + 16)) {
      delete s;
      return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "scan buffers");
    }
    s->streams.resize(n_streams);
    s->status.resize(n_streams);
    std::atomic<bool> ok{true};
    parallel([&](uint32_t k) {
      host::RawMd md;
      md.base = s->md.data();
      md.n = m_at[k];
      md.cap = m_at[k] + pm[k];
      St end;
      bool overflow;
      const uint64_t n = scan_into(datas[k], lens[k], &s->gran[g_at[k]], &s->jobs[2 * g_at[k]], pg[k], &md, &end,
                                   &overflow);
      if (overflow || n != pg[k] || md.n != m_at[k] + pm[k]) {
        ok = false;
        return;
      }
      s->streams[k].first_granule = g_at[k];
      s->streams[k].n_granules = (uint32_t)n;
      s->streams[k].flags = 0;
      s->status[k] = to_status(end);
      std::memset(&s->md[md.n], 0, m_at[k + 1] + (k + 1 == n_streams ? 16 : 0) - md.n);
    });
    if (ok) {
      *out = s;
      return MP3G_OK;
    }
    s->streams.clear();
    s->status.clear();
  }
  parallel([&](uint32_t k) { scan_all(datas[k], lens[k], &per[k]); });

  // where each stream lands; each stream's main data 16-B aligned, 16 zero
  // bytes of padding after the last (the device reads whole 8-B words)
  std::vector<uint64_t> g_at(n_streams + 1), m_at(n_streams + 1);
  for (uint32_t k = 0; k < n_streams; k++) {
    g_at[k + 1] = g_at[k] + per[k].gran.size();
    m_at[k + 1] = m_at[k] + ((per[k].md.size() + 15) & ~(size_t)15);
  }
  const uint64_t ng = g_at[n_streams], nmd = m_at[n_streams];
  if (!s->gran.alloc(ng) || !s->jobs.alloc(2 * ng) || !s->md.alloc(nmd + 16)) {
    delete s;
    return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "scan buffers");
  }
  s->streams.resize(n_streams);
  s->status.resize(n_streams);
  std::memset(s->md.data() + nmd, 0, 16);
  parallel([&](uint32_t k) {
    StreamScan& p = per[k];
    const uint64_t g = g_at[k], m = m_at[k];
    s->streams[k].first_granule = g;
    s->streams[k].n_granules = (uint32_t)p.gran.size();
    s->streams[k].flags = 0;
    s->status[k] = to_status(p.end);
    if (!p.gran.empty()) std::memcpy(&s->gran[g], p.gran.data(), p.gran.size() * sizeof(mp3g_granule));
    for (size_t i = 0; i < p.jobs.size(); i++) {
      mp3g_hjob J = p.jobs[i];
      if (J.sf_kind != MP3G_SF_NONE) {
        J.part2_start += 8 * m;
        J.bit_end += 8 * m;
      }
      s->jobs[2 * g + i] = J;
    }
    if (!p.md.empty()) std::memcpy(&s->md[m], p.md.data(), p.md.size());
    std::memset(&s->md[m + p.md.size()], 0, m_at[k + 1] - m - p.md.size());
    std::vector<mp3g_granule>().swap(p.gran);  // release as we go
    std::vector<mp3g_hjob>().swap(p.jobs);
    std::vector<uint8_t>().swap(p.md);
  });
  *out = s;
  return MP3G_OK;
}

int mp3g_scan_buffers(const mp3g_scan* s, uint64_t* n_granules, uint64_t* main_data_bytes,
                      const mp3g_granule** granules, const mp3g_hjob** jobs, const uint8_t** main_data,
                      const mp3g_stream** streams, const int** end_status) {
  if (!s) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null scan");
  if (n_granules) *n_granules = s->gran.size();
  if (main_data_bytes) *main_data_bytes = s->md.size();
  if (granules) *granules = s->gran.data();
  if (jobs) *jobs = s->jobs.data();
  if (main_data) *main_data = s->md.data();
  if (streams) *streams = s->streams.data();
  if (end_status) *end_status = s->status.data();
  return MP3G_OK;
}

void mp3g_scan_free(mp3g_scan* s) { delete s; }

int mp3g_decode_streams(int device, uint32_t n_streams, const uint8_t* const* datas, const size_t* lens,
                        int n_threads, uint32_t mode, int16_t** pcm, uint64_t* n_granules, mp3g_stream* streams,
                        int* end_status) {
  if (!pcm || !n_granules || (n_streams && (!streams || !end_status)))
    return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *pcm = nullptr;
  *n_granules = 0;
  mp3g_scan* s = nullptr;
  int rc = mp3g_scan_streams(n_streams, datas, lens, n_threads, &s);
  if (rc) return rc;
  const size_t n = s->gran.size();
  if (n_streams) {
    std::memcpy(streams, s->streams.data(), n_streams * sizeof(mp3g_stream));
    std::memcpy(end_status, s->status.data(), n_streams * sizeof(int));
  }
  int16_t* host_pcm = static_cast<int16_t*>(std::malloc(std::max<size_t>(1, n) * MP3G_PCM_BYTES_PER_GRANULE));
  if (!host_pcm) {
    mp3g_scan_free(s);
    return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "pcm");
  }
  if (n == 0) {
    mp3g_scan_free(s);
    *pcm = host_pcm;
    return MP3G_OK;
  }
  mp3g_plan* plan = nullptr;
  rc = mp3g_plan_create(device, s->streams.data(), n_streams, 0, mode, &plan);
  if (rc) {
    mp3g_scan_free(s);
    std::free(host_pcm);
    return rc;
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  void *dg = nullptr, *dj = nullptr, *dm = nullptr, *dc = nullptr, *dp = nullptr;
  hipStream_t st = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&dg, n * sizeof(mp3g_granule));
  if (e == hipSuccess) e = hipMalloc(&dj, 2 * n * sizeof(mp3g_hjob));
  if (e == hipSuccess) e = hipMalloc(&dm, s->md.size());
  if (e == hipSuccess) e = hipMalloc(&dc, n * MP3G_COEF_PER_GRANULE * sizeof(int16_t));
  if (e == hipSuccess) e = hipMalloc(&dp, n * MP3G_PCM_BYTES_PER_GRANULE);
  if (e == hipSuccess) e = hipMemcpyAsync(dg, s->gran.data(), n * sizeof(mp3g_granule), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(dj, s->jobs.data(), 2 * n * sizeof(mp3g_hjob), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(dm, s->md.data(), s->md.size(), hipMemcpyHostToDevice, st);
  rc = e == hipSuccess ? MP3G_OK : abi_fail(MP3G_ERR_DEVICE, "decode_streams: device buffers / H2D");
  if (rc == MP3G_OK)
    rc = mp3g_huffman_execute_ex(device, (const mp3g_hjob*)dj, n, (const uint8_t*)dm, (mp3g_granule*)dg,
                                 (int16_t*)dc,
                                 (mode_reads_to_count1(mode) ? MP3G_HUFF_ROWS_COUNT1 : 0u) |
                                     mp3g_huffman_stage_flags(s->jobs.data(), n),
                                 st);
  if (rc == MP3G_OK)
    rc = mp3g_plan_execute(plan, (const mp3g_granule*)dg, (const int16_t*)dc, nullptr, nullptr, (int16_t*)dp, st);
  if (rc == MP3G_OK) {
    e = hipMemcpyAsync(host_pcm, dp, n * MP3G_PCM_BYTES_PER_GRANULE, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams: decode / D2H");
  }
  for (void* q : {dg, dj, dm, dc, dp})
    if (q) (void)hipFree(q);
  if (st) (void)hipStreamDestroy(st);
  if (prev >= 0) (void)hipSetDevice(prev);
  mp3g_plan_destroy(plan);
  mp3g_scan_free(s);
  if (rc) {
    std::free(host_pcm);
    return rc;
  }
  *pcm = host_pcm;
  *n_granules = n;
  return MP3G_OK;
}

int mp3g_decode_streams_into(int device, uint32_t n_streams, const uint8_t* const* datas, const size_t* lens,
                             int n_threads, uint32_t mode, uint32_t n_groups, int16_t* pcm,
                             uint64_t pcm_cap_granules, uint64_t* n_granules, mp3g_stream* streams,
                             int* end_status) {
  if (!n_granules || (n_streams && (!datas || !lens || !streams || !end_status)))
    return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *n_granules = 0;
  const int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  const PipeTrace trace;
  // ---- the layout: a header-only pre-pass over every stream ----
  std::vector<uint64_t> pg(n_streams), pm(n_streams), g_at(n_streams + 1), m_at(n_streams + 1);
  parallel_for(0, n_streams, nt, [&](uint32_t k) { host::prescan(datas[k], lens[k], &pg[k], &pm[k]); });
  trace.mark("prescan");
  for (uint32_t k = 0; k < n_streams; k++) {
    g_at[k + 1] = g_at[k] + pg[k];
    m_at[k + 1] = m_at[k] + ((pm[k] + 15) & ~(uint64_t)15);
  }
  const uint64_t total = g_at[n_streams];
  *n_granules = total;
  if (total > pcm_cap_granules) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "pcm holds fewer blocks than needed");
  for (uint32_t k = 0; k < n_streams; k++) {
    streams[k].first_granule = g_at[k];
    streams[k].n_granules = 0;
    streams[k].flags = 0;
    end_status[k] = MP3G_OK;
  }
  if (total == 0) {
    // streams with no frame: their scan statuses
    for (uint32_t k = 0; k < n_streams; k++) {
      host::Source src;
      src.data = datas[k];
      src.len = (int64_t)lens[k];
      St st = src.skip_tags();
      if (st == St::kOk) {
        host::FrameScanner sc;
        host::ScannedFrame f;
        uint8_t one[1];
        host::RawMd md;
        md.base = one;
        st = sc.next(src, &f, &md);
      }
      end_status[k] = to_status(st == St::kOk ? St::kErr : st);
    }
    return MP3G_OK;
  }
  if (!pcm) return abi_fail(MP3G_ERR_INVALID_ARGUMENT, "null pcm");

  // ---- groups of consecutive streams with about equal granule counts ----
  // (~128 K granules, 300 MB of PCM each: the first group's scan and
  // transfers are the pipeline's fill, the PCM copy-out its steady state)
  uint32_t G = n_groups ? n_groups : (uint32_t)std::min<uint64_t>(32, std::max<uint64_t>(1, total / 131072));
  G = std::max(1u, std::min(G, n_streams));
  // (the first group half the size of the others: it is the pipeline's fill,
  // scanned and uploaded before any PCM can leave)
  std::vector<uint32_t> cut{0};
  for (uint32_t k = 0; k < n_streams && cut.size() < G; k++)
    if (g_at[k + 1] * (2 * (uint64_t)G - 1) >= total * (2 * cut.size() - 1) && k + 1 < n_streams) cut.push_back(k + 1);
  cut.push_back(n_streams);
  const size_t ng_groups = cut.size() - 1;
  uint64_t max_ng = 0, max_md = 0;
  for (size_t gi = 0; gi < ng_groups; gi++) {
    max_ng = std::max(max_ng, g_at[cut[gi + 1]] - g_at[cut[gi]]);
    max_md = std::max(max_md, m_at[cut[gi + 1]] - m_at[cut[gi]]);
  }
  // pinned arena per slot: [granules | jobs | main data + 16 | chunk table]
  // (a plan without state flags has at most one chunk per granule)
  const size_t b_gran = max_ng * sizeof(mp3g_granule), b_jobs = 2 * max_ng * sizeof(mp3g_hjob);
  const size_t b_md = (max_md + 16 + 15) & ~(size_t)15, b_chunks = max_ng * sizeof(ChunkDesc);
  trace.mark("layout");

  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return abi_fail(MP3G_ERR_NO_DEVICE, "decode_streams_into: device");
  int rc = ensure_device_ready(device);
  if (rc) {
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
  }
  // this device's cached buffer set, or a private one if it is in use
  std::unique_ptr<PipeBufs> own;
  PipeBufs* B = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    if ((size_t)device >= g_pipe.size()) {
      g_pipe.resize((size_t)device + 1);
      g_pipe_busy.resize((size_t)device + 1, false);
    }
    if (!g_pipe_busy[(size_t)device]) {
      if (!g_pipe[(size_t)device]) g_pipe[(size_t)device].reset(new (std::nothrow) PipeBufs);
      B = g_pipe[(size_t)device].get();
      if (B) g_pipe_busy[(size_t)device] = true;
    }
  }
  if (!B) {
    own.reset(new (std::nothrow) PipeBufs);
    B = own.get();
  }
  if (!B) {
    if (prev >= 0) (void)hipSetDevice(prev);
    return abi_fail(MP3G_ERR_OUT_OF_MEMORY, "decode_streams_into: buffers");
  }
  {
    // Three streams, so that a group's PCM copy-out (the long pole: 2,304 B
    // per granule over PCIe) runs back to back with the next group's
    // bitstream upload (the other direction) and kernels:
    //   up:   [wait kern(g-2)] H2D granules, jobs, main data, chunk table  -> h2d(g)
    //   comp: [wait h2d(g), d2h(g-2)] main-data kernel, granule kernel     -> kern(g)
    //   down: [wait kern(g)] D2H PCM into the caller's buffer              -> d2h(g)
    // Two buffer slots (g & 1) per input / PCM buffer; the coefficients are
    // used only on `comp`, in order, so one buffer serves every group.  The
    // host reuses a pinned arena slot after waiting for its upload (h2d(g-2)).
    rc = B->ensure_sync() ? MP3G_OK : abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: streams / events");
    for (int i = 0; i < 2 && rc == MP3G_OK; i++) {
      const bool ok = B->arena[i].reserve(b_gran + b_jobs + b_md + b_chunks) && B->d_gran[i].reserve(b_gran) &&
                      B->d_jobs[i].reserve(b_jobs) && B->d_md[i].reserve(b_md) && B->d_chunks[i].reserve(b_chunks) &&
                      B->d_pcm[i].reserve(max_ng * MP3G_PCM_BYTES_PER_GRANULE);
      if (!ok) rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: buffers");
    }
    if (rc == MP3G_OK && !B->d_coef.reserve(max_ng * MP3G_COEF_PER_GRANULE * sizeof(int16_t)))
      rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: buffers");
    trace.mark("buffers");
    hipStream_t up = B->up, comp = B->comp, down = B->down;
    // the caller's PCM buffer: pinned and 16-B aligned -> our copy kernel
    // writes it through its device address; anything else -> hipMemcpyAsync
    int16_t* pcm_dev = nullptr;
    {
      hipPointerAttribute_t pa;
      if ((reinterpret_cast<uintptr_t>(pcm) & 15u) == 0 && hipPointerGetAttributes(&pa, pcm) == hipSuccess &&
          pa.type == hipMemoryTypeHost && pa.devicePointer)
        pcm_dev = static_cast<int16_t*>(pa.devicePointer);
      (void)hipGetLastError();  // (pageable memory: an "invalid value" to clear)
    }
    std::vector<ChunkDesc> chunks;
    for (size_t gi = 0; gi < ng_groups && rc == MP3G_OK; gi++) {
      const int slot = (int)(gi & 1);
      if (gi >= 2 && hipEventSynchronize(B->h2d[slot]) != hipSuccess) {  // the arena slot's upload is done
        rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: device");
        break;
      }
      trace.mark("wait arena", gi);
      const uint32_t k0 = cut[gi], k1 = cut[gi + 1];
      const uint64_t G0 = g_at[k0], M0 = m_at[k0], ng = g_at[k1] - G0, nmd = m_at[k1] - M0;
      uint8_t* base = static_cast<uint8_t*>(B->arena[slot].p);
      auto* gran = reinterpret_cast<mp3g_granule*>(base);
      auto* jobs = reinterpret_cast<mp3g_hjob*>(base + b_gran);
      uint8_t* md = base + b_gran + b_jobs;
      auto* h_chunks = reinterpret_cast<ChunkDesc*>(base + b_gran + b_jobs + b_md);
      // host scan of the group straight into the pinned arena (jobs address
      // the group's main data; the previous groups' transfers and kernels run
      // meanwhile)
      std::vector<mp3g_stream> local(k1 - k0);
      std::atomic<bool> holes{false}, overflow{false};
      parallel_for(k0, k1, nt, [&](uint32_t k) {
        host::RawMd sink;
        sink.base = md;
        sink.n = m_at[k] - M0;
        sink.cap = sink.n + pm[k];
        St end;
        bool ovf;
        mp3g_granule* g = gran + (g_at[k] - G0);
        mp3g_hjob* j = jobs + 2 * (g_at[k] - G0);
        const uint64_t n = scan_into(datas[k], lens[k], g, j, pg[k], &sink, &end, &ovf);
        if (ovf) overflow = true;
        if (n < pg[k]) {  // ended early: the rest of its range decodes nothing
          holes = true;
          std::memset(static_cast<void*>(j + 2 * n), 0, (size_t)(2 * (pg[k] - n)) * sizeof(mp3g_hjob));
          // and its granule records hold no stale data of an earlier group
          // (the Huffman kernel visits them as jobs without scale factors)
          std::memset(static_cast<void*>(g + n), 0, (size_t)(pg[k] - n) * sizeof(mp3g_granule));
        }
        local[k - k0] = {g_at[k] - G0, (uint32_t)n, 0};
        streams[k].n_granules = (uint32_t)n;
        end_status[k] = to_status(end);
        std::memset(md + sink.n, 0, (size_t)(m_at[k + 1] - M0 - sink.n));
      });
      std::memset(md + nmd, 0, 16);
      trace.mark("scan", gi);
      if (overflow) {  // the pre-pass is an upper bound, so this cannot happen
        rc = abi_fail(MP3G_ERR_INVALID_ARGUMENT, "decode_streams_into: layout");
        break;
      }
      uint64_t pn = 0, ph = 0;
      rc = plan_chunks(device, local.data(), k1 - k0, 0, mode, &chunks, &pn, &ph);
      if (rc) break;
      if (chunks.size() > max_ng) {
        rc = abi_fail(MP3G_ERR_INVALID_ARGUMENT, "decode_streams_into: chunk table");
        break;
      }
      if (!chunks.empty()) std::memcpy(h_chunks, chunks.data(), chunks.size() * sizeof(ChunkDesc));
      // the fast kernel's zone scratch: the pieces of kZoneListPerChunk zones
      // per chunk of this group's plan (zone_list_capacity: the cost model
      // keeps chunks far fewer than granules), grown on demand -- after the kernels that use the old one
      // are done (the scratch is shared by every group on `comp`)
      if ((mode & 0xffu) == MP3G_MODE_FAST) {
        const uint64_t zone_cap = zone_list_capacity(chunks.data(), chunks.size());
        if (zone_cap > 0xffffffffu) {
          rc = abi_fail(MP3G_ERR_UNSUPPORTED, "decode_streams_into: group too large");
          break;
        }
        if (B->zone_cap < zone_cap) {
          const uint64_t grow = std::max<uint64_t>(zone_cap, (uint64_t)B->zone_cap * 2);
          const uint32_t cap = (uint32_t)std::min<uint64_t>(grow, 0xffffffffu);
          if (hipStreamSynchronize(B->comp) != hipSuccess || !B->d_zones.reserve(zone_scratch_bytes(cap)) ||
              zone_scratch_init(B->d_zones.p, cap) != hipSuccess) {
            rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: buffers");
            break;
          }
          B->zone_cap = cap;
        }
      }
      const uint32_t stage = mp3g_huffman_stage_flags(jobs, ng);
      // up
      hipError_t e = gi >= 2 ? hipStreamWaitEvent(up, B->kern[slot], 0) : hipSuccess;
      if (e == hipSuccess) e = hipMemcpyAsync(B->d_gran[slot].p, gran, ng * sizeof(mp3g_granule), hipMemcpyHostToDevice, up);
      if (e == hipSuccess)
        e = hipMemcpyAsync(B->d_jobs[slot].p, jobs, 2 * ng * sizeof(mp3g_hjob), hipMemcpyHostToDevice, up);
      if (e == hipSuccess) e = hipMemcpyAsync(B->d_md[slot].p, md, nmd + 16, hipMemcpyHostToDevice, up);
      if (e == hipSuccess && !chunks.empty())
        e = hipMemcpyAsync(B->d_chunks[slot].p, h_chunks, chunks.size() * sizeof(ChunkDesc), hipMemcpyHostToDevice, up);
      if (e == hipSuccess) e = hipEventRecord(B->h2d[slot], up);
      // comp
      if (e == hipSuccess) e = hipStreamWaitEvent(comp, B->h2d[slot], 0);
      if (e == hipSuccess && gi >= 2) e = hipStreamWaitEvent(comp, B->d2h[slot], 0);
      if (e == hipSuccess && holes)
        e = hipMemsetAsync(B->d_pcm[slot].p, 0, ng * MP3G_PCM_BYTES_PER_GRANULE, comp);
      if (e != hipSuccess) {
        rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: H2D");
        break;
      }
      rc = mp3g_huffman_execute_ex(device, static_cast<const mp3g_hjob*>(B->d_jobs[slot].p), ng,
                                   static_cast<const uint8_t*>(B->d_md[slot].p),
                                   static_cast<mp3g_granule*>(B->d_gran[slot].p), static_cast<int16_t*>(B->d_coef.p),
                                   (mode_reads_to_count1(mode) ? MP3G_HUFF_ROWS_COUNT1 : 0u) | stage, comp);
      if (rc == MP3G_OK && !chunks.empty()) {
        const ZoneScratch zs{static_cast<uint32_t*>(B->d_zones.p), B->zone_cap};
        rc = plan_launch(mode & ~(uint32_t)MP3G_FLAG_HOT_STATS, static_cast<const ChunkDesc*>(B->d_chunks[slot].p),
                         (uint32_t)chunks.size(), static_cast<const mp3g_granule*>(B->d_gran[slot].p),
                         static_cast<const int16_t*>(B->d_coef.p), nullptr, nullptr,
                         static_cast<int16_t*>(B->d_pcm[slot].p), &zs, comp);
      }
      if (rc) break;
      e = hipEventRecord(B->kern[slot], comp);
      // down
      if (e == hipSuccess) e = hipStreamWaitEvent(down, B->kern[slot], 0);
      if (e == hipSuccess && pcm_dev)
        e = launch_copy_out(B->d_pcm[slot].p, pcm_dev + G0 * (MP3G_PCM_BYTES_PER_GRANULE / sizeof(int16_t)),
                            ng * MP3G_PCM_BYTES_PER_GRANULE, 8 * B->down_cus, down);
      else if (e == hipSuccess)
        e = hipMemcpyAsync(pcm + G0 * (MP3G_PCM_BYTES_PER_GRANULE / sizeof(int16_t)), B->d_pcm[slot].p,
                           ng * MP3G_PCM_BYTES_PER_GRANULE, hipMemcpyDeviceToHost, down);
      if (e == hipSuccess) e = hipEventRecord(B->d2h[slot], down);
      if (e != hipSuccess) rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: D2H");
      trace.mark("enqueue", gi);
    }
    // (on an error too: nothing may still write into the caller's buffer or
    // read the arena after return)
    for (hipStream_t q : {up, comp, down})
      if (q && hipStreamSynchronize(q) != hipSuccess && rc == MP3G_OK)
        rc = abi_fail(MP3G_ERR_DEVICE, "decode_streams_into: device");
    trace.mark("drain");
  }
  if (!own) {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    g_pipe_busy[(size_t)device] = false;
  }
  own.reset();
  if (prev >= 0) (void)hipSetDevice(prev);
  return rc;
}

}  // extern "C"
