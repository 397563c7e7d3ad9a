// mp3g_abi.cpp -- C-ABI of libmp3g.so (declared in include/mp3g.h).
//
// Host side of the drop-in boundary for Frame.Decode (reference
// internal/frame/frame.go:121).  No exception crosses the ABI; every entry
// returns an mp3g_status.  The caller's current HIP device is restored on
// return, so a host framework sharing the process (PyTorch) is unaffected.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/mp3g.h"
#include "abi_util.h"
#include "dsp_tables.h"
#include "kernels.h"

using namespace mp3g;

namespace {

thread_local std::string t_last_error;

int fail(int status, const char* what, hipError_t e = hipSuccess) {
  t_last_error = what;
  if (e != hipSuccess) {
    t_last_error += ": ";
    t_last_error += hipGetErrorString(e);
  }
  return status;
}

#define HIP_TRY(expr)                                                   \
  do {                                                                  \
    hipError_t e_ = (expr);                                             \
    if (e_ != hipSuccess) return fail(MP3G_ERR_DEVICE, #expr, e_);      \
  } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

constexpr int kMaxDevices = 64;
std::once_flag g_host_tables_once;
DspTables* g_host_tables = nullptr;
std::mutex g_dev_mu;
bool g_dev_ready[kMaxDevices] = {};

const DspTables& host_tables() {
  std::call_once(g_host_tables_once, [] {
    g_host_tables = new DspTables;
    build_tables(g_host_tables);
  });
  return *g_host_tables;
}

// Uploads the constant tables to `dev` once.  Caller holds a DeviceGuard(dev).
int ensure_device(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return fail(MP3G_ERR_INVALID_ARGUMENT, "device index");
  std::lock_guard<std::mutex> lk(g_dev_mu);
  if (g_dev_ready[dev]) return MP3G_OK;
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(MP3G_ERR_NO_DEVICE, "device is not gfx950");
  HIP_TRY(upload_tables(host_tables()));
  HIP_TRY(hipDeviceSynchronize());
  g_dev_ready[dev] = true;
  return MP3G_OK;
}

// Automatic chunk length (granules per chunk).  A chunk costs ~k + 2 (halo)
// + 2 (prologue) granule-times, and the launch runs ~chunks / resident rounds
// (resident = CUs x chunks per CU) plus about half a round of tail (chunks
// finish at different times).  Minimising that picks k = 7 for c2 (10 %
// faster than k = 8) and ~64 granules for c3 (4 % faster than k = 256, 20 %
// faster than one round of 683-granule chunks; sweeps measured on MI355X,
// tools/gpu_chunks.sh).
// The granule kernel a plan's mode runs: fast v3, or exact v4 unless a
// cross-check kernel is asked for (MP3G_FLAG_KERNEL_V2).
int plan_variant(uint32_t mode) {
  if ((mode & 0xffu) == MP3G_MODE_FAST) return kVariantFast;
  if (mode & MP3G_FLAG_KERNEL_V2) return kVariantV2;
  return kVariantExact4;
}

}  // namespace

bool mp3g::mode_reads_to_count1(unsigned mode) {
  const int v = plan_variant(mode);
  return v == kVariantFast || v == kVariantExact4;
}

namespace {

uint32_t auto_chunk(const mp3g_stream* streams, uint32_t n_streams, int device, uint32_t mode) {
  uint64_t maxn = 0;
  for (uint32_t s = 0; s < n_streams; s++) maxn = std::max<uint64_t>(maxn, streams[s].n_granules);
  if (maxn == 0) return 1;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  const uint64_t resident =
      (uint64_t)cus * (uint64_t)chunks_per_cu(plan_variant(mode));
  uint64_t best_k = 1;
  double best = 0.0;
  for (uint64_t k = 1; k <= maxn;) {
    uint64_t chunks = 0;
    for (uint32_t s = 0; s < n_streams; s++) chunks += (streams[s].n_granules + k - 1) / k;
    const double rounds = (double)chunks / (double)resident + 0.5;
    const double cost = rounds * (double)(k + 4);
    if (best == 0.0 || cost <= best) {
      best = cost;
      best_k = k;
    }
    k = k < 64 ? k + 1 : std::max<uint64_t>(k + 1, k * 17 / 16);
  }
  return (uint32_t)std::min<uint64_t>(best_k, 1u << 20);
}

// Chunks per stream for a total of about `total` chunks: proportional to the
// stream lengths, at least 1 and at most n_granules per non-empty stream.
std::vector<uint64_t> spread_chunks(const mp3g_stream* streams, uint32_t n_streams, uint64_t total) {
  uint64_t n = 0;
  for (uint32_t s = 0; s < n_streams; s++) n += streams[s].n_granules;
  std::vector<uint64_t> c(n_streams, 0);
  for (uint32_t s = 0; s < n_streams; s++) {
    const uint64_t ns = streams[s].n_granules;
    if (!ns) continue;
    const uint64_t want = (uint64_t)((double)ns * (double)total / (double)n + 0.5);
    c[s] = std::min<uint64_t>(ns, std::max<uint64_t>(1, want));
  }
  return c;
}

// Automatic chunk counts.  The cost model's length k first; then, when the
// plan fills at least half a round of resident chunks, the total is rounded up
// to whole rounds (every wave slot of every round gets a chunk: on c2 the
// model's 3,334 chunks put 4 workgroups on 66 CUs and 3 on the others, and
// the 4-workgroup CUs set the launch time) and the streams are cut into
// chunks of equal length.
//
// Whole rounds (round 6): the number of rounds R is then chosen on the plans
// it actually yields -- R x resident chunks spread over the streams, the
// longest chunk k_R -- at cost (R + tail) (k_R + 4): 4 granule-steps of
// per-chunk overhead (the two-granule halo and the prologue; fitted to the
// c3 chunk sweep, tools/chunk_sweep.sh: 7.90 / 7.67 / 7.60 / 7.79 M cycles at
// 8 / 4 / 2 / 1 rounds) and a tail of MP3G_CHUNK_TAIL rounds, far below the
// 0.5 round of the fractional model (equal chunks in whole rounds end
// together).  c3: 8 -> 4 rounds of 128 granules (-1.4 % in time at the clock
// the chip then holds); c2 stays one round.
#ifndef MP3G_CHUNK_TAIL
#define MP3G_CHUNK_TAIL 0.15
#endif
std::vector<uint64_t> auto_chunks(const mp3g_stream* streams, uint32_t n_streams, int device, uint32_t mode) {
  const uint64_t k = auto_chunk(streams, n_streams, device, mode);
  uint64_t c0 = 0;
  for (uint32_t s = 0; s < n_streams; s++) c0 += (streams[s].n_granules + k - 1) / k;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  const uint64_t resident =
      (uint64_t)cus * (uint64_t)chunks_per_cu(plan_variant(mode));
  if (2 * c0 < resident) {
    std::vector<uint64_t> c(n_streams);
    for (uint32_t s = 0; s < n_streams; s++) c[s] = (streams[s].n_granules + k - 1) / k;
    return c;
  }
  const uint64_t r0 = (c0 + resident - 1) / resident;
  if (MP3G_CHUNK_TAIL <= 0.0) return spread_chunks(streams, n_streams, r0 * resident);
  // candidates: the fractional model's R and every R below it down to 1
  uint64_t best_r = r0;
  double best = 0.0;
  for (uint64_t r = r0; r >= 1; r--) {
    const std::vector<uint64_t> c = spread_chunks(streams, n_streams, r * resident);
    uint64_t kr = 0;
    for (uint32_t s = 0; s < n_streams; s++)
      if (c[s]) kr = std::max<uint64_t>(kr, (streams[s].n_granules + c[s] - 1) / c[s]);
    const double cost = ((double)r + MP3G_CHUNK_TAIL) * (double)(kr + 4);
    if (best == 0.0 || cost < best) {
      best = cost;
      best_r = r;
    }
  }
  return spread_chunks(streams, n_streams, best_r * resident);
}

}  // namespace

int mp3g::abi_fail(int status, const char* what) { return fail(status, what); }

int mp3g::ensure_device_ready(int device) {
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  return ensure_device(device);
}

// The chunk table of a plan (chunks per stream from granules_per_chunk: 0 =
// the cost model, bit 31 = a total chunk count spread over the streams, else
// the length), after the checks of mp3g_plan_create; the device's tables are
// uploaded on first use.
int mp3g::plan_chunks(int device, const mp3g_stream* streams, uint32_t n_streams, uint32_t granules_per_chunk,
                      uint32_t mode, std::vector<ChunkDesc>* chunks, uint64_t* n_granules, uint64_t* n_halo) {
  if (n_streams && !streams) return fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  const uint32_t base_mode = mode & 0xffu;
  if (base_mode != MP3G_MODE_EXACT && base_mode != MP3G_MODE_FAST)
    return fail(MP3G_ERR_UNSUPPORTED, "mode not available");
  if (mode & MP3G_FLAG_KERNEL_V1) return fail(MP3G_ERR_UNSUPPORTED, "the v1 exact kernel was retired (ABI 3)");
  for (uint32_t s = 0; s < n_streams; s++) {
    // the one-wave kernels (fast v3, exact v4) index granules with 32-bit
    // wave-uniform scalars
    const int v = plan_variant(mode);
    if ((v == kVariantFast || v == kVariantExact4) && streams[s].first_granule + streams[s].n_granules >= (1ull << 32))
      return fail(MP3G_ERR_UNSUPPORTED, "granule index >= 2^32 (use MP3G_FLAG_KERNEL_V2 in exact mode)");
  }
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  int st = ensure_device(device);
  if (st) return st;
  // chunks per stream (lengths within a stream differ by at most one)
  std::vector<uint64_t> nc;
  if (granules_per_chunk == 0) {
    nc = auto_chunks(streams, n_streams, device, mode);
  } else if (granules_per_chunk & 0x80000000u) {
    nc = spread_chunks(streams, n_streams, std::max<uint32_t>(1, granules_per_chunk & 0x7fffffffu));
  } else {
    nc.resize(n_streams);
    for (uint32_t s = 0; s < n_streams; s++)
      nc[s] = (streams[s].n_granules + granules_per_chunk - 1) / granules_per_chunk;
  }
  // ChunkDesc::n_out is 32-bit: a stream cut into too few chunks is refused
  for (uint32_t s = 0; s < n_streams; s++)
    if (streams[s].n_granules && (nc[s] == 0 || (streams[s].n_granules + nc[s] - 1) / nc[s] >= (1ull << 32)))
      return fail(MP3G_ERR_UNSUPPORTED, "chunk of >= 2^32 granules");
  chunks->clear();
  *n_granules = *n_halo = 0;
  for (uint32_t s = 0; s < n_streams; s++) {
    const mp3g_stream& S = streams[s];
    const uint64_t cs = nc[s];
    for (uint64_t i = 0, off = 0; i < cs && off < S.n_granules; i++) {
      // chunk i of cs: granules [i n / cs, (i + 1) n / cs)
      const uint64_t next = (i + 1) * S.n_granules / cs;
      ChunkDesc c{};
      c.out_first = S.first_granule + off;
      c.stream_first = S.first_granule;
      c.n_out = (uint32_t)(next - off);
      c.stream = s;
      c.flags = (S.flags & MP3G_STREAM_STATE_IN) ? kChunkStateIn : 0u;
      if ((S.flags & MP3G_STREAM_STATE_OUT) && off + c.n_out == S.n_granules) c.flags |= kChunkStateOut;
      chunks->push_back(c);
      *n_granules += c.n_out;
      *n_halo += std::min<uint64_t>(off, 2);
      off = next;
    }
    if (S.n_granules == 0 && (S.flags & MP3G_STREAM_STATE_OUT)) {
      // empty stream exporting state: state_out = state_in (or zero)
      ChunkDesc c{};
      c.out_first = S.first_granule;
      c.stream_first = S.first_granule;
      c.n_out = 0;
      c.stream = s;
      c.flags = kChunkStateOut | ((S.flags & MP3G_STREAM_STATE_IN) ? kChunkStateIn : 0u);
      chunks->push_back(c);
    }
  }
  return MP3G_OK;
}

// Launch of a chunk table already on the device (d_hot: the fast kernel's
// hot-granule counters, or null).
int mp3g::plan_launch(uint32_t mode, const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                      const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm,
                      const ZoneScratch* zones, hipStream_t stream) {
  HIP_TRY(launch_granule(plan_variant(mode), d_chunks, n_chunks, d_gran, d_coef, d_state_in, d_state_out, d_pcm,
                         zones, (mode & MP3G_FLAG_HOT_STATS) != 0, stream));
  return MP3G_OK;
}

struct mp3g_plan {
  int device = 0;
  uint32_t mode = 0;
  uint32_t n_streams = 0;
  std::vector<ChunkDesc> chunks;
  // one device allocation: the chunk table, then (fast mode) the zone scratch
  // of the deferred hot zones with the hot-granule counters in its header
  ChunkDesc* d_chunks = nullptr;
  void* d_zones = nullptr;
  uint32_t zone_cap = 0;
  uint64_t n_granules = 0;
  uint64_t n_halo = 0;
};

extern "C" {

int mp3g_abi_version(void) { return MP3G_ABI_VERSION; }

const char* mp3g_status_string(int s) {
  switch (s) {
    case MP3G_OK: return "ok";
    case MP3G_ERR_INVALID_ARGUMENT: return "invalid argument";
    case MP3G_ERR_INVALID_GRANULE: return "invalid granule descriptor";
    case MP3G_ERR_NO_DEVICE: return "no gfx950 device";
    case MP3G_ERR_DEVICE: return "HIP runtime error";
    case MP3G_ERR_OUT_OF_MEMORY: return "out of memory";
    case MP3G_ERR_PARSE: return "bitstream parse error";
    case MP3G_EOF: return "end of stream";
    case MP3G_ERR_UNSUPPORTED: return "unsupported stream";
    case MP3G_ERR_NO_XING_HEADER: return "lameinfo: no Xing/Info header found";
    case MP3G_ERR_UNEXPECTED_EOF: return "unexpected EOF";
    case MP3G_ERR_READ: return "reader error";
  }
  return "unknown status";
}

const char* mp3g_last_error(void) { return t_last_error.c_str(); }

int mp3g_device_count(int* out_count) {
  if (!out_count) return fail(MP3G_ERR_INVALID_ARGUMENT, "null out_count");
  *out_count = 0;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return MP3G_OK;
  int k = 0;
  for (int d = 0; d < n; d++) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0) k++;
  }
  *out_count = k;
  return MP3G_OK;
}

// Range checks of everything the DSP reads (what the reference bitstream
// parse can produce); MPEG-2 mixed blocks are rejected because the reference
// panics on them (maindata.go:139-178).
int mp3g_validate(const mp3g_granule* g, const int16_t* coef, uint64_t n, uint64_t* bad) {
  if (bad) *bad = 0;
  if (n && (!g || !coef)) return fail(MP3G_ERR_INVALID_ARGUMENT, "null granules/coeffs");
  for (uint64_t k = 0; k < n; k++) {
    const uint32_t h = g[k].header;
    bool ok = (h & 0xffe00000u) == 0xffe00000u;
    const uint32_t id = (h >> 19) & 3u;
    ok = ok && id != 1 && id != 0;             // reserved / MPEG 2.5 (frame.go:79-81)
    ok = ok && ((h >> 17) & 3u) == 1u;         // layer III
    ok = ok && ((h >> 12) & 15u) != 15u && ((h >> 12) & 15u) != 0u;
    ok = ok && ((h >> 10) & 3u) != 3u;
    const int nch = ((h >> 6) & 3u) == 3u ? 1 : 2;
    const bool lsf = id != 3;
    for (int ch = 0; ok && ch < nch; ch++) {
      const mp3g_channel& c = g[k].ch[ch];
      ok = c.count1 <= 576 && c.scalefac_scale <= 1 && c.preflag <= 1 && c.win_switch_flag <= 1 &&
           c.block_type <= 3 && c.mixed_block_flag <= 1;
      if (ok && !c.win_switch_flag) ok = c.block_type == 0 && c.mixed_block_flag == 0;
      if (ok && lsf && c.block_type == 2 && c.mixed_block_flag) ok = false;
      for (int w = 0; ok && w < 3; w++) ok = c.subblock_gain[w] <= 7;
      for (int s = 0; ok && s < 22; s++) ok = c.scalefac_l[s] <= 15;
      for (int s = 0; ok && s < 13; s++)
        for (int w = 0; ok && w < 3; w++) ok = c.scalefac_s[s][w] <= 15;
      const int16_t* x = coef + k * MP3G_COEF_PER_GRANULE + ch * MP3G_LINES;
      for (int i = 0; ok && i < MP3G_LINES; i++) {
        ok = x[i] <= 8206 && x[i] >= -8206;
        if (ok && i >= c.count1) ok = x[i] == 0;  // zero region (maindata/huffman.go:130-134)
      }
    }
    if (!ok) {
      if (bad) *bad = k;
      return fail(MP3G_ERR_INVALID_GRANULE, "granule descriptor out of range");
    }
  }
  return MP3G_OK;
}

int mp3g_plan_create(int device, const mp3g_stream* streams, uint32_t n_streams,
                     uint32_t granules_per_chunk, uint32_t mode, mp3g_plan** out_plan) {
  if (!out_plan) return fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  *out_plan = nullptr;
  mp3g_plan* p = new (std::nothrow) mp3g_plan;
  if (!p) return fail(MP3G_ERR_OUT_OF_MEMORY, "plan");
  int st = mp3g::plan_chunks(device, streams, n_streams, granules_per_chunk, mode, &p->chunks, &p->n_granules,
                             &p->n_halo);
  if (st) {
    delete p;
    return st;
  }
  p->device = device;
  p->mode = mode;
  p->n_streams = n_streams;
  DeviceGuard guard(device);
  // the chunk table, then the zone scratch (as many zones as the fast kernel
  // can record per chunk: the list never overflows)
  const size_t tb = (p->chunks.size() * sizeof(ChunkDesc) + 255) & ~(size_t)255;
  const bool fast = plan_variant(mode) == kVariantFast;
  const uint64_t zone_cap = fast ? zone_list_capacity(p->chunks.data(), p->chunks.size()) : 0u;
  if (zone_cap > 0xffffffffu) {
    delete p;
    return fail(MP3G_ERR_UNSUPPORTED, "fast-mode plan of more than 2^29 chunks");
  }
  p->zone_cap = (uint32_t)zone_cap;
  const size_t zb = fast ? zone_scratch_bytes(p->zone_cap) : 0;
  hipError_t e = hipMalloc(&p->d_chunks, std::max<size_t>(tb + zb, 256));
  if (e != hipSuccess) {
    delete p;
    return fail(MP3G_ERR_OUT_OF_MEMORY, "hipMalloc(chunks)", e);
  }
  if (fast) p->d_zones = reinterpret_cast<uint8_t*>(p->d_chunks) + tb;
  if (!p->chunks.empty()) e = hipMemcpy(p->d_chunks, p->chunks.data(), p->chunks.size() * sizeof(ChunkDesc),
                                        hipMemcpyHostToDevice);
  if (e == hipSuccess && fast) e = zone_scratch_init(p->d_zones, p->zone_cap);
  if (e != hipSuccess) {
    (void)hipFree(p->d_chunks);
    delete p;
    return fail(MP3G_ERR_DEVICE, "hipMemcpy(chunks)", e);
  }
  *out_plan = p;
  return MP3G_OK;
}

int mp3g_plan_destroy(mp3g_plan* p) {
  if (!p) return MP3G_OK;
  if (p->d_chunks) {
    DeviceGuard guard(p->device);
    (void)hipFree(p->d_chunks);
  }
  delete p;
  return MP3G_OK;
}

int mp3g_plan_info(const mp3g_plan* p, uint64_t* n_chunks, uint64_t* n_granules, uint64_t* n_halo) {
  if (!p) return fail(MP3G_ERR_INVALID_ARGUMENT, "null plan");
  if (n_chunks) *n_chunks = p->chunks.size();
  if (n_granules) *n_granules = p->n_granules;
  if (n_halo) *n_halo = p->n_halo;
  return MP3G_OK;
}

int mp3g_plan_execute(mp3g_plan* p, const mp3g_granule* d_gran, const int16_t* d_coef,
                      const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm,
                      void* hip_stream) {
  if (!p) return fail(MP3G_ERR_INVALID_ARGUMENT, "null plan");
  if (p->chunks.empty()) return MP3G_OK;
  if (!d_gran || !d_coef || !d_pcm) return fail(MP3G_ERR_INVALID_ARGUMENT, "null device buffer");
  DeviceGuard guard(p->device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  for (const ChunkDesc& c : p->chunks) {
    if ((c.flags & kChunkStateOut) && !d_state_out) return fail(MP3G_ERR_INVALID_ARGUMENT, "state_out needed");
  }
  const ZoneScratch zs{static_cast<uint32_t*>(p->d_zones), p->zone_cap};
  return plan_launch(p->mode, p->d_chunks, (uint32_t)p->chunks.size(), d_gran, d_coef, d_state_in, d_state_out,
                     d_pcm, p->d_zones ? &zs : nullptr, static_cast<hipStream_t>(hip_stream));
}

// The fast kernel's hot-granule counters of this plan (MP3G_FLAG_HOT_STATS),
// summed over its launches since creation or the last reset (kernels.h
// kHotCounters).  Synchronous.
int mp3g_plan_hot_stats(mp3g_plan* p, uint64_t* out4, int reset) {
  if (!p || !out4) return fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  DeviceGuard guard(p->device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  uint32_t h[kHotCounters] = {};
  for (int i = 0; i < kHotCounters; i++) out4[i] = 0;
  if (!p->d_zones) return MP3G_OK;  // an exact-mode plan: no fallback to count
  uint32_t* hot = static_cast<uint32_t*>(p->d_zones) + 4;  // kernels.h ZoneScratch header
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h, hot, sizeof(h), hipMemcpyDeviceToHost));
  for (int i = 0; i < kHotCounters; i++) out4[i] = h[i];
  if (reset) HIP_TRY(hipMemset(hot, 0, sizeof(h)));
  return MP3G_OK;
}

int mp3g_plan_synth_execute(mp3g_plan* p, const mp3g_granule* d_gran, const float* d_lines,
                            const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm, void* hip_stream) {
  if (!p) return fail(MP3G_ERR_INVALID_ARGUMENT, "null plan");
  if ((p->mode & 0xffu) != MP3G_MODE_FAST) return fail(MP3G_ERR_INVALID_ARGUMENT, "not a fast-mode plan");
  if (p->chunks.empty()) return MP3G_OK;
  if (!d_gran || !d_lines || !d_pcm) return fail(MP3G_ERR_INVALID_ARGUMENT, "null device buffer");
  DeviceGuard guard(p->device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  for (const ChunkDesc& c : p->chunks) {
    if ((c.flags & kChunkStateOut) && !d_state_out) return fail(MP3G_ERR_INVALID_ARGUMENT, "state_out needed");
  }
  HIP_TRY(launch_synth(p->d_chunks, (uint32_t)p->chunks.size(), d_gran, d_lines, d_state_in, d_state_out, d_pcm,
                       static_cast<hipStream_t>(hip_stream)));
  return MP3G_OK;
}

int mp3g_huffman_execute(int device, const mp3g_hjob* d_jobs, uint64_t n_granules, const uint8_t* d_md,
                         mp3g_granule* d_gran, int16_t* d_coef, void* hip_stream) {
  return mp3g_huffman_execute_ex(device, d_jobs, n_granules, d_md, d_gran, d_coef, 0u, hip_stream);
}

int mp3g_huffman_execute_ex(int device, const mp3g_hjob* d_jobs, uint64_t n_granules, const uint8_t* d_md,
                            mp3g_granule* d_gran, int16_t* d_coef, uint32_t flags, void* hip_stream) {
  if (flags & ~(uint32_t)(MP3G_HUFF_ROWS_COUNT1 | MP3G_HUFF_STAGE_WIDE | MP3G_HUFF_STAGE_MID) ||
      ((flags & MP3G_HUFF_STAGE_WIDE) && (flags & MP3G_HUFF_STAGE_MID)))
    return fail(MP3G_ERR_INVALID_ARGUMENT, "huffman flags");
  if (n_granules == 0) return MP3G_OK;
  if (!d_jobs || !d_md || !d_gran || !d_coef) return fail(MP3G_ERR_INVALID_ARGUMENT, "null device buffer");
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  int st = ensure_device(device);
  if (st) return st;
  HIP_TRY(launch_huffman(d_jobs, 2 * n_granules, d_md, d_gran, d_coef, !(flags & MP3G_HUFF_ROWS_COUNT1),
                         (flags & MP3G_HUFF_STAGE_WIDE) ? 2 : (flags & MP3G_HUFF_STAGE_MID) ? 1 : 0,
                         static_cast<hipStream_t>(hip_stream)));
  return MP3G_OK;
}

// The kernel's blocks are kHuffJobsPerBlock consecutive jobs; a block stages
// the main data from its lowest job base to its highest bit_end (jobs that
// read nothing aside) when that span fits the stage (huffman_dev.hip).  The
// stage picked is the one of least modelled time, a block costing
// (1.86 + 0.0186 * span KB) x the stage's occupancy factor (1 / 1.1 / 1.45 for
// 16 / 12 / 8 waves per CU) x 1.9 when it does not fit and reads global
// memory -- a fit of tools/huff_time.py's c3-shape times at 128, 192 and 320
// kbps, the unstaged factor raised from the 1.7 of uniform batches because in
// a mixed batch the unstaged blocks also set the launch's tail (half 128, half
// 320 kbps: default 4.47 ms, mid 4.99, wide 4.33).
uint32_t mp3g_huffman_stage_flags(const mp3g_hjob* jobs, uint64_t n_granules) {
  if (!jobs) return 0u;
  const uint64_t n = 2 * n_granules;
  const uint64_t words[3] = {(uint64_t)kHuffStageWords, (uint64_t)kHuffStageWordsMid, (uint64_t)kHuffStageWordsWide};
  const double occupancy[3] = {1.0, 1.1, 1.45}, unstaged = 1.9;
  double cost[3] = {0.0, 0.0, 0.0};
  for (uint64_t b0 = 0; b0 < n; b0 += kHuffJobsPerBlock) {
    uint64_t lo = ~0ull, hi = 0;
    for (uint64_t j = b0; j < n && j < b0 + kHuffJobsPerBlock; j++) {
      if (jobs[j].sf_kind == MP3G_SF_NONE) continue;
      lo = std::min<uint64_t>(lo, (jobs[j].part2_start - jobs[j].scf0_delta) & ~63ull);
      hi = std::max<uint64_t>(hi, jobs[j].bit_end);
    }
    const uint64_t span = hi > lo && lo != ~0ull ? (hi - lo + 63) >> 6 : 0;  // 64-bit words
    const double work = 1.86 + 0.0186 * (double)span * 8.0 / 1024.0;
    for (int k = 0; k < 3; k++) cost[k] += work * occupancy[k] * (span <= words[k] ? 1.0 : unstaged);
  }
  int best = 0;
  for (int k = 1; k < 3; k++)
    if (cost[k] < cost[best]) best = k;
  return best == 0 ? 0u : best == 1 ? MP3G_HUFF_STAGE_MID : MP3G_HUFF_STAGE_WIDE;
}

// stamped launch of a fast plan: kFastStampSlots per chunk into h
static int run_stamped(mp3g_plan* p, const mp3g_granule* d_gran, const int16_t* d_coef, int16_t* d_pcm,
                       std::vector<unsigned long long>* h, void* hip_stream) {
  if ((p->mode & 0xffu) != MP3G_MODE_FAST) return fail(MP3G_ERR_INVALID_ARGUMENT, "not a fast-mode plan");
  for (const ChunkDesc& c : p->chunks)
    if (c.flags & (kChunkStateIn | kChunkStateOut)) return fail(MP3G_ERR_INVALID_ARGUMENT, "stateful plan");
  h->assign(p->chunks.size() * kFastStampSlots, 0ull);
  if (p->chunks.empty()) return MP3G_OK;
  DeviceGuard guard(p->device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  unsigned long long* d_st = nullptr;
  hipError_t e = hipMalloc(&d_st, h->size() * sizeof(unsigned long long));
  if (e != hipSuccess) return fail(MP3G_ERR_OUT_OF_MEMORY, "hipMalloc(stamps)", e);
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  e = launch_fast_stamped(p->d_chunks, (uint32_t)p->chunks.size(), d_gran, d_coef, nullptr, nullptr, d_pcm, d_st, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(h->data(), d_st, h->size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d_st);
  if (e != hipSuccess) return fail(MP3G_ERR_DEVICE, "stamped launch", e);
  return MP3G_OK;
}

int mp3g_plan_debug_phases(mp3g_plan* p, const mp3g_granule* d_gran, const int16_t* d_coef, int16_t* d_pcm,
                           uint64_t* out_cycles, void* hip_stream) {
  if (!p || !out_cycles) return fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  for (int i = 0; i < kFastPhases; i++) out_cycles[i] = 0;
  std::vector<unsigned long long> h;
  const int rc = run_stamped(p, d_gran, d_coef, d_pcm, &h, hip_stream);
  if (rc) return rc;
  for (size_t i = 0; i < h.size(); i++)
    if (i % kFastStampSlots < (size_t)kFastPhases) out_cycles[i % kFastStampSlots] += h[i];
  return MP3G_OK;
}

int mp3g_plan_debug_timeline(mp3g_plan* p, const mp3g_granule* d_gran, const int16_t* d_coef, int16_t* d_pcm,
                             uint64_t* out_ticks, void* hip_stream) {
  if (!p || !out_ticks) return fail(MP3G_ERR_INVALID_ARGUMENT, "null argument");
  std::vector<unsigned long long> h;
  const int rc = run_stamped(p, d_gran, d_coef, d_pcm, &h, hip_stream);
  if (rc) return rc;
  for (size_t c = 0; c < p->chunks.size(); c++)
    for (int k = 0; k < 4; k++) out_ticks[4 * c + k] = h[c * kFastStampSlots + kFastPhases + k];
  return MP3G_OK;
}

int mp3g_debug_clock_probe(int device, const uint32_t* d_flag, uint64_t* d_out, uint32_t n_waves,
                           uint32_t max_ms, void* hip_stream) {
  if (!d_flag || !d_out || n_waves == 0 || n_waves > 1024 || max_ms == 0 || max_ms > 10000)
    return fail(MP3G_ERR_INVALID_ARGUMENT, "clock probe arguments");
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return fail(MP3G_ERR_NO_DEVICE, "hipSetDevice", guard.err);
  const hipError_t e = launch_clock_probe(d_flag, reinterpret_cast<unsigned long long*>(d_out), n_waves,
                                          100000ull * max_ms, static_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(MP3G_ERR_DEVICE, "clock probe launch", e);
  return MP3G_OK;
}

int mp3g_decode_host(int device, const mp3g_granule* granules, const int16_t* coeffs,
                     uint64_t n_granules, const mp3g_stream* streams, uint32_t n_streams,
                     const mp3g_state* state_in, mp3g_state* state_out, int16_t* pcm,
                     uint32_t mode) {
  if (n_granules && (!granules || !coeffs || !pcm)) return fail(MP3G_ERR_INVALID_ARGUMENT, "null buffer");
  bool need_in = false, need_out = false;
  for (uint32_t s = 0; s < n_streams; s++) {
    if (streams[s].first_granule + streams[s].n_granules > n_granules)
      return fail(MP3G_ERR_INVALID_ARGUMENT, "stream exceeds granule array");
    need_in |= (streams[s].flags & MP3G_STREAM_STATE_IN) != 0;
    need_out |= (streams[s].flags & MP3G_STREAM_STATE_OUT) != 0;
  }
  if ((need_in && !state_in) || (need_out && !state_out))
    return fail(MP3G_ERR_INVALID_ARGUMENT, "state buffer missing");
  if (mode & MP3G_FLAG_CHECKED) {
    int st = mp3g_validate(granules, coeffs, n_granules, nullptr);
    if (st) return st;
  }
  mp3g_plan* plan = nullptr;
  int st = mp3g_plan_create(device, streams, n_streams, 0, mode & ~MP3G_FLAG_CHECKED, &plan);
  if (st) return st;
  DeviceGuard guard(device);
  void *dg = nullptr, *dc = nullptr, *dsi = nullptr, *dso = nullptr, *dp = nullptr;
  hipStream_t stream = nullptr;
  auto cleanup = [&]() {
    if (stream) (void)hipStreamDestroy(stream);
    for (void* q : {dg, dc, dsi, dso, dp})
      if (q) (void)hipFree(q);
    mp3g_plan_destroy(plan);
  };
  const size_t gb = n_granules * sizeof(mp3g_granule), cb = n_granules * MP3G_COEF_PER_GRANULE * 2,
               pb = n_granules * MP3G_PCM_BYTES_PER_GRANULE, sb = n_streams * sizeof(mp3g_state);
  hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
  if (e == hipSuccess && gb) e = hipMalloc(&dg, gb);
  if (e == hipSuccess && cb) e = hipMalloc(&dc, cb);
  if (e == hipSuccess && pb) e = hipMalloc(&dp, pb);
  if (e == hipSuccess && need_in) e = hipMalloc(&dsi, sb);
  if (e == hipSuccess && need_out) e = hipMalloc(&dso, sb);
  if (e != hipSuccess) {
    cleanup();
    return fail(MP3G_ERR_OUT_OF_MEMORY, "hipMalloc", e);
  }
  if (gb) e = hipMemcpyAsync(dg, granules, gb, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess && cb) e = hipMemcpyAsync(dc, coeffs, cb, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess && need_in) e = hipMemcpyAsync(dsi, state_in, sb, hipMemcpyHostToDevice, stream);
  // streams without MP3G_STREAM_STATE_OUT keep the caller's state_out bytes
  if (e == hipSuccess && need_out) e = hipMemcpyAsync(dso, state_out, sb, hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) {
    cleanup();
    return fail(MP3G_ERR_DEVICE, "hipMemcpyAsync(H2D)", e);
  }
  st = mp3g_plan_execute(plan, (const mp3g_granule*)dg, (const int16_t*)dc, (const mp3g_state*)dsi,
                         (mp3g_state*)dso, (int16_t*)dp, stream);
  if (st) {
    cleanup();
    return st;
  }
  if (pb) e = hipMemcpyAsync(pcm, dp, pb, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess && need_out) e = hipMemcpyAsync(state_out, dso, sb, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  cleanup();
  if (e != hipSuccess) return fail(MP3G_ERR_DEVICE, "decode", e);
  return MP3G_OK;
}

}  // extern "C"
