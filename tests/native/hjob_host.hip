// hjob_host.hip -- TEST INFRASTRUCTURE: the device main-data job decoder
// (go-mp3_amd/csrc/huffman_job.h, __host__ __device__) compiled for the CPU,
// so tests/test_scan_cpu.py can check the scan's job decomposition against
// the host parse byte for byte without a GPU.  Not linked into libmp3g.so.
#include <vector>

#include "../../go-mp3_amd/csrc/huffman_job.h"

extern "C" int hjob_decode_host(const mp3g_hjob* jobs, uint64_t n_granules, const uint8_t* md, mp3g_granule* gran,
                                int16_t* coef) {
  static mp3g::HuffLut lut;
  static const bool ok = mp3g::build_huff_lut(&lut);
  if (!ok) return 1;
  for (uint64_t j = 0; j < 2 * n_granules; j++)
    mp3g::huff::zero_fill_row(coef + j * MP3G_LINES,
                              mp3g::huff::decode_job_direct(jobs[j], j, md, gran, coef, lut.e, lut.root, lut.linbits));
  return 0;
}

// The kernel's LDS path (huffman_dev.hip): per group of 64 consecutive jobs,
// the main-data span [lo, hi) is copied byte-swapped into a staging buffer
// and the jobs read it through Reader<false>.  `stage_words` is the capacity
// (groups that do not fit read directly, as on the device).
extern "C" int hjob_decode_host_staged(const mp3g_hjob* jobs, uint64_t n_granules, const uint8_t* md,
                                       mp3g_granule* gran, int16_t* coef, uint32_t stage_words) {
  static mp3g::HuffLut lut;
  static const bool ok = mp3g::build_huff_lut(&lut);
  if (!ok) return 1;
  const uint64_t n = 2 * n_granules;
  std::vector<uint64_t> stage(stage_words + 4);  // the reader loads up to 3 words past nw
  for (uint64_t j0 = 0; j0 < n; j0 += 64) {
    const uint64_t j1 = j0 + 64 < n ? j0 + 64 : n;
    uint64_t lo = ~0ull, hi = 0;
    for (uint64_t j = j0; j < j1; j++) {
      if (jobs[j].sf_kind == MP3G_SF_NONE) continue;
      const uint64_t b = mp3g::huff::job_base(jobs[j]);
      lo = b < lo ? b : lo;
      hi = jobs[j].bit_end > hi ? jobs[j].bit_end : hi;
    }
    const uint64_t nwords = hi > lo && lo != ~0ull ? (hi - lo + 63) >> 6 : 0;
    const bool staged = nwords <= stage_words;
    if (staged)
      for (uint64_t k = 0; k < nwords; k++) {
        uint64_t v;
        __builtin_memcpy(&v, md + (lo >> 3) + 8 * k, 8);
        stage[k] = mp3g::huff::bswap64(v);
      }
    for (uint64_t j = j0; j < j1; j++) {
      if (!staged) {
        mp3g::huff::zero_fill_row(coef + j * MP3G_LINES, mp3g::huff::decode_job_direct(jobs[j], j, md, gran, coef,
                                                                                      lut.e, lut.root, lut.linbits));
        continue;
      }
      const uint32_t off = jobs[j].sf_kind != MP3G_SF_NONE ? (uint32_t)((mp3g::huff::job_base(jobs[j]) - lo) >> 6) : 0;
      const int z = mp3g::huff::decode_job<false>(jobs[j], j, stage.data() + off, (uint32_t)nwords - off, gran, coef,
                                                  lut.e, lut.root, lut.linbits);
      mp3g::huff::zero_fill_row(coef + j * MP3G_LINES, z);
    }
  }
  return 0;
}
