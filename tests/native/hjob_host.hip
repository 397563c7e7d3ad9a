// hjob_host.hip -- TEST INFRASTRUCTURE: the device main-data job decoder
// (go-mp3_amd/csrc/huffman_job.h, __host__ __device__) compiled for the CPU,
// so tests/test_scan_cpu.py can check the scan's job decomposition against
// the host parse byte for byte without a GPU.  Not linked into libmp3g.so.
#include "../../go-mp3_amd/csrc/huffman_job.h"

extern "C" int hjob_decode_host(const mp3g_hjob* jobs, uint64_t n_granules, const uint8_t* md, mp3g_granule* gran,
                                int16_t* coef) {
  static mp3g::HuffLut lut;
  static const bool ok = mp3g::build_huff_lut(&lut);
  if (!ok) return 1;
  for (uint64_t j = 0; j < 2 * n_granules; j++)
    mp3g::huff::decode_job(jobs[j], j, md, gran, coef, lut.e, lut.root, lut.linbits);
  return 0;
}
