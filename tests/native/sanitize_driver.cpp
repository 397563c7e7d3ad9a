// sanitize_driver.cpp -- the untrusted-input host code under ASan + UBSan
// (sanitizers on the CPU side; the role of the reference's
// fuzzing_test.go:22-107 regression corpus).
//
// Built by `make -C go-mp3_amd/csrc asan` with every host object of
// libmp3g.so and the oracle instrumented (build/asan/sanitize_driver).  For
// each input file: the batched host parse (mp3g_parse_stream /
// mp3g_parse_streams), the host scan of the GPU main-data path
// (mp3g_scan_streams), the Xing/LAME tag parsers and, as a second restatement
// of the same parse, the oracle's NewDecoder + ReadAll and a few seeks.  No
// GPU call.  A sanitizer report aborts the process (halt_on_error); exit 0
// means every input went through clean.  tests/test_sanitize_cpu.py feeds it
// the sample files, the fuzz corpus, seeded mutations and synthetic streams.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/mp3g.h"
#include "../../oracle/mp3_oracle.h"

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> b;
  FILE* f = std::fopen(path, "rb");
  if (!f) return b;
  uint8_t buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
  std::fclose(f);
  return b;
}

int main(int argc, char** argv) {
  long granules = 0;
  for (int a = 1; a < argc; a++) {
    std::vector<uint8_t> d = slurp(argv[a]);
    const uint8_t* p = d.empty() ? nullptr : d.data();
    // batched host parse
    mp3g_granule* g = nullptr;
    int16_t* c = nullptr;
    uint64_t n = 0;
    int end = 0;
    if (mp3g_parse_stream(p, d.size(), &g, &c, &n, &end) == MP3G_OK) granules += (long)n;
    mp3g_free(g);
    mp3g_free(c);
    // the same stream twice through the multi-threaded form
    const uint8_t* ds[2] = {p, p};
    size_t ls[2] = {d.size(), d.size()};
    mp3g_stream st[2];
    int ends[2];
    g = nullptr;
    c = nullptr;
    if (mp3g_parse_streams(2, ds, ls, 2, &g, &c, &n, st, ends) == MP3G_OK) granules += (long)n;
    mp3g_free(g);
    mp3g_free(c);
    // host scan (reservoir resolution, Huffman jobs)
    mp3g_scan* sc = nullptr;
    if (mp3g_scan_streams(2, ds, ls, 2, &sc) == MP3G_OK) {
      uint64_t ng = 0, nmd = 0;
      const mp3g_granule* sg;
      const mp3g_hjob* sj;
      const uint8_t* smd;
      const mp3g_stream* sst;
      const int* ses;
      mp3g_scan_buffers(sc, &ng, &nmd, &sg, &sj, &smd, &sst, &ses);
      mp3g_scan_free(sc);
    }
    // Xing / LAME tag parsers on the head of the stream and on every offset
    // of the first KiB
    mp3g_lame_info li;
    size_t used = 0;
    mp3g_lame_parse_reader(p, d.size(), &li, &used);
    for (size_t off = 0; off < d.size() && off < 1024; off++) {
      if (mp3g_lame_parse(p + off, d.size() - off, &li) == MP3G_OK) {
        uint64_t first, count, toc;
        mp3g_lame_trim(&li, 1u << 20, 1152, &first, &count);
        mp3g_lame_toc_offset(&li, 37.5, d.size(), &toc);
      }
    }
    // the oracle's restatement of the same parse (test infrastructure)
    uint8_t* pcm = nullptr;
    size_t pl = 0;
    orc_decode_all(p, d.size(), &pcm, &pl);
    orc_free(pcm);
    orc_decoder* dec = nullptr;
    if (orc_decoder_new(p, d.size(), 1, &dec) == ORC_OK) {
      static uint8_t buf[4608 * 4];
      size_t k = 0;
      int64_t np = 0;
      for (int i = 0; i < 8 && orc_decoder_read(dec, buf, sizeof buf, &k) == ORC_OK; i++) {
      }
      orc_decoder_seek(dec, 4608 * 3 + 100, 0, &np);
      orc_decoder_read(dec, buf, sizeof buf, &k);
      orc_decoder_seek(dec, -5000, 1, &np);
      orc_decoder_read(dec, buf, sizeof buf, &k);
      orc_decoder_free(dec);
    }
  }
  std::printf("sanitize_driver: %d inputs clean (%ld granules parsed)\n", argc - 1, granules);
  return 0;
}
