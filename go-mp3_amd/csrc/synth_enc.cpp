// synth_enc.cpp -- seeded synthetic MPEG-1/2 Layer III bitstream writer.
// BENCH / TEST TOOLING (libmp3gsynth.so), not part of the decode path.
//
// There is no MP3 encoder in the reference or in this image,
// so the bitstream workloads -- c2/c3 as real 128 kbps CBR streams, and
// streams with intensity stereo, mixed blocks and linbits tables that neither
// sample file exercises -- are written here: random quantized spectra and
// scale factors with the statistics of a 44.1 kHz 128 kbps joint-stereo
// stream, Huffman-coded with the ISO 11172-3 Table B.7 codes
// (huffman_codes.inc), packed into frames of the exact CBR size through the
// bit reservoir (main_data_begin) as a real encoder does.  Alongside the
// bytes it returns what a decoder must recover (granule descriptors +
// coefficients in the boundary layout of include/mp3g.h): an independent
// check of every bitstream parse (tests/test_synth_cpu.py).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/mp3g.h"

extern "C" {
typedef struct mp3g_synth_params {
  uint64_t seed;
  int32_t n_frames;
  int32_t lsf;            // 0: MPEG-1, 1: MPEG-2 LSF
  int32_t mode;           // 0 stereo, 1 joint stereo, 2 dual channel, 3 mono
  int32_t bitrate_index;  // 9 = 128 kbps (MPEG-1); 8 = 64 kbps (MPEG-2)
  int32_t sfreq;          // 0 = 44.1 / 22.05 kHz
  int32_t gain_boost;     // added to every granule's global_gain (capped at 255): loud content
  double p_ms;            // joint stereo: P(mode_ext MS bit) per frame
  double p_is;            // joint stereo: P(mode_ext IS bit) per frame
  double p_event;         // P(a long -> start -> short.. -> stop run starts) per granule
  double p_mixed;         // P(mixed block) per short granule (MPEG-1 only)
  double p_big;           // P(a big-values line needs linbits)
  double fill;            // mean fraction of the frame budget a granule aims at
} mp3g_synth_params;
}

namespace {

#include "huffman_codes.inc"  // ISO 11172-3 Table B.7 codeword lists (data)

struct Rng {
  uint64_t s;
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  int range(int lo, int hi) { return hi <= lo ? lo : lo + (int)(next() % (uint64_t)(hi - lo)); }
  double laplace(double b) { return -b * std::log(1.0 - uni()); }
};

struct Bw {
  std::vector<uint8_t> v;
  uint64_t pos = 0;
  void put(uint32_t val, int n) {
    for (int i = n - 1; i >= 0; i--) {
      if ((pos >> 3) >= v.size()) v.push_back(0);
      if ((val >> i) & 1u) v[pos >> 3] |= (uint8_t)(0x80u >> (pos & 7));
      pos++;
    }
  }
};

struct Codes {
  uint32_t code[34][16][16];
  uint8_t len[34][16][16];
  int xmax[34];
  Codes() {
    std::memset(this, 0, sizeof *this);
    for (int k = 0; k < HUFF_N_CODES; k++) {
      const huff_code_t& c = HUFF_CODES[k];
      code[c.tree][c.x][c.y] = c.code;
      len[c.tree][c.x][c.y] = (uint8_t)c.len;
      if (c.x > xmax[c.tree]) xmax[c.tree] = c.x;
    }
  }
};
const Codes& codes() {
  static const Codes c;
  return c;
}

// largest magnitude table t can code (-1: none)
int table_cap(int t) {
  const int tree = HUFF_TABLE_TREE[t];
  if (tree < 0) return -1;
  const int lb = HUFF_TABLE_LINBITS[t];
  return lb ? 15 + (1 << lb) - 1 : codes().xmax[tree];
}

const int kSfbLong[2][3][23] = {
    {{0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576},
     {0, 4, 8, 12, 16, 20, 24, 30, 36, 42, 50, 60, 72, 88, 106, 128, 156, 190, 230, 276, 330, 384, 576},
     {0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 54, 66, 82, 102, 126, 156, 194, 240, 296, 364, 448, 550, 576}},
    {{0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576},
     {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 114, 136, 162, 194, 232, 278, 332, 394, 464, 540, 576},
     {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576}}};
const int kSlen1[16][2] = {{0, 0}, {0, 1}, {0, 2}, {0, 3}, {3, 0}, {1, 1}, {1, 2}, {1, 3},
                           {2, 1}, {2, 2}, {2, 3}, {3, 1}, {3, 2}, {3, 3}, {4, 2}, {4, 3}};
const int kNsfb2[3][6][4] = {
    {{6, 5, 5, 5}, {6, 5, 7, 3}, {11, 10, 0, 0}, {7, 7, 7, 0}, {6, 6, 6, 3}, {8, 8, 5, 0}},
    {{9, 9, 9, 9}, {9, 9, 12, 6}, {18, 18, 0, 0}, {12, 12, 12, 0}, {12, 9, 9, 6}, {15, 12, 9, 0}},
    {{6, 9, 9, 9}, {6, 9, 12, 6}, {15, 18, 0, 0}, {6, 15, 12, 0}, {6, 12, 9, 6}, {6, 18, 9, 0}}};
// MPEG-2 scalefac_compress (9 bits) -> 3-bit slen fields, table row, preflag
// (ISO 13818-3 2.4.3.2; the packing of reference maindata.go:52-81)
int slen2_word(int sc) {
  if (sc >= 500) {
    const int a = (sc - 500) / 3, b = (sc - 500) % 3;
    return a | (b << 3) | (2 << 12) | (1 << 15);
  }
  if (sc >= 400) {
    const int r = sc - 400, a = r / 20, b = (r / 4) % 5, c = r % 4;
    return a | (b << 3) | (c << 6) | (1 << 12);
  }
  const int a = sc / 80, b = (sc / 16) % 5, c = (sc / 4) % 4, d = sc % 4;
  return a | (b << 3) | (c << 6) | (d << 9);
}

int bitrate_bps(int lsf, int idx) {
  static const int k1[16] = {0, 32000, 40000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 160000,
                             192000, 224000, 256000, 320000, 0};
  static const int k2[16] = {0, 8000, 16000, 24000, 32000, 40000, 48000, 56000, 64000, 80000, 96000,
                             112000, 128000, 144000, 160000, 0};
  return lsf ? k2[idx] : k1[idx];
}
int sample_rate(int lsf, int sf) {
  static const int k[3] = {44100, 48000, 32000};
  return k[sf] >> lsf;
}

// side info of one granule-channel (sideinfo.go field order)
struct Gc {
  int part2_3_length = 0, big_values = 0, global_gain = 0, scalefac_compress = 0;
  int win_switch = 0, block_type = 0, mixed = 0;
  int table_select[3] = {0, 0, 0}, subblock_gain[3] = {0, 0, 0};
  int region0_count = 0, region1_count = 0, preflag = 0, scalefac_scale = 0, count1_table = 0;
};

struct Encoder {
  const mp3g_synth_params& P;
  Rng rng;
  int lsf, nch;
  explicit Encoder(const mp3g_synth_params& p)
      : P(p), rng{p.seed * 0x2545F4914F6CDD1Dull + 1}, lsf(p.lsf != 0), nch(p.mode == 3 ? 1 : 2) {}

  // a random table among the three tightest that can code maxabs
  int pick_table(int maxabs) {
    if (maxabs == 0 && rng.uni() < 0.5) return 0;
    int cand[32], n = 0;
    for (int t = 1; t < 32; t++)
      if (table_cap(t) >= maxabs) cand[n++] = t;
    std::stable_sort(cand, cand + n, [](int a, int b) { return table_cap(a) < table_cap(b); });
    return cand[rng.range(0, n < 3 ? n : 3)];
  }

  void put_pair(Bw& w, int t, int x, int y) {
    const int tree = HUFF_TABLE_TREE[t];
    if (tree < 0) return;  // table 0: all-zero region, no bits
    const int lb = HUFF_TABLE_LINBITS[t];
    const int ax = std::abs(x), ay = std::abs(y);
    const int cx = lb && ax > 15 ? 15 : ax, cy = lb && ay > 15 ? 15 : ay;
    w.put(codes().code[tree][cx][cy], codes().len[tree][cx][cy]);
    if (lb && cx == 15) w.put((uint32_t)(ax - 15), lb);
    if (ax) w.put(x < 0, 1);
    if (lb && cy == 15) w.put((uint32_t)(ay - 15), lb);
    if (ay) w.put(y < 0, 1);
  }

  // Scale factors + Huffman data of one granule-channel into w; fills its side
  // info and the expected decoder output (descriptor channel + 576 lines).
  // scfsi: MPEG-1 granule-1 copy mask; sf0: granule 0's long scale factors.
  void granule(Bw& w, int gr, int scfsi, const uint8_t* sf0, double size, int sfreq, Gc* s, mp3g_channel* out,
               int16_t* lines) {
    const uint64_t start = w.pos;
    const bool shortblk = s->win_switch && s->block_type == 2;
    s->global_gain = std::min(255, rng.range(140, 181) + P.gain_boost);
    s->scalefac_scale = rng.uni() < 0.2;
    s->preflag = !lsf && !shortblk && rng.uni() < 0.3;
    for (int k = 0; k < 3; k++) s->subblock_gain[k] = s->win_switch ? rng.range(0, 8) : 0;
    std::memset(out, 0, sizeof *out);
    // ---- part 2: scale factors (maindata.go:119-279) ----
    auto val = [&](int nb) { return nb ? rng.range(0, 1 << nb) : 0; };
    if (!lsf) {
      s->scalefac_compress = rng.range(0, 16);
      const int s1 = kSlen1[s->scalefac_compress][0], s2 = kSlen1[s->scalefac_compress][1];
      if (shortblk) {
        int sfb0 = 0;
        if (s->mixed) {
          for (int sfb = 0; sfb < 8; sfb++) {
            out->scalefac_l[sfb] = (uint8_t)val(s1);
            w.put(out->scalefac_l[sfb], s1);
          }
          sfb0 = 3;
        }
        for (int sfb = sfb0; sfb < 12; sfb++)
          for (int win = 0; win < 3; win++) {
            const int nb = sfb < 6 ? s1 : s2;
            out->scalefac_s[sfb][win] = (uint8_t)val(nb);
            w.put(out->scalefac_s[sfb][win], nb);
          }
      } else {
        static const int lo[4] = {0, 6, 11, 16}, hi[4] = {6, 11, 16, 21};
        for (int part = 0; part < 4; part++) {
          const int nb = part < 2 ? s1 : s2;
          for (int sfb = lo[part]; sfb < hi[part]; sfb++) {
            if (gr == 1 && ((scfsi >> (3 - part)) & 1)) {
              out->scalefac_l[sfb] = sf0[sfb];  // copied from granule 0, not transmitted
            } else {
              out->scalefac_l[sfb] = (uint8_t)val(nb);
              w.put(out->scalefac_l[sfb], nb);
            }
          }
        }
      }
    } else {
      s->scalefac_compress = rng.range(0, 512);
      int slen = slen2_word(s->scalefac_compress);
      s->preflag = (slen >> 15) & 1;
      const int blk = s->block_type == 2 ? 1 : 0;  // (no MPEG-2 mixed blocks: the reference panics)
      const int row = (slen >> 12) & 7;
      int k = 0;
      for (int part = 0; part < 4; part++) {
        const int nb = slen & 7;
        slen >>= 3;
        for (int n = 0; n < kNsfb2[blk][row][part]; n++, k++) {
          const int v = val(nb);
          if (nb) w.put((uint32_t)v, nb);
          if (blk == 0) out->scalefac_l[k] = (uint8_t)v;
          else out->scalefac_s[k / 3][k % 3] = (uint8_t)v;
        }
      }
    }
    // ---- part 3: spectrum ----
    std::memset(lines, 0, 576 * sizeof(int16_t));
    int bv = (int)std::lround(size * rng.range(30, 200));
    bv = std::min(bv, 288);
    const double amp = 0.8 + 2.2 * rng.uni(), decay = 60.0 + 140.0 * rng.uni();
    for (int i = 0; i < 2 * bv; i++) {
      double m = rng.laplace(amp * std::exp(-i / decay));
      if (rng.uni() < P.p_big) m = rng.laplace(60.0);
      const int v = std::min((int)std::lround(m), 8206);
      lines[i] = (int16_t)(rng.uni() < 0.5 ? -v : v);
    }
    int nq = (int)std::lround(size * rng.uni() * ((576 - 2 * bv) / 4) * 0.6);
    nq = std::min(nq, (576 - 2 * bv) / 4);
    for (int i = 2 * bv; i < 2 * bv + 4 * nq; i++) {
      const double u = rng.uni();
      lines[i] = (int16_t)(u < 0.25 ? -1 : u < 0.5 ? 1 : 0);
    }
    // regions (maindata/huffman.go:39-64; sideinfo.go:128-136 for the implicit
    // window-switching counts) and their tables
    int r1, r2;
    if (shortblk) {
      r1 = 36;
      r2 = 576;
    } else {
      if (s->win_switch) {
        s->region0_count = 7;  // not transmitted: start/stop blocks
        s->region1_count = 13;
      } else {
        s->region0_count = rng.range(0, 16);
        s->region1_count = rng.range(0, 8);
      }
      const int* l = kSfbLong[lsf][sfreq];
      r1 = l[s->region0_count + 1];
      const int j = s->region0_count + s->region1_count + 2;
      r2 = j >= 23 ? 576 : l[j];
    }
    const int bounds[4] = {0, std::min(r1, 2 * bv), std::min(r2, 2 * bv), 2 * bv};
    for (int r = 0; r < 3; r++) {
      int mx = 0;
      for (int i = bounds[r]; i < bounds[r + 1]; i++) mx = std::max(mx, (int)std::abs(lines[i]));
      s->table_select[r] = pick_table(mx);
    }
    if (s->win_switch) s->table_select[2] = 0;  // two table selects only (region 2 unused)
    s->count1_table = rng.range(0, 2);
    s->big_values = bv;
    for (int i = 0; i < 2 * bv; i += 2) {
      const int t = i < r1 ? s->table_select[0] : i < r2 ? s->table_select[1] : s->table_select[2];
      put_pair(w, t, lines[i], lines[i + 1]);
    }
    const int qt = 32 + s->count1_table;
    for (int q = 0; q < nq; q++) {
      const int i = 2 * bv + 4 * q;
      const int v = lines[i], ww = lines[i + 1], x = lines[i + 2], y = lines[i + 3];
      const int code = ((v != 0) << 3) | ((ww != 0) << 2) | ((x != 0) << 1) | (y != 0);
      w.put(codes().code[qt][0][code], codes().len[qt][0][code]);
      if (v) w.put(v < 0, 1);
      if (ww) w.put(ww < 0, 1);
      if (x) w.put(x < 0, 1);
      if (y) w.put(y < 0, 1);
    }
    s->part2_3_length = (int)(w.pos - start);
    // expected decoder output
    out->count1 = (uint16_t)(s->part2_3_length ? 2 * bv + 4 * nq : 0);
    if (!s->part2_3_length) std::memset(lines, 0, 576 * sizeof(int16_t));
    out->global_gain = (uint8_t)s->global_gain;
    out->scalefac_scale = (uint8_t)s->scalefac_scale;
    out->preflag = (uint8_t)s->preflag;
    out->win_switch_flag = (uint8_t)s->win_switch;
    out->block_type = (uint8_t)s->block_type;
    out->mixed_block_flag = (uint8_t)s->mixed;
    for (int k = 0; k < 3; k++) out->subblock_gain[k] = (uint8_t)s->subblock_gain[k];
  }

  // sideinfo.go:88-156 field order
  void side_info(Bw& w, int mdb, const int scfsi[2], const Gc g[2][2]) {
    const int ng = lsf ? 1 : 2;
    w.put((uint32_t)mdb, lsf ? 8 : 9);
    w.put(0, lsf ? (nch == 1 ? 1 : 2) : (nch == 1 ? 5 : 3));  // private bits
    if (!lsf)
      for (int ch = 0; ch < nch; ch++) w.put((uint32_t)scfsi[ch], 4);
    for (int gr = 0; gr < ng; gr++)
      for (int ch = 0; ch < nch; ch++) {
        const Gc& s = g[gr][ch];
        w.put((uint32_t)s.part2_3_length, 12);
        w.put((uint32_t)s.big_values, 9);
        w.put((uint32_t)s.global_gain, 8);
        w.put((uint32_t)s.scalefac_compress, lsf ? 9 : 4);
        w.put((uint32_t)s.win_switch, 1);
        if (s.win_switch) {
          w.put((uint32_t)s.block_type, 2);
          w.put((uint32_t)s.mixed, 1);
          w.put((uint32_t)s.table_select[0], 5);
          w.put((uint32_t)s.table_select[1], 5);
          for (int k = 0; k < 3; k++) w.put((uint32_t)s.subblock_gain[k], 3);
        } else {
          for (int k = 0; k < 3; k++) w.put((uint32_t)s.table_select[k], 5);
          w.put((uint32_t)s.region0_count, 4);
          w.put((uint32_t)s.region1_count, 3);
        }
        if (!lsf) w.put((uint32_t)s.preflag, 1);
        w.put((uint32_t)s.scalefac_scale, 1);
        w.put((uint32_t)s.count1_table, 1);
      }
  }

  int64_t run(uint8_t* out, int64_t cap, mp3g_granule* gran, int16_t* coef) {
    const int ng = lsf ? 1 : 2, sfreq = P.sfreq;
    const int br = bitrate_bps(lsf, P.bitrate_index), fs = sample_rate(lsf, sfreq);
    const int si_bytes = lsf ? (nch == 1 ? 9 : 17) : (nch == 1 ? 17 : 32);
    const int max_back = lsf ? 255 : 511;
    const int nf = P.n_frames;
    std::vector<uint32_t> hdr(nf);
    std::vector<int64_t> slot(nf + 1);  // start of each frame's main-data area in the concatenation
    std::vector<std::vector<uint8_t>> side(nf);
    // frame sizes: CBR padding accumulator (MPEG-1); MPEG-2 frames unpadded (the
    // reference sizes them ((144 br)/f + pad) >> 1, frameheader.go:223-232)
    int64_t acc = 0, total = 0, bytes = 0;
    for (int f = 0; f < nf; f++) {
      int pad = 0;
      if (!lsf) {
        acc += (144LL * br) % fs;
        if (acc >= fs) {
          acc -= fs;
          pad = 1;
        }
      }
      const int fsize = ((144 * br) / fs + pad) >> lsf;
      int modeext = 0;
      if (P.mode == 1) modeext = ((rng.uni() < P.p_ms) << 1) | (rng.uni() < P.p_is);
      hdr[f] = (lsf ? 0xFFF30000u : 0xFFFB0000u) | ((uint32_t)P.bitrate_index << 12) | ((uint32_t)sfreq << 10) |
               ((uint32_t)pad << 9) | ((uint32_t)P.mode << 6) | ((uint32_t)modeext << 4) | 4u;
      slot[f] = total;
      total += fsize - 4 - si_bytes;
      bytes += fsize;
    }
    slot[nf] = total;
    if (bytes > cap || total <= 0) return 0;
    std::vector<uint8_t> G((size_t)total);
    for (auto& b : G) b = (uint8_t)rng.next();  // ancillary / stuffing bytes

    int state[2] = {0, 0};  // window switching per channel: 0 long, k>0 short granules left, -1 stop next
    int64_t prev_end = 0;
    const double budget = (double)(total * 8) / ((double)nf * ng * nch);  // bits per granule-channel
    std::vector<uint8_t> sf0_zero(22, 0);
    for (int f = 0; f < nf; f++) {
      Gc g[2][2];
      mp3g_granule D[2];
      std::memset(D, 0, sizeof D);
      int16_t L[2][2][576];
      std::memset(L, 0, sizeof L);
      int scfsi[2] = {0, 0};
      for (int gr = 0; gr < ng; gr++) {
        // channel 1 follows channel 0's window switching 80 % of the time
        const bool shared = rng.uni() < 0.8 && state[1] == state[0];
        for (int ch = 0; ch < nch; ch++) {
          Gc& s = g[gr][ch];
          int bt = 0, mx = 0;
          if (ch == 1 && shared) {
            bt = g[gr][0].block_type;
            mx = g[gr][0].mixed;
            state[1] = state[0];
          } else {
            int& st = state[ch];
            if (st == 0) {
              if (rng.uni() < P.p_event) {
                bt = 1;  // start block, then 1..3 short granules, then a stop block
                st = rng.range(1, 4);
              }
            } else if (st > 0) {
              bt = 2;
              mx = !lsf && rng.uni() < P.p_mixed;
              st = st == 1 ? -1 : st - 1;
            } else {
              bt = 3;
              st = 0;
            }
          }
          s.block_type = bt;
          s.win_switch = bt != 0;
          s.mixed = bt == 2 ? mx : 0;
        }
      }
      if (!lsf)
        for (int ch = 0; ch < nch; ch++) scfsi[ch] = rng.uni() < 0.3 ? rng.range(0, 16) : 0;
      const bool is_frame = P.mode == 1 && (hdr[f] & 0x10u);
      // encode; shrink the spectra until the frame's data fits its reservoir window
      double size = P.fill * budget / 700.0;
      int64_t pos_f = 0;
      for (int attempt = 0;; attempt++) {
        Bw w;
        for (int gr = 0; gr < ng; gr++)
          for (int ch = 0; ch < nch; ch++) {
            double sz = size * (0.6 + 0.8 * rng.uni());
            if (is_frame && ch == 1) sz *= 0.4;
            if (attempt >= 12) sz = 0.0;
            granule(w, gr, scfsi[ch], gr ? D[0].ch[ch].scalefac_l : sf0_zero.data(), sz, sfreq, &g[gr][ch],
                    &D[gr].ch[ch], L[gr][ch]);
          }
        bool ok = true;
        for (int gr = 0; gr < ng; gr++)
          for (int ch = 0; ch < nch; ch++) ok = ok && g[gr][ch].part2_3_length <= 4095;
        const int64_t len = (int64_t)((w.pos + 7) / 8);
        pos_f = f == 0 ? 0 : std::max<int64_t>(prev_end, std::max<int64_t>(0, slot[f] - max_back));
        if (ok && pos_f + len <= slot[f + 1]) {
          if (len) std::memcpy(&G[(size_t)pos_f], w.v.data(), (size_t)len);
          prev_end = pos_f + len;
          break;
        }
        if (attempt >= 12) return 0;  // not even empty granules fit (cannot happen for valid params)
        size *= 0.7;
      }
      Bw si;
      side_info(si, (int)(slot[f] - pos_f), scfsi, g);
      side[f] = si.v;
      side[f].resize((size_t)si_bytes, 0);
      for (int gr = 0; gr < ng; gr++) {
        D[gr].header = hdr[f];
        D[gr].gr = (uint32_t)gr;
      }
      if (gran) std::memcpy(gran + (size_t)f * ng, D, (size_t)ng * sizeof(mp3g_granule));
      if (coef)
        for (int gr = 0; gr < ng; gr++)
          std::memcpy(coef + ((size_t)f * ng + gr) * MP3G_COEF_PER_GRANULE, L[gr], sizeof L[gr]);
    }
    // frames: header | side info | the frame's slot of the main-data concatenation
    int64_t o = 0;
    for (int f = 0; f < nf; f++) {
      out[o++] = (uint8_t)(hdr[f] >> 24);
      out[o++] = (uint8_t)(hdr[f] >> 16);
      out[o++] = (uint8_t)(hdr[f] >> 8);
      out[o++] = (uint8_t)hdr[f];
      std::memcpy(out + o, side[f].data(), (size_t)si_bytes);
      o += si_bytes;
      const int64_t n = slot[f + 1] - slot[f];
      std::memcpy(out + o, &G[(size_t)slot[f]], (size_t)n);
      o += n;
    }
    return o;
  }
};

}  // namespace

extern "C" {

// Writes the stream into out[0, cap) and returns its length (0: it does not
// fit or the parameters are invalid).  gran / coef (optional) receive the
// expected decoder output: n_frames * (2 - lsf) descriptors and coefficient
// blocks (include/mp3g.h layout).
int64_t mp3g_synth_encode(const mp3g_synth_params* p, uint8_t* out, int64_t cap, mp3g_granule* gran,
                          int16_t* coef) {
  if (!p || !out || p->n_frames <= 0 || p->bitrate_index <= 0 || p->bitrate_index >= 15 || p->sfreq < 0 ||
      p->sfreq > 2 || p->mode < 0 || p->mode > 3)
    return 0;
  Encoder e(*p);
  return e.run(out, cap, gran, coef);
}

}  // extern "C"
