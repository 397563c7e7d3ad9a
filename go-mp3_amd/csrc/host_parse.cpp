// host_parse.cpp -- see host_parse.h.  Reference file:line citations on each
// function; all behaviour below is what go-mp3 does, restated for a byte
// buffer and batched output.
#include "host_parse.h"

#include <algorithm>
#include <cstring>
#include <mutex>

namespace mp3g {
namespace host {
namespace {

#include "huffman_codes.inc"  // ISO 11172-3 Table B.7 codeword lists (data)

// ---- frame header accessors (frameheader.go:82-251) ----------------------
inline int h_id(uint32_t h) { return (int)((h >> 19) & 3u); }
inline int h_layer(uint32_t h) { return (int)((h >> 17) & 3u); }
inline int h_protection(uint32_t h) { return (int)((h >> 16) & 1u); }
inline int h_bitrate_index(uint32_t h) { return (int)((h >> 12) & 15u); }
inline int h_sfreq(uint32_t h) { return (int)((h >> 10) & 3u); }
inline int h_padding(uint32_t h) { return (int)((h >> 9) & 1u); }
inline int h_mode(uint32_t h) { return (int)((h >> 6) & 3u); }
inline int h_emphasis(uint32_t h) { return (int)(h & 3u); }
inline int h_lsf(uint32_t h) { return h_id(h) == 3 ? 0 : 1; }
inline int h_nch(uint32_t h) { return h_mode(h) == 3 ? 1 : 2; }

bool h_valid(uint32_t h) {  // frameheader.go:168-189
  return (h & 0xffe00000u) == 0xffe00000u && h_id(h) != 1 && h_bitrate_index(h) != 15 &&
         h_sfreq(h) != 3 && h_layer(h) == 1 && h_emphasis(h) != 2;
}

int h_bitrate(uint32_t h) {  // frameheader.go:191-221 (layer III rows used; the table is ISO's)
  static const int kBr[2][3][16] = {
      {{0, 32000, 40000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 160000, 192000, 224000, 256000, 320000, 0},
       {0, 32000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 160000, 192000, 224000, 256000, 320000, 384000, 0},
       {0, 32000, 64000, 96000, 128000, 160000, 192000, 224000, 256000, 288000, 320000, 352000, 384000, 416000, 448000, 0}},
      {{0, 8000, 16000, 24000, 32000, 40000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 144000, 160000, 0},
       {0, 8000, 16000, 24000, 32000, 40000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 144000, 160000, 0},
       {0, 32000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 144000, 160000, 176000, 192000, 224000, 256000, 0}}};
  const int layer = h_layer(h);
  return layer < 1 ? 0 : kBr[h_lsf(h)][layer - 1][h_bitrate_index(h)];
}

int h_side_info_size(uint32_t h) {  // frameheader.go:234-251
  const bool mono = h_mode(h) == 3;
  return h_lsf(h) ? (mono ? 9 : 17) : (mono ? 17 : 32);
}

// scale-factor band starts (consts.go:68-97): long bands [lsf][sfreq]
const int kSfbLong[2][3][23] = {
    {{0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576},
     {0, 4, 8, 12, 16, 20, 24, 30, 36, 42, 50, 60, 72, 88, 106, 128, 156, 190, 230, 276, 330, 384, 576},
     {0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 54, 66, 82, 102, 126, 156, 194, 240, 296, 364, 448, 550, 576}},
    {{0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576},
     {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 114, 136, 162, 194, 232, 278, 332, 394, 464, 540, 576},
     {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576}}};

// ---- bit reader (bits.go:22-94) --------------------------------------------
// Reads that would pass the end return 0 and leave the position unchanged
// (the reference never checks the error, so decoding carries on with zeros).
// The backing buffer has >= 8 zero bytes of padding for 32-bit peeks.
struct Bits {
  const uint8_t* v;
  int64_t len;  // bytes
  int64_t pos = 0;
  Bits(const uint8_t* p, int64_t n) : v(p), len(n) {}
  int64_t nbits() const { return len * 8; }
  uint32_t peek32() const {  // big-endian 32 bits at pos (pos < nbits)
    const int64_t b = pos >> 3;
    const uint32_t w = ((uint32_t)v[b] << 24) | ((uint32_t)v[b + 1] << 16) | ((uint32_t)v[b + 2] << 8) | v[b + 3];
    const uint32_t nx = v[b + 4];
    const int s = (int)(pos & 7);
    return s ? (w << s) | (nx >> (8 - s)) : w;
  }
  int bit() {  // bits.go:45-56
    if (pos >= nbits()) return 0;
    const int r = (v[pos >> 3] >> (7 - (pos & 7))) & 1;
    pos++;
    return r;
  }
  int bits(int n) {  // bits.go:58-77
    if (n == 0) return 0;
    if (pos + n > nbits()) return 0;
    const int r = (int)(peek32() >> (32 - n));
    pos += n;
    return r;
  }
};

// ---- Huffman tables ---------------------------------------------------------
// Per tree: a 10-bit first-level table; codewords longer than 10 bits go
// through a second level indexed by the next 9 bits (max length 19).
// Entry: len (bits 0..4) and x<<4|y (bits 8..15); len 0 marks a link whose
// second-level block offset is in bits 5..31.
constexpr int kL1 = 10, kL2 = 9;
struct HuffLut {
  std::vector<uint32_t> e;  // [tree][1 << kL1] then second-level blocks
  int base[34] = {};
  // bit-serial tree for the exact end-of-buffer path
  std::vector<int> child0, child1, leaf;  // per node
  int root[34] = {};
};
HuffLut* g_lut = nullptr;
std::once_flag g_lut_once;

void build_lut() {
  HuffLut* L = new HuffLut;
  for (int t = 0; t < 34; t++) {
    L->base[t] = -1;
    L->root[t] = -1;
  }
  for (int tree = 0; tree < 34; tree++) {
    bool used = false;
    for (int k = 0; k < HUFF_N_CODES; k++) used |= HUFF_CODES[k].tree == tree;
    if (!used) continue;
    // tree nodes
    const int r = (int)L->child0.size();
    L->root[tree] = r;
    L->child0.push_back(-1);
    L->child1.push_back(-1);
    L->leaf.push_back(-1);
    const int b1 = (int)L->e.size();
    L->base[tree] = b1;
    L->e.resize(b1 + (1 << kL1), 0);
    for (int k = 0; k < HUFF_N_CODES; k++) {
      const huff_code_t& c = HUFF_CODES[k];
      if (c.tree != tree) continue;
      const uint32_t val = (uint32_t)((c.x << 4) | c.y);
      int node = r;
      for (int b = c.len - 1; b >= 0; b--) {
        const int bit = (c.code >> b) & 1;
        int& nx = bit ? L->child1[node] : L->child0[node];
        if (nx < 0) {
          nx = (int)L->child0.size();
          L->child0.push_back(-1);
          L->child1.push_back(-1);
          L->leaf.push_back(-1);
        }
        node = bit ? L->child1[node] : L->child0[node];
      }
      L->leaf[node] = (int)val;
      if (c.len <= kL1) {
        const int shift = kL1 - c.len;
        const uint32_t first = c.code << shift;
        for (uint32_t i = 0; i < (1u << shift); i++) L->e[b1 + first + i] = (uint32_t)c.len | (val << 8);
      } else {
        const uint32_t hi = c.code >> (c.len - kL1);
        if (L->e[b1 + hi] == 0) {  // no second-level block yet (index, not reference: e grows)
          const uint32_t off = (uint32_t)L->e.size();
          L->e.resize(off + (1 << kL2), 0);
          L->e[b1 + hi] = off << 5;
        }
        const uint32_t off = L->e[b1 + hi] >> 5;
        const int rem = c.len - kL1;  // <= 9
        const int shift = kL2 - rem;
        const uint32_t lo = c.code & ((1u << rem) - 1u);
        for (uint32_t i = 0; i < (1u << shift); i++) L->e[off + (lo << shift) + i] = (uint32_t)c.len | (val << 8);
      }
    }
  }
  g_lut = L;
}

// huffman.Decode (huffman/huffman.go:348-419).  Returns false on a decode
// error (cannot happen with the complete Table B.7 codes, kept for parity).
bool huff_decode(Bits& m, int table, int* x, int* y, int* v, int* w) {
  *x = *y = *v = *w = 0;
  const int tree = HUFF_TABLE_TREE[table];
  const int linbits = HUFF_TABLE_LINBITS[table];
  if (tree < 0) return true;  // tables 0, 4, 14 code nothing
  int xy;
  if (m.pos + 19 <= m.nbits()) {
    const uint32_t p = m.peek32();
    uint32_t e = g_lut->e[g_lut->base[tree] + (p >> (32 - kL1))];
    if ((e & 31u) == 0) e = g_lut->e[(e >> 5) + ((p << kL1) >> (32 - kL2))];
    m.pos += e & 31u;
    xy = (int)((e >> 8) & 0xffu);
  } else {  // near the end: exact bit-serial walk (bits past the end read 0)
    int node = g_lut->root[tree], left = 32;
    while (g_lut->leaf[node] < 0) {
      node = m.bit() ? g_lut->child1[node] : g_lut->child0[node];
      if (--left <= 0 || node < 0) return false;
    }
    xy = g_lut->leaf[node];
  }
  *x = (xy >> 4) & 15;
  *y = xy & 15;
  if (table > 31) {  // count1 quadruples
    const int q = *y;
    *v = (q >> 3) & 1;
    *w = (q >> 2) & 1;
    *x = (q >> 1) & 1;
    *y = q & 1;
    if (*v && m.bit() == 1) *v = -*v;
    if (*w && m.bit() == 1) *w = -*w;
    if (*x && m.bit() == 1) *x = -*x;
    if (*y && m.bit() == 1) *y = -*y;
  } else {
    if (linbits && *x == 15) *x += m.bits(linbits);
    if (*x && m.bit() == 1) *x = -*x;
    if (linbits && *y == 15) *y += m.bits(linbits);
    if (*y && m.bit() == 1) *y = -*y;
  }
  return true;
}

// ---- side info (sideinfo.go:33-156) -----------------------------------------
struct SideInfo {
  int main_data_begin;
  int scfsi[2][4];
  int part2_3_length[2][2], big_values[2][2], global_gain[2][2], scalefac_compress[2][2];
  int win_switch_flag[2][2], block_type[2][2], mixed_block_flag[2][2];
  int table_select[2][2][3], subblock_gain[2][2][3];
  int region0_count[2][2], region1_count[2][2];
  int preflag[2][2], scalefac_scale[2][2], count1_table_select[2][2], count1[2][2];
};

St read_side_info(Source& s, uint32_t h, SideInfo* si) {
  static const int kBitsToRead[2][4] = {{9, 5, 3, 4}, {8, 1, 2, 9}};
  const int nch = h_nch(h);
  const int fsize = header_frame_size(h);
  if (fsize < 0 || fsize > 2000) return St::kErr;
  const int size = h_side_info_size(h);
  uint8_t buf[32 + 8] = {};
  bool short_read;
  if (s.read_full(buf, size, &short_read) < size) return short_read ? St::kEof : St::kErr;
  Bits b(buf, size);
  const int lsf = h_lsf(h);
  const int* btr = kBitsToRead[lsf];
  std::memset(si, 0, sizeof *si);
  si->main_data_begin = b.bits(btr[0]);
  (void)b.bits(h_mode(h) == 3 ? btr[1] : btr[2]);  // private bits
  if (!lsf)
    for (int ch = 0; ch < nch; ch++)
      for (int k = 0; k < 4; k++) si->scfsi[ch][k] = b.bits(1);
  for (int gr = 0; gr < header_granules(h); gr++) {
    for (int ch = 0; ch < nch; ch++) {
      si->part2_3_length[gr][ch] = b.bits(12);
      si->big_values[gr][ch] = b.bits(9);
      si->global_gain[gr][ch] = b.bits(8);
      si->scalefac_compress[gr][ch] = b.bits(btr[3]);
      si->win_switch_flag[gr][ch] = b.bits(1);
      if (si->win_switch_flag[gr][ch] == 1) {
        si->block_type[gr][ch] = b.bits(2);
        si->mixed_block_flag[gr][ch] = b.bits(1);
        for (int r = 0; r < 2; r++) si->table_select[gr][ch][r] = b.bits(5);
        for (int w = 0; w < 3; w++) si->subblock_gain[gr][ch][w] = b.bits(3);
        si->region0_count[gr][ch] = (si->block_type[gr][ch] == 2 && si->mixed_block_flag[gr][ch] == 0) ? 8 : 7;
        si->region1_count[gr][ch] = 20 - si->region0_count[gr][ch];
      } else {
        for (int r = 0; r < 3; r++) si->table_select[gr][ch][r] = b.bits(5);
        si->region0_count[gr][ch] = b.bits(4);
        si->region1_count[gr][ch] = b.bits(3);
        si->block_type[gr][ch] = 0;
        if (lsf) si->mixed_block_flag[0][ch] = 0;
      }
      if (!lsf) si->preflag[gr][ch] = b.bits(1);
      si->scalefac_scale[gr][ch] = b.bits(1);
      si->count1_table_select[gr][ch] = b.bits(1);
    }
  }
  return St::kOk;
}

// ---- main data --------------------------------------------------------------
struct MainData {
  int scalefac_l[2][2][22];
  int scalefac_s[2][2][13][3];
};

// readHuffman (maindata/huffman.go:27-138): integers straight into int16 lines.
bool read_huffman(Bits& m, uint32_t h, SideInfo* si, int64_t part2_start, int gr, int ch, int16_t* is) {
  if (si->part2_3_length[gr][ch] == 0) {
    std::memset(is, 0, 576 * sizeof(int16_t));
    si->count1[gr][ch] = 0;  // (the reference leaves Count1 untouched; it is 0 from the side info)
    return true;
  }
  const int64_t bit_pos_end = part2_start + si->part2_3_length[gr][ch] - 1;
  int region1_start, region2_start;
  if (si->win_switch_flag[gr][ch] == 1 && si->block_type[gr][ch] == 2) {
    region1_start = 36;
    region2_start = 576;
  } else {
    const int* l = kSfbLong[h_lsf(h)][h_sfreq(h)];
    const int i = si->region0_count[gr][ch] + 1;
    if (i < 0 || 23 <= i) return false;
    region1_start = l[i];
    const int j = si->region0_count[gr][ch] + si->region1_count[gr][ch] + 2;
    if (j < 0) return false;
    region2_start = j >= 23 ? 576 : l[j];
  }
  const int bv2 = si->big_values[gr][ch] * 2;
  for (int pos = 0; pos < bv2; pos++) {
    if (pos >= 576) return false;
    const int table = pos < region1_start   ? si->table_select[gr][ch][0]
                      : pos < region2_start ? si->table_select[gr][ch][1]
                                            : si->table_select[gr][ch][2];
    int x, y, v, w;
    if (!huff_decode(m, table, &x, &y, &v, &w)) return false;
    is[pos] = (int16_t)x;
    pos++;
    is[pos] = (int16_t)y;  // (pos <= 575: bv2 is even)
  }
  const int table = si->count1_table_select[gr][ch] + 32;
  int pos = bv2;
  while (pos <= 572 && m.pos <= bit_pos_end) {
    int x, y, v, w;
    if (!huff_decode(m, table, &x, &y, &v, &w)) return false;
    is[pos++] = (int16_t)v;
    if (pos >= 576) break;
    is[pos++] = (int16_t)w;
    if (pos >= 576) break;
    is[pos++] = (int16_t)x;
    if (pos >= 576) break;
    is[pos++] = (int16_t)y;
  }
  if (m.pos > bit_pos_end + 1) pos -= 4;
  if (pos < 0) pos = 0;
  si->count1[gr][ch] = pos;
  for (; pos < 576; pos++) is[pos] = 0;
  m.pos = bit_pos_end + 1;
  return true;
}

const int kSlenMpeg1[16][2] = {{0, 0}, {0, 1}, {0, 2}, {0, 3}, {3, 0}, {1, 1}, {1, 2}, {1, 3},
                               {2, 1}, {2, 2}, {2, 3}, {3, 1}, {3, 2}, {3, 3}, {4, 2}, {4, 3}};
// nr_of_sfb per [block kind][row][part] (ISO 13818-3 Table 6, maindata.go:44-50)
const int kNsfbMpeg2[3][6][4] = {
    {{6, 5, 5, 5}, {6, 5, 7, 3}, {11, 10, 0, 0}, {7, 7, 7, 0}, {6, 6, 6, 3}, {8, 8, 5, 0}},
    {{9, 9, 9, 9}, {9, 9, 12, 6}, {18, 18, 0, 0}, {12, 12, 12, 0}, {12, 9, 9, 6}, {15, 12, 9, 0}},
    {{6, 9, 9, 9}, {6, 9, 12, 6}, {15, 18, 0, 0}, {6, 15, 12, 0}, {6, 12, 9, 6}, {6, 18, 9, 0}}};

// packed slen words of scalefac_compress (maindata.go:52-81): 3-bit slen
// fields, row in bits 12..14, preflag in bit 15
struct Slen2 {
  int v[512] = {};
  Slen2() {
    for (int a = 0; a < 4; a++)
      for (int b = 0; b < 3; b++) v[500 + b + 3 * a] = a | (b << 3) | (2 << 12) | (1 << 15);
    for (int a = 0; a < 5; a++)
      for (int b = 0; b < 5; b++)
        for (int c = 0; c < 4; c++)
          for (int d = 0; d < 4; d++) v[d + 4 * c + 16 * b + 80 * a] = a | (b << 3) | (c << 6) | (d << 9);
    for (int a = 0; a < 5; a++)
      for (int b = 0; b < 5; b++)
        for (int c = 0; c < 4; c++) v[400 + c + 4 * b + 20 * a] = a | (b << 3) | (c << 6) | (1 << 12);
  }
};
const Slen2 kSlen2;

// getScaleFactorsMpeg2 (maindata.go:119-188)
St scale_factors_mpeg2(Bits& m, uint32_t h, SideInfo* si, MainData* md, int16_t (*is)[2][576]) {
  const int nch = h_nch(h);
  std::memset(md, 0, sizeof *md);
  for (int ch = 0; ch < nch; ch++) {
    const int64_t part2_start = m.pos;
    int slen = kSlen2.v[si->scalefac_compress[0][ch]];
    si->preflag[0][ch] = (slen >> 15) & 1;
    int blk = 0;
    if (si->block_type[0][ch] == 2) {
      blk++;
      if (si->mixed_block_flag[0][ch] != 0) blk++;
    }
    int sf[64], nsf = 0;
    const int row = (slen >> 12) & 7;
    for (int part = 0; part < 4; part++) {
      const int nbits = slen & 7;
      slen >>= 3;
      for (int k = 0; k < kNsfbMpeg2[blk][row][part]; k++) sf[nsf++] = nbits > 0 ? m.bits(nbits) : 0;
    }
    for (int k = 0; k < (blk << 1) + 1; k++) sf[nsf++] = 0;
    if (nsf == 22) {
      for (int i = 0; i < 22; i++) md->scalefac_l[0][ch][i] = sf[i];
    } else {
      if (nsf < 39) return St::kPanic;  // index out of range in the reference
      for (int x = 0; x < 13; x++)
        for (int w = 0; w < 3; w++) md->scalefac_s[0][ch][x][w] = sf[3 * x + w];
    }
    if (!read_huffman(m, h, si, part2_start, 0, ch, is[0][ch])) return St::kErr;
  }
  return St::kOk;
}

// getScaleFactorsMpeg1 (maindata.go:190-288)
St scale_factors_mpeg1(Bits& m, uint32_t h, SideInfo* si, MainData* md, int16_t (*is)[2][576]) {
  static const int kPartLo[4] = {0, 6, 11, 16}, kPartHi[4] = {6, 11, 16, 21};
  const int nch = h_nch(h);
  std::memset(md, 0, sizeof *md);
  for (int gr = 0; gr < 2; gr++) {
    for (int ch = 0; ch < nch; ch++) {
      const int64_t part2_start = m.pos;
      const int slen1 = kSlenMpeg1[si->scalefac_compress[gr][ch]][0];
      const int slen2 = kSlenMpeg1[si->scalefac_compress[gr][ch]][1];
      if (si->win_switch_flag[gr][ch] == 1 && si->block_type[gr][ch] == 2) {
        if (si->mixed_block_flag[gr][ch] != 0) {
          for (int sfb = 0; sfb < 8; sfb++) md->scalefac_l[gr][ch][sfb] = m.bits(slen1);
          for (int sfb = 3; sfb < 12; sfb++)
            for (int w = 0; w < 3; w++) md->scalefac_s[gr][ch][sfb][w] = m.bits(sfb < 6 ? slen1 : slen2);
        } else {
          for (int sfb = 0; sfb < 12; sfb++)
            for (int w = 0; w < 3; w++) md->scalefac_s[gr][ch][sfb][w] = m.bits(sfb < 6 ? slen1 : slen2);
        }
      } else {
        for (int part = 0; part < 4; part++) {
          const int nb = part < 2 ? slen1 : slen2;
          if (si->scfsi[ch][part] == 0 || gr == 0) {
            for (int sfb = kPartLo[part]; sfb < kPartHi[part]; sfb++) md->scalefac_l[gr][ch][sfb] = m.bits(nb);
          } else if (si->scfsi[ch][part] == 1 && gr == 1) {
            for (int sfb = kPartLo[part]; sfb < kPartHi[part]; sfb++)
              md->scalefac_l[1][ch][sfb] = md->scalefac_l[0][ch][sfb];
          }
        }
      }
      if (!read_huffman(m, h, si, part2_start, gr, ch, is[gr][ch])) return St::kErr;
    }
  }
  return St::kOk;
}

}  // namespace

// ---- source.go ----------------------------------------------------------------
bool Source::fill(int64_t end) {  // reader mode: io.Reader.Read into the window
  if (!may_fetch) {
    starved = true;
    return false;
  }
  // drop what no rollback or read can reach any more
  const int64_t drop = std::min(keep_from, rpos) - base;
  if (drop > 0 && drop >= (int64_t)(win.size() / 2)) {
    win.erase(win.begin(), win.begin() + drop);
    base += drop;
  }
  const int64_t have_end = base + (int64_t)win.size();
  const size_t want = std::max<size_t>(fetch_bytes, end > have_end ? (size_t)(end - have_end) : 0);
  const size_t old = win.size();
  win.resize(old + want);
  const int64_t r = rd->read(rd->user, win.data() + old, want);
  if (r <= 0) {
    win.resize(old);
    if (r < 0) read_failed = true;
    return false;
  }
  win.resize(old + (size_t)std::min<int64_t>(r, (int64_t)want));
  return true;
}

int64_t Source::read_full(uint8_t* buf, int64_t n, bool* short_read) {  // source.go:99-122
  int64_t got = 0;
  *short_read = false;
  if (n_unread > 0) {
    const int64_t k = n < n_unread ? n : n_unread;
    std::memcpy(buf, unread, (size_t)k);
    std::memmove(unread, unread + k, (size_t)(n_unread - k));
    n_unread -= (int)k;
    got = k;
    if (got == n) return got;
  }
  const int64_t want = n - got;
  if (rd) {
    // io.ReadFull on the reader: Read until n bytes, EOF or an error
    while (base + (int64_t)win.size() < rpos + want && fill(rpos + want)) {
    }
    int64_t avail = base + (int64_t)win.size() - rpos;
    if (avail < 0) avail = 0;
    const int64_t k = want < avail ? want : avail;
    if (k > 0) std::memcpy(buf + got, win.data() + (rpos - base), (size_t)k);
    rpos += k;
    pos += k;
    if (k < want) *short_read = true;
    return got + k;
  }
  int64_t avail = len - rpos;
  if (avail < 0) avail = 0;
  const int64_t k = want < avail ? want : avail;
  if (k > 0) std::memcpy(buf + got, data + rpos, (size_t)k);
  rpos += k;
  pos += k;
  if (k < want) *short_read = true;  // io.ReadFull: EOF / ErrUnexpectedEOF
  return got + k;
}

void Source::unread_bytes(const uint8_t* b, int n) {  // source.go:94-97
  std::memmove(unread + n, unread, (size_t)n_unread);
  std::memcpy(unread, b, (size_t)n);
  n_unread += n;
  pos -= n;
}

bool Source::seek(int64_t off, int whence, int64_t* res) {  // source.go:28-40
  if (!seekable) return false;
  if (rd) {
    int64_t a;
    if (whence == 2) {  // the end is the reader's to know
      a = rd->seek(rd->user, off, 2);
      if (a < 0) return false;
      base = a;
      win.clear();
    } else {
      a = whence == 0 ? off : rpos + off;
      if (a < 0) return false;
      if (a < base || a > base + (int64_t)win.size()) {
        a = rd->seek(rd->user, a, 0);
        if (a < 0) return false;
        base = a;
        win.clear();
      }
    }
    n_unread = 0;
    rpos = pos = a;
    if (res) *res = a;
    return true;
  }
  n_unread = 0;
  const int64_t a = whence == 0 ? off : whence == 1 ? rpos + off : len + off;
  if (a < 0) return false;
  rpos = a;
  pos = a;
  if (res) *res = a;
  return true;
}

Source::Mark Source::mark() const {
  Mark m;
  m.rpos = rpos;
  m.pos = pos;
  m.n_unread = n_unread;
  std::memcpy(m.unread, unread, sizeof unread);
  return m;
}

void Source::restore(const Mark& m) {
  rpos = m.rpos;
  pos = m.pos;
  n_unread = m.n_unread;
  std::memcpy(unread, m.unread, sizeof unread);
}

St Source::skip_tags() {  // source.go:42-83
  for (;;) {
    uint8_t b3[3];
    bool sr;
    read_full(b3, 3, &sr);
    if (sr) return St::kEof;
    if (std::memcmp(b3, "TAG", 3) == 0) {
      uint8_t tmp[125];
      read_full(tmp, 125, &sr);
      if (sr) return St::kEof;
    } else if (std::memcmp(b3, "ID3", 3) == 0) {
      uint8_t tmp[4];
      read_full(tmp, 3, &sr);
      if (sr) return St::kEof;
      const int64_t n = read_full(tmp, 4, &sr);
      if (sr) return St::kEof;
      if (n != 4) return St::kOk;
      const int64_t size = ((int64_t)tmp[0] << 21) | ((int64_t)tmp[1] << 14) | ((int64_t)tmp[2] << 7) | tmp[3];
      // skip `size` bytes (io.ReadFull into a scratch buffer)
      if (rd) {
        uint8_t scratch[4096];
        for (int64_t left = size; left > 0;) {
          const int64_t k = left < (int64_t)sizeof scratch ? left : (int64_t)sizeof scratch;
          left -= read_full(scratch, k, &sr);
          if (sr) return St::kEof;
          keep_from = rpos;  // the tag's bytes are never read again
        }
        continue;
      }
      const int64_t avail = n_unread + (len - rpos > 0 ? len - rpos : 0);
      const int64_t k = size < avail ? size : avail;
      int64_t left = k;
      while (left > 0 && n_unread > 0) {
        uint8_t c;
        read_full(&c, 1, &sr);
        left--;
      }
      rpos += left;
      pos += left;
      if (k < size && size > 0) return St::kEof;
    } else {
      unread_bytes(b3, 3);
      return St::kOk;
    }
  }
}

// ---- frameheader.go -------------------------------------------------------------
int header_granules(uint32_t h) { return 2 >> h_lsf(h); }
int header_bytes_per_frame(uint32_t h) { return 576 * header_granules(h) * 4; }
int header_sample_rate(uint32_t h) {  // frameheader.go:304-318
  const int lsf = h_lsf(h);
  switch (h_sfreq(h)) {
    case 0: return 44100 >> lsf;
    case 1: return 48000 >> lsf;
    case 2: return 32000 >> lsf;
  }
  return 0;
}
int header_frame_size(uint32_t h) {  // frameheader.go:223-232
  const int f = header_sample_rate(h);
  if (f == 0) return -1;
  return ((144 * h_bitrate(h)) / f + h_padding(h)) >> h_lsf(h);
}

St read_header(Source& s, int64_t* pos_io, uint32_t* out) {  // frameheader.go:279-328
  uint8_t b[4];
  bool sr;
  if (s.read_full(b, 4, &sr) < 4) return St::kEof;  // EOF / UnexpectedEOF -> EOF
  uint32_t h = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  int64_t searched = 4, position = *pos_io;
  while (!h_valid(h)) {
    if (searched >= 64 * 1024) return St::kEof;  // SyncSearchLimitError -> EOF (decode.go:59-61)
    uint8_t c;
    s.read_full(&c, 1, &sr);
    if (sr) return St::kEof;
    h = (h << 8) | c;
    position++;
    searched++;
  }
  if (h_bitrate_index(h) == 0) return St::kErr;  // free format
  *pos_io = position;
  *out = h;
  return St::kOk;
}

void prescan(const uint8_t* data, size_t len, uint64_t* n_granules, uint64_t* md_bytes) {
  // counted in locals, stored once: callers pass neighbouring elements of one
  // array per stream, and a store per frame from many threads into one cache
  // line serialised the pre-pass (8 threads no faster than 1)
  uint64_t ng = 0, nmd = 0;
  *n_granules = *md_bytes = 0;
  Source src;
  src.data = data;
  src.len = (int64_t)len;
  if (src.skip_tags() != St::kOk) return;
  uint8_t skip[2048];
  for (;;) {  // the checks of FrameScanner::next that need no side info
    uint32_t h;
    int64_t pos = src.pos;
    if (read_header(src, &pos, &h) != St::kOk) break;
    const int crc = h_protection(h) == 0 ? 2 : 0;
    if (h_id(h) == 0 || h_layer(h) != 1) break;
    const int fsize = header_frame_size(h);
    if (fsize < 0 || fsize > 2000) break;
    const int sis = h_side_info_size(h);
    const int size = fsize - sis - 4 - crc;
    if (size > 1500 || size < 0) break;
    bool sr;
    if (src.read_full(skip, crc + sis + size, &sr) < crc + sis + size) break;
    ng += (uint64_t)header_granules(h);
    nmd += (uint64_t)size;
  }
  *n_granules = ng;
  *md_bytes = nmd;
}

// ---- frame.Read (frame.go:67-115) + maindata.Read (maindata.go:85-117, :290-323) ----
St FrameParser::next(Source& s, ParsedFrame* out) {
  std::call_once(g_lut_once, build_lut);
  uint32_t h;
  int64_t pos = s.pos;
  St st = read_header(s, &pos, &h);
  if (st != St::kOk) return st;
  if (h_protection(h) == 0) {
    uint8_t crc[2];
    bool sr;
    if (s.read_full(crc, 2, &sr) < 2) return sr ? St::kEof : St::kErr;
  }
  if (h_id(h) == 0) return St::kErr;     // MPEG 2.5
  if (h_layer(h) != 1) return St::kErr;  // layer III only
  SideInfo si;
  st = read_side_info(s, h, &si);
  if (st != St::kOk) return st;
  const int fsize = header_frame_size(h);
  if (fsize > 2000) return St::kErr;
  int size = fsize - h_side_info_size(h) - 4;
  if (h_protection(h) == 0) size -= 2;
  if (size > 1500) return St::kErr;
  if (size < 0) return St::kPanic;  // make([]byte, <0) panics
  // reservoir: keep main_data_begin bytes of the previous main data (or, on
  // underflow, all of it -- the reference appends without an error)
  const int offset = si.main_data_begin;
  const bool underflow = have_prev_ && offset > (int)prev_md_.size();
  const int64_t keep = !have_prev_ ? 0 : underflow ? (int64_t)prev_md_.size() : offset;
  md_.assign((size_t)(keep + size + 8), 0);  // + zero padding for the bit reader
  if (keep) std::memcpy(md_.data(), prev_md_.data() + (prev_md_.size() - keep), (size_t)keep);
  bool sr;
  if (s.read_full(md_.data() + keep, size, &sr) < size) return sr ? St::kEof : St::kErr;
  const int64_t md_len = keep + size;

  Bits m(md_.data(), md_len);
  MainData md;
  int16_t is[2][2][576];
  st = h_lsf(h) ? scale_factors_mpeg2(m, h, &si, &md, is) : scale_factors_mpeg1(m, h, &si, &md, is);
  if (st != St::kOk) return st;

  // the new frame becomes `prev` (its main-data bytes form the next reservoir)
  prev_md_.assign(md_.begin(), md_.begin() + md_len);
  have_prev_ = true;

  const int ng = header_granules(h), nch = h_nch(h);
  out->header = h;
  out->start = pos;
  out->n_granules = ng;
  for (int gr = 0; gr < ng; gr++) {
    mp3g_granule& G = out->gran[gr];
    std::memset(&G, 0, sizeof G);
    std::memset(out->coef[gr], 0, sizeof out->coef[gr]);
    G.header = h;
    G.gr = (uint32_t)gr;
    for (int ch = 0; ch < nch; ch++) {
      mp3g_channel& c = G.ch[ch];
      c.count1 = (uint16_t)si.count1[gr][ch];
      c.global_gain = (uint8_t)si.global_gain[gr][ch];
      c.scalefac_scale = (uint8_t)si.scalefac_scale[gr][ch];
      c.preflag = (uint8_t)si.preflag[gr][ch];
      c.win_switch_flag = (uint8_t)si.win_switch_flag[gr][ch];
      c.block_type = (uint8_t)si.block_type[gr][ch];
      c.mixed_block_flag = (uint8_t)si.mixed_block_flag[gr][ch];
      for (int w = 0; w < 3; w++) c.subblock_gain[w] = (uint8_t)si.subblock_gain[gr][ch][w];
      for (int k = 0; k < 22; k++) c.scalefac_l[k] = (uint8_t)md.scalefac_l[gr][ch][k];
      for (int k = 0; k < 13; k++)
        for (int w = 0; w < 3; w++) c.scalefac_s[k][w] = (uint8_t)md.scalefac_s[gr][ch][k][w];
      std::memcpy(out->coef[gr] + ch * 576, is[gr][ch], 576 * sizeof(int16_t));
    }
  }
  return St::kOk;
}

// ---- frame.Read without the main-data decode ----------
namespace {

// Bit position after a job's scale factors: the reads of maindata.go:132-279
// in order, each skipped (no advance) when it would pass the end (bits.go:58-68).
int64_t sf_end(int64_t pos, int64_t end, const mp3g_hjob& j) {
  auto rd = [&](int n) {
    if (n > 0 && pos + n <= end) pos += n;
  };
  switch (j.sf_kind) {
    case MP3G_SF_MPEG1_LONG:
      for (int part = 0; part < 4; part++) {
        if ((j.scfsi >> part) & 1) continue;
        for (int k = 0; k < (part == 0 ? 6 : 5); k++) rd(part < 2 ? j.slen[0] : j.slen[1]);
      }
      break;
    case MP3G_SF_MPEG1_SHORT:
    case MP3G_SF_MPEG1_MIXED:
      if (j.sf_kind == MP3G_SF_MPEG1_MIXED)
        for (int sfb = 0; sfb < 8; sfb++) rd(j.slen[0]);
      for (int sfb = j.sf_kind == MP3G_SF_MPEG1_MIXED ? 3 : 0; sfb < 12; sfb++)
        for (int w = 0; w < 3; w++) rd(sfb < 6 ? j.slen[0] : j.slen[1]);
      break;
    case MP3G_SF_MPEG2_LONG:
    case MP3G_SF_MPEG2_SHORT:
      for (int part = 0; part < 4; part++)
        for (int k = 0; k < j.nsf[part]; k++) rd(j.slen[part]);
      break;
  }
  return pos;
}

}  // namespace

namespace {
// appends to the main-data sinks (n bytes in use afterwards)
bool md_resize(std::vector<uint8_t>* v, size_t n) {
  v->resize(n);
  return true;
}
bool md_resize(RawMd* r, size_t n) {
  if (n > r->cap) {
    r->overflow = true;
    return false;
  }
  r->n = n;
  return true;
}
}  // namespace

St FrameScanner::next(Source& s, ScannedFrame* out, std::vector<uint8_t>* md) { return next_impl(s, out, md); }
St FrameScanner::next(Source& s, ScannedFrame* out, RawMd* md) { return next_impl(s, out, md); }

template <class Md>
St FrameScanner::next_impl(Source& s, ScannedFrame* out, Md* md) {
  // header, CRC, side info and sizes exactly as FrameParser::next
  uint32_t h;
  int64_t pos = s.pos;
  St st = read_header(s, &pos, &h);
  if (st != St::kOk) return st;
  if (h_protection(h) == 0) {
    uint8_t crc[2];
    bool sr;
    if (s.read_full(crc, 2, &sr) < 2) return sr ? St::kEof : St::kErr;
  }
  if (h_id(h) == 0) return St::kErr;
  if (h_layer(h) != 1) return St::kErr;
  SideInfo si;
  st = read_side_info(s, h, &si);
  if (st != St::kOk) return st;
  const int fsize = header_frame_size(h);
  if (fsize > 2000) return St::kErr;
  int size = fsize - h_side_info_size(h) - 4;
  if (h_protection(h) == 0) size -= 2;
  if (size > 1500) return St::kErr;
  if (size < 0) return St::kPanic;

  // reservoir (maindata.go:290-323): the frame's bit buffer is the suffix of
  // the main-data concatenation starting at `vstart` -- the tail of the
  // previous buffer, all of it on an underflow, nothing without a previous
  // frame.  (An underflow needs main_data_begin > the previous buffer, and
  // main_data_begin < 512, so a bit buffer never exceeds ~2 KB.)
  const int64_t g0 = (int64_t)md->size();
  const int offset = si.main_data_begin;
  const bool underflow = have_prev_ && offset > g0 - prev_start_;
  const int64_t vstart = !have_prev_ ? g0 : underflow ? prev_start_ : g0 - offset;
  if (!md_resize(md, (size_t)(g0 + size))) return St::kErr;
  bool sr;
  if (s.read_full(md->data() + g0, size, &sr) < size) {
    md_resize(md, (size_t)g0);
    return sr ? St::kEof : St::kErr;
  }
  const int64_t end = (int64_t)md->size() * 8;

  const int lsf = h_lsf(h), nch = h_nch(h), ng = header_granules(h);
  out->header = h;
  out->start = pos;
  out->n_granules = ng;
  std::memset(out->gran, 0, sizeof out->gran);
  std::memset(out->job, 0, sizeof out->job);
  int64_t bit = vstart * 8;  // m.BitPos() as an absolute position
  for (int gr = 0; gr < ng; gr++) {
    mp3g_granule& G = out->gran[gr];
    G.header = h;
    G.gr = (uint32_t)gr;
    for (int ch = 0; ch < nch; ch++) {
      mp3g_channel& c = G.ch[ch];
      c.global_gain = (uint8_t)si.global_gain[gr][ch];
      c.scalefac_scale = (uint8_t)si.scalefac_scale[gr][ch];
      c.preflag = (uint8_t)si.preflag[gr][ch];
      c.win_switch_flag = (uint8_t)si.win_switch_flag[gr][ch];
      c.block_type = (uint8_t)si.block_type[gr][ch];
      c.mixed_block_flag = (uint8_t)si.mixed_block_flag[gr][ch];
      for (int w = 0; w < 3; w++) c.subblock_gain[w] = (uint8_t)si.subblock_gain[gr][ch][w];

      mp3g_hjob& J = out->job[gr][ch];
      J.part2_start = (uint64_t)bit;
      J.bit_end = (uint64_t)end;
      J.part2_3_length = (uint16_t)si.part2_3_length[gr][ch];
      J.big_values = (uint16_t)si.big_values[gr][ch];
      for (int r = 0; r < 3; r++) J.table_select[r] = (uint8_t)si.table_select[gr][ch][r];
      J.count1_table = (uint8_t)si.count1_table_select[gr][ch];
      // region boundaries (maindata/huffman.go:39-64)
      const bool shortblk = si.win_switch_flag[gr][ch] == 1 && si.block_type[gr][ch] == 2;
      if (shortblk) {
        J.region1_start = 36;
        J.region2_start = 576;
      } else {
        const int* l = kSfbLong[lsf][h_sfreq(h)];
        J.region1_start = (uint16_t)l[si.region0_count[gr][ch] + 1];  // index <= 16 < 23
        const int j = si.region0_count[gr][ch] + si.region1_count[gr][ch] + 2;
        J.region2_start = (uint16_t)(j >= 23 ? 576 : l[j]);
      }
      if (lsf) {  // getScaleFactorsMpeg2 (maindata.go:132-179)
        int slen = kSlen2.v[si.scalefac_compress[0][ch]];
        c.preflag = (uint8_t)((slen >> 15) & 1);
        int blk = 0;
        if (si.block_type[0][ch] == 2) blk = si.mixed_block_flag[0][ch] != 0 ? 2 : 1;
        if (blk == 2) return St::kPanic;  // 38 scale factors: index out of range in the reference
        const int row = (slen >> 12) & 7;
        for (int part = 0; part < 4; part++) {
          J.slen[part] = (uint8_t)(slen & 7);
          slen >>= 3;
          J.nsf[part] = (uint8_t)kNsfbMpeg2[blk][row][part];
        }
        J.sf_kind = blk ? MP3G_SF_MPEG2_SHORT : MP3G_SF_MPEG2_LONG;
      } else {  // getScaleFactorsMpeg1 (maindata.go:190-279)
        J.slen[0] = (uint8_t)kSlenMpeg1[si.scalefac_compress[gr][ch]][0];
        J.slen[1] = (uint8_t)kSlenMpeg1[si.scalefac_compress[gr][ch]][1];
        J.sf_kind = !shortblk                            ? MP3G_SF_MPEG1_LONG
                    : si.mixed_block_flag[gr][ch] != 0 ? MP3G_SF_MPEG1_MIXED
                                                       : MP3G_SF_MPEG1_SHORT;
        if (gr == 1 && J.sf_kind == MP3G_SF_MPEG1_LONG) {
          for (int part = 0; part < 4; part++) J.scfsi |= (uint8_t)((si.scfsi[ch][part] == 1) << part);
          if (J.scfsi) {
            const mp3g_hjob& J0 = out->job[0][ch];
            J.scf0_delta = (uint32_t)(J.part2_start - J0.part2_start);
            J.sf0_kind = J0.sf_kind;
            J.sf0_slen[0] = J0.slen[0];
            J.sf0_slen[1] = J0.slen[1];
          }
        }
      }
      const int64_t after_sf = sf_end(bit, end, J);
      if (J.part2_3_length == 0) {
        bit = after_sf;  // readHuffman returns before m.SetPos (maindata/huffman.go:29-34)
      } else {
        if (J.big_values > 288) return St::kErr;  // "isPos was too big" (maindata/huffman.go:67-70)
        bit += J.part2_3_length;                   // m.SetPos(bitPosEnd + 1)
      }
    }
  }
  prev_start_ = vstart;
  have_prev_ = true;
  return St::kOk;
}

// ---- the decoder's read-ahead step (decode.go:45-67 repeated) -----------------
namespace {
template <class Next, class Emit>
St scan_frames(Source& src, size_t max_frames, bool must, Next next, Emit emit) {
  const bool eager = !src.rd || src.seekable;
  St st = St::kOk;
  for (size_t i = 0; i < max_frames; i++) {
    src.may_fetch = eager || (must && i == 0);
    src.starved = false;
    src.keep_from = src.rpos;
    const Source::Mark m = src.mark();
    st = next();
    if (st != St::kOk) {
      if (src.starved) {  // not all of it has arrived: leave it for a later call
        src.restore(m);
        st = St::kOk;
      } else if (src.read_failed) {
        st = St::kRead;
      }
      break;
    }
    emit();
  }
  src.may_fetch = true;
  src.starved = false;
  src.read_failed = false;
  return st;
}
}  // namespace

St scan_some(Source& src, FrameScanner& sc, std::vector<uint8_t>* md, size_t max_frames, bool must,
             void (*emit)(void* ctx, const ScannedFrame& f, int64_t src_pos), void* ctx) {
  ScannedFrame f;
  return scan_frames(
      src, max_frames, must, [&] { return sc.next(src, &f, md); }, [&] { emit(ctx, f, src.pos); });
}

St parse_some(Source& src, FrameParser& fp, size_t max_frames, bool must,
              void (*emit)(void* ctx, const ParsedFrame& f, int64_t src_pos), void* ctx) {
  ParsedFrame f;
  return scan_frames(
      src, max_frames, must, [&] { return fp.next(src, &f); }, [&] { emit(ctx, f, src.pos); });
}

}  // namespace host
}  // namespace mp3g
