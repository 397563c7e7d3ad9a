// huff_lut.cpp -- builds the device Huffman tables (see huff_lut.h).
#include "huff_lut.h"

#include <cstring>
#include <vector>

namespace mp3g {
namespace {

#include "huffman_codes.inc"  // ISO 11172-3 Table B.7 codeword lists (data)

struct Code {
  uint32_t code;
  int len;
  uint32_t val;  // the leaf's value bits (huff_lut.h)
};

struct Builder {
  HuffLut* t;
  uint32_t n = 0;
  bool ok = true;
  uint32_t tree_base = 0;  // the current tree's root block (links count from it)

  // Block for the codes `cs`, which share their first `depth` bits; returns
  // the block's offset and its width in *w_out.
  uint32_t block(const std::vector<Code>& cs, int depth, int wmax, int* w_out) {
    int maxlen = 0;
    for (const Code& c : cs) maxlen = c.len > maxlen ? c.len : maxlen;
    const int w = maxlen - depth < wmax ? maxlen - depth : wmax;
    *w_out = w;
    const uint32_t off = n;
    n += 1u << w;
    if (n > (uint32_t)kHuffMaxEntries) {
      ok = false;
      return 0;
    }
    std::vector<std::vector<Code>> sub(1u << w);
    for (const Code& c : cs) {
      const int rem = c.len - depth;
      const uint32_t bits = c.code & ((1u << rem) - 1u);  // the code's bits after `depth`
      if (rem <= w) {
        const uint32_t first = bits << (w - rem);
        for (uint32_t i = 0; i < (1u << (w - rem)); i++) t->e[off + first + i] = (uint16_t)(((uint32_t)c.len << 8) | c.val);
      } else {
        sub[bits >> (rem - w)].push_back(c);
      }
    }
    for (uint32_t i = 0; i < (1u << w); i++) {
      if (sub[i].empty()) continue;
      int cw = 0;
      const uint32_t child = block(sub[i], depth + w, 6, &cw);
      if (!ok) return 0;
      const uint32_t rel = child - tree_base;
      if ((rel & 1u) || (rel >> 1) > 0xfffu) {
        ok = false;
        return 0;
      }
      t->e[off + i] = (uint16_t)(0x8000u | ((uint32_t)cw << 12) | (rel >> 1));
    }
    return off;
  }
};

}  // namespace

bool build_huff_lut(HuffLut* t) {
  std::memset(t, 0, sizeof *t);
  Builder b{t};
  uint32_t tree_root[34] = {};
  bool have[34] = {};
  for (int tree = 0; tree < 34; tree++) {
    std::vector<Code> cs;
    for (int k = 0; k < HUFF_N_CODES; k++)
      if (HUFF_CODES[k].tree == tree) {
        const uint32_t x = HUFF_CODES[k].x, y = HUFF_CODES[k].y;
        // count1 trees code vwxy in y: a = v, b = w, c = x, d = y
        const uint32_t val = tree >= 32 ? ((y >> 3) & 1u) << 4 | ((y >> 2) & 1u) | ((y >> 1) & 1u) << 13 |
                                              (y & 1u) << 14
                                        : x << 4 | y;
        cs.push_back({HUFF_CODES[k].code, HUFF_CODES[k].len, val});
      }
    if (cs.empty()) continue;
    int w0 = 0;
    b.tree_base = b.n;
    const uint32_t off = b.block(cs, 0, kHuffRootBits, &w0);
    if (!b.ok) return false;
    tree_root[tree] = off | ((uint32_t)w0 << 24);  // w0 >= 1: never 0
    have[tree] = true;
  }
  // complete prefix codes: every entry is a leaf (len >= 1) or a link
  for (uint32_t i = 0; i < b.n; i++)
    if (t->e[i] == 0) return false;
  // tables that code nothing (0, 4, 14) point at a 1-bit block of two
  // zero-length x = y = 0 leaves: decoding them reads nothing, branch-free
  if (b.n + 2 > (uint32_t)kHuffMaxEntries) return false;
  const uint32_t null_root = b.n | (1u << 24);
  t->e[b.n] = t->e[b.n + 1] = 0;
  b.n += 2;
  for (int table = 0; table < 34; table++) {
    const int tree = HUFF_TABLE_TREE[table];
    t->root[table] = tree >= 0 && have[tree] ? tree_root[tree] : null_root;
    t->linbits[table] = (uint32_t)HUFF_TABLE_LINBITS[table];
  }
  t->n_entries = b.n;
  return true;
}

}  // namespace mp3g
