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
  uint32_t val;  // x << 4 | y
};

struct Builder {
  HuffLut* t;
  uint32_t n = 0;
  bool ok = true;

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
        for (uint32_t i = 0; i < (1u << (w - rem)); i++) t->e[off + first + i] = ((uint32_t)c.len << 8) | c.val;
      } else {
        sub[bits >> (rem - w)].push_back(c);
      }
    }
    for (uint32_t i = 0; i < (1u << w); i++) {
      if (sub[i].empty()) continue;
      int cw = 0;
      const uint32_t child = block(sub[i], depth + w, 6, &cw);
      if (!ok) return 0;
      t->e[off + i] = 0x80000000u | ((uint32_t)cw << 24) | child;
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
      if (HUFF_CODES[k].tree == tree)
        cs.push_back({HUFF_CODES[k].code, HUFF_CODES[k].len, (uint32_t)((HUFF_CODES[k].x << 4) | HUFF_CODES[k].y)});
    if (cs.empty()) continue;
    int w0 = 0;
    const uint32_t off = b.block(cs, 0, 8, &w0);
    if (!b.ok) return false;
    tree_root[tree] = off | ((uint32_t)w0 << 24);  // w0 >= 1: never 0
    have[tree] = true;
  }
  // complete prefix codes: every entry is a leaf (len >= 1) or a link
  for (uint32_t i = 0; i < b.n; i++)
    if (t->e[i] == 0) return false;
  for (int table = 0; table < 34; table++) {
    const int tree = HUFF_TABLE_TREE[table];
    t->root[table] = tree >= 0 && have[tree] ? tree_root[tree] : 0u;
    t->linbits[table] = (uint32_t)HUFF_TABLE_LINBITS[table];
  }
  t->n_entries = b.n;
  return true;
}

}  // namespace mp3g
