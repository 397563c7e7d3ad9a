// huff_lut.h -- Huffman lookup tables of the device main-data decoder
// (huffman_dev.hip), built on the host from the ISO 11172-3 Table B.7
// codeword lists (huffman_codes.inc; table directory of reference
// internal/huffman/huffman.go:311-346) and uploaded once per device.
//
// Every tree is a multi-level table of 16-bit entries: the root block is
// indexed by the next w0 bits of the stream (w0 = min(longest codeword,
// kHuffRootBits)), each deeper block by the next w bits (w = min(remaining
// length, 6)).
//   leaf : bit 15 = 0, bits 8..12 = codeword length, bits 4..7 = a, 0..3 = b,
//          bit 13 = c, bit 14 = d.  Big-value trees: (a, b) = (x, y), c = d =
//          0; count1 trees 32/33: (a, b, c, d) = (v, w, x, y).  The decoder
//          then reads, for a, b, c, d in turn, the linbits of a 15 and the
//          sign of a non-zero value: one code path for both regions.
//   link : bit 15 = 1, bits 12..14 = width of the next block, bits 0..11 =
//          its first entry, counted from the tree's root block, / 2 (blocks
//          are >= 2 entries, so offsets are even)
// The builder checks that every entry is filled (the trees are complete
// prefix codes), so a lookup cannot fail: huffman.Decode's error return
// (huffman.go:382-386) is unreachable for bitstream input, as for the host
// parse (host_parse.cpp).
#pragma once
#include <cstdint>

namespace mp3g {

#ifndef MP3G_HUFF_ROOT_BITS
#define MP3G_HUFF_ROOT_BITS 8
#endif
constexpr int kHuffRootBits = MP3G_HUFF_ROOT_BITS;
static_assert(kHuffRootBits >= 6 && kHuffRootBits <= 11, "root block width");
// entries used (+ 2 for the null tree): root 8: 4,506 (9 KB of LDS), 9: 6,722,
// 10: 11,022, 11: 17,972
constexpr int kHuffMaxEntries = kHuffRootBits <= 8 ? 4608 : kHuffRootBits == 9 ? 6784 : kHuffRootBits == 10 ? 11072 : 18048;
struct HuffLut {
  // per table 0..33: root block offset | w0 << 24.  Tables that code
  // nothing (0, 4, 14: huffman.go:354-356) share a block of zero-length
  // x = y = 0 leaves.
  uint32_t root[34];
  uint32_t linbits[34];
  uint32_t n_entries;
  uint32_t pad[3];
  uint16_t e[kHuffMaxEntries];
};

// Builds the tables; returns false if they do not fit or a tree is incomplete.
bool build_huff_lut(HuffLut* t);

}  // namespace mp3g
