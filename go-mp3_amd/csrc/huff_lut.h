// huff_lut.h -- Huffman lookup tables of the device main-data decoder
// (huffman_dev.hip), built on the host from the ISO 11172-3 Table B.7
// codeword lists (huffman_codes.inc; table directory of reference
// internal/huffman/huffman.go:311-346) and uploaded once per device.
//
// Every tree is a multi-level table of 32-bit entries: the root block is
// indexed by the next w0 bits of the stream (w0 = min(longest codeword, 8)),
// each deeper block by the next w bits (w = min(remaining length, 6)).
//   leaf : bit 31 = 0, bits 8..12 = codeword length, bits 0..7 = x << 4 | y
//          (count1 trees 32/33: x = 0, y = vwxy)
//   link : bit 31 = 1, bits 24..27 = width of the next block, bits 0..23 =
//          its first entry
// The builder checks that every entry is filled (the trees are complete
// prefix codes), so a lookup cannot fail: huffman.Decode's error return
// (huffman.go:382-386) is unreachable for bitstream input, as for the host
// parse (host_parse.cpp).
#pragma once
#include <cstdint>

namespace mp3g {

constexpr int kHuffMaxEntries = 4608;  // 4,504 used (18 KB of LDS)
struct HuffLut {
  // per table 0..33: root block offset | w0 << 24; 0 = the table codes
  // nothing (tables 0, 4, 14: huffman.go:354-356)
  uint32_t root[34];
  uint32_t linbits[34];
  uint32_t n_entries;
  uint32_t pad[3];
  uint32_t e[kHuffMaxEntries];
};

// Builds the tables; returns false if they do not fit or a tree is incomplete.
bool build_huff_lut(HuffLut* t);

}  // namespace mp3g
