// huffman_job.h -- one (granule, channel) job of the GPU main-data decode
// (huffman_dev.hip): scale factors (maindata.go:119-288)
// and Huffman codes (maindata/huffman.go:27-138, huffman/huffman.go:348-419)
// of one channel, read straight out of the concatenated main-data buffer.
//
// Bit semantics are the reference's bits.Bits (bits.go:45-77): a read that
// would pass the end of the frame's main-data buffer returns 0 and does not
// advance.  The 64-bit window is masked with zeros from bit_end on, and every
// advance is clamped exactly as the reference's bit-by-bit tree walk and
// Bit()/Bits() calls advance.
//
// __host__ __device__: the kernel runs it per lane; tests/hjob_host.hip
// compiles the same code for the CPU to check the job decomposition against
// the host parse without a GPU (test infrastructure, not a product path).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/mp3g.h"
#include "huff_lut.h"

#define MP3G_HD_INLINE __host__ __device__ __forceinline__

namespace mp3g {
namespace huff {

MP3G_HD_INLINE uint64_t bswap64(uint64_t v) { return __builtin_bswap64(v); }

// Big-endian reader over the main-data buffer, 64 bits at a time.  `w` is
// the job's word 0 (bit `base` of the concatenated main data, a multiple of
// 64); only words [0, nw) are loaded, others read as 0.  kSwap: the words
// are stored in stream byte order (global memory) and swapped on load; the
// LDS staging copy (huffman_dev.hip) is swapped once when it is filled.
// Bits past `end` are only masked where a read could reach them (the slow
// paths); the fast paths first check that they stay below `end`.
template <bool kSwap>
struct Reader {
  const uint64_t* w;
  uint32_t nw;
  uint32_t end;   // bit_end - base (0 if the job starts past its buffer)
  uint32_t wpos;  // bit offset of win's MSB (multiple of 64)
  uint32_t pos;
  uint64_t win;   // bits [wpos, wpos + 64)
  uint64_t nxt;   // bits [wpos + 64, wpos + 128)
  uint64_t nn;    // the stored word of bits [wpos + 128, wpos + 192), in flight

  // kSwap (memory): nothing at or past word nw is loaded.  LDS staging: the
  // buffer holds 3 words past nw (huffman_dev.hip) and bits past `end` never
  // reach a result, so the load is unconditional, only clamped to the buffer
  // (a corrupt stream's part 2 may start past its end).
  MP3G_HD_INLINE uint64_t load(uint32_t k) const {
    return kSwap ? (k < nw ? w[k] : 0ull) : w[k < nw + 3u ? k : nw + 3u];
  }
  MP3G_HD_INLINE static uint64_t order(uint64_t raw) { return kSwap ? bswap64(raw) : raw; }
  MP3G_HD_INLINE void seek(uint32_t p) {
    pos = p;
    wpos = p & ~63u;
    win = order(load(wpos >> 6));
    nxt = order(load((wpos >> 6) + 1));
    nn = load((wpos >> 6) + 2);
  }
  // restores pos - wpos < 64 after at most 64 bits were consumed since the
  // last call.  The next word is loaded two words ahead, so its latency
  // overlaps ~64 bits of decoding.
  MP3G_HD_INLINE void refill() {
    if (kSwap) {
      if (pos - wpos >= 64u) {
        win = nxt;
        nxt = order(nn);
        wpos += 64;
        nn = load((wpos >> 6) + 2);
      }
    } else {  // LDS: branch-free, the next word is read every time
      const bool adv = pos - wpos >= 64u;
      const uint64_t n3 = load((wpos >> 6) + 3);
      win = adv ? nxt : win;
      nxt = adv ? nn : nxt;
      nn = adv ? n3 : nn;
      wpos += adv ? 64u : 0u;
    }
  }
  // the 64 stream bits from pos (not masked at the end)
  MP3G_HD_INLINE uint64_t peek64() const {
    const uint32_t sh = pos - wpos;
    return (win << sh) | ((nxt >> 1) >> (63u - sh));
  }
  // the same with zeros from `end` on (bits.Bit past the end, bits.go:45-56)
  MP3G_HD_INLINE uint64_t peek64m() const {
    const uint32_t left = end > pos ? end - pos : 0u;
    const uint64_t v = peek64();
    return left >= 64u ? v : v & ~(~0ull >> left);
  }
  // bits.Bits(n), 1 <= n <= 13: 0 and no advance if it would pass the end
  MP3G_HD_INLINE uint32_t bits(int n) {
    refill();
    if (pos + (uint32_t)n > end) return 0u;
    const uint32_t v = (uint32_t)(peek64() >> (64 - n));
    pos += (uint32_t)n;
    return v;
  }
  // bits.Bit()
  MP3G_HD_INLINE uint32_t bit() {
    refill();
    if (pos >= end) return 0u;
    const uint32_t v = (uint32_t)(peek64() >> 63);
    pos++;
    return v;
  }
};

// The leaf the 32 stream bits `p` reach in the table at `root` (huff_lut.h);
// *len = its codeword length.
MP3G_HD_INLINE uint32_t lut_leaf(const uint16_t* T, uint32_t root, uint32_t p, uint32_t* len) {
  int used = (int)(root >> 24);
  const uint32_t base = root & 0xffffffu;
  uint32_t e = T[base + (p >> (32 - used))];
  while (e & 0x8000u) {
    const int wd = (int)((e >> 12) & 7u);
    e = T[base + ((e & 0xfffu) << 1) + ((p << used) >> (32 - wd))];
    used += wd;
  }
  *len = (e >> 8) & 31u;
  return e;
}

// huffman.Decode's tree walk near the end of the buffer: the leaf the next
// bits reach (zeros past the end) and the advance of its Bit() calls,
// min(len, end - pos).
template <bool kSwap>
MP3G_HD_INLINE uint32_t decode_xy(Reader<kSwap>& r, const uint16_t* T, uint32_t root) {
  r.refill();
  uint32_t len;
  const uint32_t e = lut_leaf(T, root, (uint32_t)(r.peek64m() >> 32), &len);
  if (r.pos < r.end) r.pos = r.pos + len < r.end ? r.pos + len : r.end;
  return e;
}

// One symbol: a big-values pair (maindata/huffman.go:66-104: codeword, x
// linbits, x sign, y linbits, y sign) or a count1 quad (huffman.go:106-131:
// codeword, v w x y signs), in one code path (lb = 0 for quads, c = d = 0 for
// pairs: huff_lut.h).  Far from the end (<= 19 + 2 * 14 = 47 bits to go)
// every field comes out of one 64-bit peek; otherwise each read follows the
// reference's clamping.
// kQuad = false: a big-values pair (c = d = 0 at compile time: no quad sign
// work in the pair loop, c3 -1 %); kQuad = true: a count1 quad (lb = 0).
template <bool kSwap, bool kQuad>
MP3G_HD_INLINE void decode_sym(Reader<kSwap>& r, const uint16_t* T, uint32_t root, uint32_t lb, int& ao, int& bo,
                               int& co, int& dox) {
  r.refill();
  int a, b, c, d;
  if (r.pos + 47u <= r.end) {
    const uint64_t p64 = r.peek64();
    uint32_t len;
    const uint32_t e = lut_leaf(T, root, (uint32_t)(p64 >> 32), &len);
    const int a0 = (int)((e >> 4) & 15u), b0 = (int)(e & 15u);
    c = kQuad ? (int)((e >> 13) & 1u) : 0;
    d = kQuad ? (int)((e >> 14) & 1u) : 0;
    // The symbol's length comes from the leaf alone (linbits of a 15, one
    // sign bit per non-zero value): the next symbol's position does not wait
    // for the values below, which only feed the stores.
    const uint32_t na = a0 == 15 ? lb : 0u, nb = b0 == 15 ? lb : 0u;
    const uint32_t sa = a0 ? 1u : 0u, sb = b0 ? 1u : 0u;
    r.pos += len + na + sa + nb + sb + (uint32_t)(c + d);
    uint32_t q = (uint32_t)((p64 << len) >> 32);  // the <= 28 bits after the codeword
    a = a0 + (int)((q >> 1) >> (31u - na));
    const bool nega = (q << na) & (sa << 31);
    q <<= na + sa;
    b = b0 + (int)((q >> 1) >> (31u - nb));
    const bool negb = (q << nb) & (sb << 31);
    q <<= nb + sb;
    // c, d: quads only (0 / 1, no linbits)
    const bool negc = c && (q >> 31);
    q <<= (uint32_t)c;
    const bool negd = d && (q >> 31);
    a = nega ? -a : a;
    b = negb ? -b : b;
    c = negc ? -c : c;
    d = negd ? -d : d;
  } else {
    const uint32_t e = decode_xy(r, T, root);
    a = (int)((e >> 4) & 15u);
    b = (int)(e & 15u);
    c = kQuad ? (int)((e >> 13) & 1u) : 0;
    d = kQuad ? (int)((e >> 14) & 1u) : 0;
    if (lb && a == 15) a += (int)r.bits((int)lb);
    if (a && r.bit()) a = -a;
    if (lb && b == 15) b += (int)r.bits((int)lb);
    if (b && r.bit()) b = -b;
    if (c && r.bit()) c = -c;
    if (d && r.bit()) d = -d;
  }
  ao = a;
  bo = b;
  co = c;
  dox = d;
}

// Staging of consecutive line pairs into whole blocks of kBlk lines
// (lines are produced strictly in order from 0, two at a time).  A block is
// written by back-to-back 16-B stores of one lane: with 32-B blocks (the
// default) every 32-B sector of the row is complete when it reaches the L2,
// where 16-B blocks left half sectors that were written back to HBM as 32-B
// requests twice (c3 write traffic 1.66x the coefficient bytes).
#ifndef MP3G_HUFF_BLOCK_LINES
#define MP3G_HUFF_BLOCK_LINES 16
#endif
constexpr int kBlk = MP3G_HUFF_BLOCK_LINES;  // 8, 16 or 32
static_assert(kBlk == 8 || kBlk == 16 || kBlk == 32, "writer block");
struct LineWriter {
  int16_t* row;
  uint32_t b[kBlk / 2];
  MP3G_HD_INLINE void flush(int first) const {
    uint4* d = reinterpret_cast<uint4*>(row + first);
#pragma unroll
    for (int q = 0; q < kBlk / 8; q++) d[q] = make_uint4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
  }
  MP3G_HD_INLINE void put(int i, int x, int y) {
    const uint32_t v = (uint32_t)(uint16_t)(int16_t)x | ((uint32_t)(uint16_t)(int16_t)y << 16);
    const int slot = (i >> 1) & (kBlk / 2 - 1);
#pragma unroll
    for (int q = 0; q < kBlk / 2; q++) b[q] = slot == q ? v : b[q];
    if (slot == kBlk / 2 - 1) {
      flush(i & ~(kBlk - 1));
#pragma unroll
      for (int q = 0; q < kBlk / 2; q++) b[q] = 0u;
    }
  }
  // flushes the pending block (lines up to i, i even, then zeros to the end
  // of the block); returns the first line after it: the first line of the
  // row left for the zero fill (a multiple of 8)
  MP3G_HD_INLINE int finish(int i) {
    if (i & (kBlk - 1)) flush(i & ~(kBlk - 1));
    return (i + kBlk - 1) & ~(kBlk - 1);
  }
};

// lines [z, 576) of a row = 0 (z a multiple of 8): one lane's own stores,
// for the host build; the kernel zero-fills a wave's rows together
// (huffman_dev.hip), so the tail of a job is not 72 scattered stores
MP3G_HD_INLINE void zero_fill_row(int16_t* row, int z) {
  for (int k = z; k < MP3G_LINES; k += 8) *reinterpret_cast<uint4*>(row + k) = make_uint4(0u, 0u, 0u, 0u);
}

// MPEG-1 scale factors of a channel, collected in registers: bytes [8, 72)
// of the mp3g_channel (scalefac_l from byte 11, scalefac_s from byte 33) as
// 16 dwords, written with 6 vector stores instead of up to 61 scattered byte
// stores.  Every factor is put at most once, into a zeroed byte, and the
// indices are compile-time constants once the loops are unrolled.
struct SfRegs {
  uint32_t r[16] = {};
  MP3G_HD_INLINE void put_l(int k, uint32_t v) { r[(3 + k) >> 2] |= v << (8 * ((3 + k) & 3)); }
  MP3G_HD_INLINE void put_s(int k, uint32_t v) { r[(25 + k) >> 2] |= v << (8 * ((25 + k) & 3)); }
  // channel bytes [11, 72) (bytes 8..10, subblock_gain, belong to the scan);
  // ch selects the alignment of the channel inside its 160-byte granule
  MP3G_HD_INLINE void store(mp3g_channel& C, int ch) const {
    uint8_t* cb = reinterpret_cast<uint8_t*>(&C);
    cb[11] = (uint8_t)(r[0] >> 24);
    *reinterpret_cast<uint32_t*>(cb + 12) = r[1];
    if (ch == 0) {  // cb = granule + 8
      *reinterpret_cast<uint2*>(cb + 16) = make_uint2(r[2], r[3]);
      *reinterpret_cast<uint4*>(cb + 24) = make_uint4(r[4], r[5], r[6], r[7]);
      *reinterpret_cast<uint4*>(cb + 40) = make_uint4(r[8], r[9], r[10], r[11]);
      *reinterpret_cast<uint4*>(cb + 56) = make_uint4(r[12], r[13], r[14], r[15]);
    } else {  // cb = granule + 80
      *reinterpret_cast<uint4*>(cb + 16) = make_uint4(r[2], r[3], r[4], r[5]);
      *reinterpret_cast<uint4*>(cb + 32) = make_uint4(r[6], r[7], r[8], r[9]);
      *reinterpret_cast<uint4*>(cb + 48) = make_uint4(r[10], r[11], r[12], r[13]);
      *reinterpret_cast<uint2*>(cb + 64) = make_uint2(r[14], r[15]);
    }
  }
};
static_assert(offsetof(mp3g_channel, scalefac_l) == 11 && offsetof(mp3g_channel, scalefac_s) == 33 &&
                  offsetof(mp3g_granule, ch) == 8 && sizeof(mp3g_channel) == 72,
              "SfRegs byte layout");

// MPEG-1 long-block scale factors (maindata.go:233-279): parts in `read` are
// read from the stream, parts in `store` are kept.
template <bool kSwap>
MP3G_HD_INLINE void sf_mpeg1_long(Reader<kSwap>& r, int slen1, int slen2, uint32_t read, uint32_t store,
                                              SfRegs& sf) {
#pragma unroll
  for (int part = 0; part < 4; part++) {
    if (!((read >> part) & 1u)) continue;
    const int lo = part == 0 ? 0 : part == 1 ? 6 : part == 2 ? 11 : 16;
    const int hi = part == 0 ? 6 : part == 1 ? 11 : part == 2 ? 16 : 21;
    const int nb = part < 2 ? slen1 : slen2;
    const bool st = (store >> part) & 1u;
    for (int sfb = lo; sfb < hi; sfb++) {
      const uint32_t v = nb ? r.bits(nb) : 0u;
      if (st) sf.put_l(sfb, v);
    }
  }
}

// The 64-bit-aligned bit position the job's reads start from (granule 0's
// part 2 for an scfsi copy).
MP3G_HD_INLINE uint64_t job_base(const mp3g_hjob& J) { return (J.part2_start - J.scf0_delta) & ~63ull; }

// Decodes job j (= 2 * granule + channel): scale factors and count1 into
// gran[j / 2].ch[j % 2], the 576 lines into coef[j * 576 ..] up to the
// returned line z (a multiple of 8); lines [z, 576) are left for the caller
// to zero (zero_fill_row).  words / nw: the main data from job_base(job) on
// (Reader); T / s_root / s_lin: the HuffLut entries, roots and linbits (LDS
// on the device).
template <bool kSwap>
MP3G_HD_INLINE int decode_job(const mp3g_hjob& job, uint64_t j, const uint64_t* words, uint32_t nw,
                               mp3g_granule* gran, int16_t* coef, const uint16_t* T, const uint32_t* s_root,
                               const uint32_t* s_lin) {
  // a register copy: the coefficient / scale-factor stores below could alias
  // the job in the compiler's eyes, which would re-load its fields from memory
  // (with a full vmcnt wait) in every loop iteration
  const mp3g_hjob J = job;
#ifdef MP3G_HUFF_SINK_ROWS  // timing experiments only: every row into one of 64 L2-resident rows
  int16_t* row = coef + (j & 63) * MP3G_LINES;
#else
  int16_t* row = coef + j * MP3G_LINES;
#endif
  LineWriter out{row, {}};
  if (J.sf_kind == MP3G_SF_NONE) {  // absent channel of a mono granule
    return 0;
  }
  mp3g_channel& C = gran[j >> 1].ch[j & 1];
  SfRegs sf;

  const uint64_t base = job_base(J);
  Reader<kSwap> r;
  r.w = words;
  r.nw = nw;
  r.end = J.bit_end > base ? (uint32_t)(J.bit_end - base) : 0u;
  const uint32_t part2 = (uint32_t)(J.part2_start - base);

  // ---- scale factors ----
  const int slen1 = J.slen[0], slen2 = J.slen[1];
  switch (J.sf_kind) {
    case MP3G_SF_MPEG1_LONG:
      if (J.scfsi) {
        // granule 1 copies the scfsi parts from granule 0 (maindata.go:239-278):
        // re-read them from granule 0's part 2 (zero where granule 0 has none)
        r.seek(part2 - J.scf0_delta);
        if (J.sf0_kind == MP3G_SF_MPEG1_LONG) {
          sf_mpeg1_long(r, J.sf0_slen[0], J.sf0_slen[1], 15u, J.scfsi, sf);
        } else if (J.sf0_kind == MP3G_SF_MPEG1_MIXED) {
          const int nb = J.sf0_slen[0];
          for (int sfb = 0; sfb < 8; sfb++) {
            const uint32_t v = nb ? r.bits(nb) : 0u;
            if ((J.scfsi >> (sfb < 6 ? 0 : 1)) & 1u) sf.put_l(sfb, v);
          }
        }
      }
      r.seek(part2);
      sf_mpeg1_long(r, slen1, slen2, ~(uint32_t)J.scfsi & 15u, ~(uint32_t)J.scfsi & 15u, sf);
      break;
    case MP3G_SF_MPEG1_SHORT:
    case MP3G_SF_MPEG1_MIXED: {
      r.seek(part2);
      const bool mixed = J.sf_kind == MP3G_SF_MPEG1_MIXED;
      if (mixed)
        for (int sfb = 0; sfb < 8; sfb++) sf.put_l(sfb, slen1 ? r.bits(slen1) : 0u);
      for (int sfb = 0; sfb < 12; sfb++) {  // from band 3 when mixed
        if (mixed && sfb < 3) continue;
        const int nb = sfb < 6 ? slen1 : slen2;
        for (int win = 0; win < 3; win++) sf.put_s(3 * sfb + win, nb ? r.bits(nb) : 0u);
      }
      break;
    }
    default: {  // MPEG-2 (maindata.go:132-179): nsf[part] factors of slen[part] bits
      r.seek(part2);
      const bool lng = J.sf_kind == MP3G_SF_MPEG2_LONG;
      int k = 0;
      for (int part = 0; part < 4; part++) {
        const int nb = J.slen[part];
        for (int n = 0; n < (int)J.nsf[part]; n++, k++) {
          const uint32_t v = nb ? r.bits(nb) : 0u;
          if (lng) {  // runtime indices: plain byte stores
            if (k < 22) C.scalefac_l[k] = (uint8_t)v;
          } else if (k < 39) {
            (&C.scalefac_s[0][0])[k] = (uint8_t)v;
          }
        }
      }
      break;
    }
  }

  if (J.sf_kind <= MP3G_SF_MPEG1_MIXED) sf.store(C, (int)(j & 1));

  // ---- Huffman (maindata/huffman.go:27-138) ----
  int i = 0, count1 = 0;
  const uint32_t p23 = J.part2_3_length;
  if (p23) {
    const uint32_t pend = part2 + p23 - 1;  // bitPosEnd
    const int bv2 = 2 * (int)J.big_values;  // <= 576 (the scan rejects more)
    const int r1 = J.region1_start, r2 = J.region2_start;
    const uint32_t root0 = s_root[J.table_select[0]], root1 = s_root[J.table_select[1]],
                   root2 = s_root[J.table_select[2]], qroot = s_root[32 + J.count1_table];
    const uint32_t lb0 = s_lin[J.table_select[0]], lb1 = s_lin[J.table_select[1]], lb2 = s_lin[J.table_select[2]];
    // big values one writer block (kBlk / 2 pairs) per step: the block's
    // words sit in fixed registers (no per-pair slot select) and full blocks
    // are stored straight away; the block holding bv2 (when it is not a
    // multiple of kBlk) goes on in the writer for the count1 quads
    for (int i0 = 0; i0 < bv2; i0 += kBlk) {
      uint32_t w[kBlk / 2];
#pragma unroll
      for (int sl = 0; sl < kBlk / 2; sl++) {
        const int ii = i0 + 2 * sl;
        w[sl] = 0u;
        if (ii < bv2) {
          const uint32_t root = ii < r1 ? root0 : ii < r2 ? root1 : root2;
          const uint32_t lb = ii < r1 ? lb0 : ii < r2 ? lb1 : lb2;
          int a, b, c, d;
          decode_sym<kSwap, false>(r, T, root, lb, a, b, c, d);
          w[sl] = (uint32_t)(uint16_t)(int16_t)a | ((uint32_t)(uint16_t)(int16_t)b << 16);
        }
      }
#pragma unroll
      for (int sl = 0; sl < kBlk / 2; sl++) out.b[sl] = w[sl];
      if (i0 + kBlk <= bv2) {
        out.flush(i0);
#pragma unroll
        for (int sl = 0; sl < kBlk / 2; sl++) out.b[sl] = 0u;
      }
    }
    // count1 quads (huffman.go:106-131), one writer block per step as well:
    // every quad of the phase starts at a line = bv2 (mod 4), i.e. at dword
    // slot 2q (even phase) or 2q + 1 (odd phase) of its 16-line block, so the
    // four quad slots of a block write fixed registers (an odd phase's fourth
    // quad carries its second dword into the next block).  The block holding
    // bv2 starts with the pairs' partial block and skips the slots before it.
    i = bv2;
    bool act = i <= 572 && r.pos <= pend;
    const bool odd = (bv2 & 2) != 0;
    const int k0 = (bv2 & (kBlk - 1)) >> 1;  // first free dword slot of the first block
    bool pend_blk = act || k0 != 0;           // this block has lines to store
    int blk = bv2 & ~(kBlk - 1);
    bool first_blk = true;
    uint32_t w[kBlk / 2];
#pragma unroll
    for (int sl = 0; sl < kBlk / 2; sl++) w[sl] = out.b[sl];
    while (pend_blk) {
      uint32_t carry = 0u;
      bool carried = false;
#pragma unroll
      for (int q = 0; q < kBlk / 4; q++) {
        const int slot = odd ? 2 * q + 1 : 2 * q;
        if (act && (!first_blk || slot >= k0)) {
          int a, b, c, d;
          decode_sym<kSwap, true>(r, T, qroot, 0u, a, b, c, d);
          const uint32_t v0 = (uint32_t)(uint16_t)(int16_t)a | ((uint32_t)(uint16_t)(int16_t)b << 16);
          const uint32_t v1 = (uint32_t)(uint16_t)(int16_t)c | ((uint32_t)(uint16_t)(int16_t)d << 16);
          if (odd) {
            w[2 * q + 1] = v0;
            if (q + 1 < kBlk / 4) {
              w[2 * q + 2] = v1;
            } else {
              carry = v1;
              carried = true;
            }
          } else {
            w[2 * q] = v0;
            w[2 * q + 1] = v1;
          }
          i += 4;
          act = i <= 572 && r.pos <= pend;
        }
      }
#pragma unroll
      for (int sl = 0; sl < kBlk / 2; sl++) out.b[sl] = w[sl];
      out.flush(blk);
#pragma unroll
      for (int sl = 0; sl < kBlk / 2; sl++) w[sl] = 0u;
      w[0] = carry;
      blk += kBlk;
      first_blk = false;
      pend_blk = act || carried;
    }
    count1 = i;
    if (r.pos > pend + 1) count1 = i >= 4 ? i - 4 : 0;  // the last word overran its part
  }
  const int z = p23 ? (i + kBlk - 1) & ~(kBlk - 1) : out.finish(i);
  for (int k = count1; k < i; k++) row[k] = 0;  // lines the overrun check removed
  C.count1 = (uint16_t)count1;
  return z;
}

// decode_job straight from the main data in memory (stream byte order; must
// be 8-byte aligned and readable up to 8 bytes past the last bit_end).
MP3G_HD_INLINE int decode_job_direct(const mp3g_hjob& job, uint64_t j, const uint8_t* md, mp3g_granule* gran,
                                      int16_t* coef, const uint16_t* T, const uint32_t* s_root,
                                      const uint32_t* s_lin) {
  const uint64_t base = job_base(job);
  const uint32_t nw = job.bit_end > base ? (uint32_t)((job.bit_end - base + 63) >> 6) : 0u;
  return decode_job<true>(job, j, reinterpret_cast<const uint64_t*>(md + (base >> 3)), nw, gran, coef, T, s_root,
                          s_lin);
}

}  // namespace huff
}  // namespace mp3g
