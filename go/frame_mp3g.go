//go:build mp3g

// Package frame (go-mp3 internal/frame) -- the GPU batch shim.
//
// Drop-in for the per-frame DSP seam of llehouerou/go-mp3: a maintainer adds
// this file next to internal/frame/frame.go; with the build tag `mp3g` the
// decoder collects parsed frames into a Batch and replaces the per-frame
// `d.frame.Decode()` (reference decode.go:65, frame.go:121) by one
// DecodeBatch call per read-ahead batch.  The Huffman / side-info parse
// stays in Go: frame.Read (frame.go:67-115) still fills SideInfo and
// MainData, and Add copies exactly the fields Decode reads (SURVEY.md 8a
// row a10) into the C-ABI's granule descriptors (include/mp3g.h
// mp3g_granule) and the integer MainData.Is values into int16 coefficients.
//
// Written from include/mp3g.h (ABI version 5) field by field;
// tests/test_cgo_shim_cpu.py checks every C identifier used here against the
// header (no Go toolchain in the build image).  INTEGRATION.md explains the
// read-ahead in decode.go that drives it.
package frame

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/mp3g/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/mp3g/lib -lmp3g -Wl,-rpath,${SRCDIR}/../../third_party/mp3g/lib
#include <stdlib.h>
#include "mp3g.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

// ABIVersion is the C-ABI version this shim was written against.
const ABIVersion = 5

// Batch collects parsed frames; DecodeBatch replaces calling Decode() on each.
// Not safe for concurrent use (like Decoder, decode.go:31-33).
type Batch struct {
	gran  []C.mp3g_granule // Go memory, read by C during the call only (cgo pointer rules)
	coef  []int16
	state C.mp3g_state // Frame.store / vVec of the stream (frame.go:48-49)
	valid bool         // state carried from the previous batch
	mode  C.uint32_t
}

// NewBatch: fast = true selects MP3G_MODE_FAST (PCM within +-1 LSB of the
// reference), false the bit-exact mode.
func NewBatch(fast bool) *Batch {
	b := &Batch{mode: C.MP3G_MODE_EXACT}
	if fast {
		b.mode = C.MP3G_MODE_FAST
	}
	if rc := C.mp3g_abi_version(); int(rc) != ABIVersion {
		panic(fmt.Sprintf("mp3g: shim for ABI %d, library %d", ABIVersion, int(rc)))
	}
	return b
}

// Add appends the granules of a frame read by frame.Read (its Decode is not called).
func (b *Batch) Add(f *Frame) {
	nch := f.header.NumberOfChannels()
	for gr := 0; gr < f.header.Granules(); gr++ {
		var g C.mp3g_granule
		g.header = C.uint32_t(f.header)
		g.gr = C.uint32_t(gr)
		si := f.sideInfo
		for ch := 0; ch < nch; ch++ {
			c := &g.ch[ch]
			c.count1 = C.uint16_t(si.Count1[gr][ch])
			c.global_gain = C.uint8_t(si.GlobalGain[gr][ch])
			c.scalefac_scale = C.uint8_t(si.ScalefacScale[gr][ch])
			c.preflag = C.uint8_t(si.Preflag[gr][ch])
			c.win_switch_flag = C.uint8_t(si.WinSwitchFlag[gr][ch])
			c.block_type = C.uint8_t(si.BlockType[gr][ch])
			c.mixed_block_flag = C.uint8_t(si.MixedBlockFlag[gr][ch])
			for w := 0; w < 3; w++ {
				c.subblock_gain[w] = C.uint8_t(si.SubblockGain[gr][ch][w])
			}
			for s := 0; s < 22; s++ {
				c.scalefac_l[s] = C.uint8_t(f.mainData.ScalefacL[gr][ch][s])
			}
			for s := 0; s < 13; s++ {
				for w := 0; w < 3; w++ {
					c.scalefac_s[s][w] = C.uint8_t(f.mainData.ScalefacS[gr][ch][s][w])
				}
			}
		}
		b.gran = append(b.gran, g)
		var lines [2 * C.MP3G_LINES]int16
		for ch := 0; ch < nch; ch++ {
			for i, v := range f.mainData.Is[gr][ch] {
				lines[ch*C.MP3G_LINES+i] = int16(v) // integer-valued, |v| <= 8206
			}
		}
		b.coef = append(b.coef, lines[:]...)
	}
}

// Len is the number of granules waiting.
func (b *Batch) Len() int { return len(b.gran) }

// DecodeBatch returns the concatenated Decode() output of every added frame
// (s16le stereo, BytesPerFrame per frame) and carries Frame.store / vVec to
// the next batch, as frame.Read copies them from the previous frame
// (frame.go:110-113).  Decode cannot fail (frame.go:121); an error here is a
// device / ABI error.
func (b *Batch) DecodeBatch() ([]byte, error) {
	n := len(b.gran)
	pcm := make([]byte, n*C.MP3G_PCM_BYTES_PER_GRANULE)
	if n == 0 {
		return pcm, nil
	}
	var flags C.uint32_t = C.MP3G_STREAM_STATE_OUT
	if b.valid {
		flags |= C.MP3G_STREAM_STATE_IN
	}
	s := C.mp3g_stream{first_granule: 0, n_granules: C.uint32_t(n), flags: flags}
	in := b.state // copy: state_in and state_out may not alias
	st := C.mp3g_decode_host(0,
		(*C.mp3g_granule)(unsafe.Pointer(&b.gran[0])),
		(*C.int16_t)(unsafe.Pointer(&b.coef[0])), C.uint64_t(n),
		&s, 1, &in, &b.state,
		(*C.int16_t)(unsafe.Pointer(&pcm[0])), b.mode)
	if st != C.MP3G_OK {
		return nil, fmt.Errorf("mp3g: %s: %s", C.GoString(C.mp3g_status_string(st)),
			C.GoString(C.mp3g_last_error()))
	}
	b.gran, b.coef, b.valid = b.gran[:0], b.coef[:0], true
	return pcm, nil
}

// Reset drops the carried state, as `d.frame = nil` does on Seek (decode.go:106-108).
func (b *Batch) Reset() { b.valid = false }
