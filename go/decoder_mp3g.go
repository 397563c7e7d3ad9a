//go:build mp3g

// Package mp3 -- the whole decoder behind the C-ABI (alternative to
// frame_mp3g.go): mp3.NewDecoder / io.Reader / io.Seeker and the time API of
// llehouerou/go-mp3 (decode.go:27-388) over mp3g_decoder_* (include/mp3g.h),
// which scans on the host with read-ahead and decodes batches of frames on
// the GPU (main data and DSP), carrying the DSP state between batches.
// Also DecodeMany, the batch API for servers (mp3g_decode_streams).
//
// The io.Reader is streamed, not slurped: NewDecoder hands the library two
// callbacks (reader_mp3g.c trampolines into mp3gGoRead / mp3gGoSeek below),
// so it returns once the tags and frame 0 are in, as the reference's does
// (decode.go:361-388), and Read pulls input only as the read-ahead needs it
// (source.go:99-122) -- a live stream that has not ended gets a decoder and
// every frame that has arrived.
//
// Written from include/mp3g.h (ABI version 5, checked against the loaded
// library by checkABI); tests/test_cgo_shim_cpu.py checks every C identifier
// used here against the header.
package mp3

/*
#cgo CFLAGS: -I${SRCDIR}/third_party/mp3g/include
#cgo LDFLAGS: -L${SRCDIR}/third_party/mp3g/lib -lmp3g -Wl,-rpath,${SRCDIR}/third_party/mp3g/lib
#include <stdlib.h>
#include <stdint.h>
#include "mp3g.h"
// reader_mp3g.c: an mp3g_reader whose callbacks call the exported Go
// functions below with the cgo.Handle h as the user value
int goreader_decoder_new(uintptr_t h, int seekable, int device, uint32_t mode, mp3g_decoder** out);
*/
import "C"

import (
	"errors"
	"fmt"
	"io"
	"runtime"
	"runtime/cgo"
	"sync"
	"time"
	"unsafe"
)

// ABIVersion is the C-ABI version this shim was written against.
const ABIVersion = 5

var abiOnce sync.Once
var abiErr error

// checkABI: the loaded libmp3g must speak the ABI this file was written for.
func checkABI() error {
	abiOnce.Do(func() {
		if v := int(C.mp3g_abi_version()); v != ABIVersion {
			abiErr = fmt.Errorf("mp3: shim written for libmp3g ABI %d, library has %d", ABIVersion, v)
		}
	})
	return abiErr
}

// Mode: bit-exact PCM or within +-1 LSB of the reference (faster).
var Mode C.uint32_t = C.MP3G_MODE_EXACT

func statusError(st C.int) error {
	switch st {
	case C.MP3G_OK:
		return nil
	case C.MP3G_EOF:
		return io.EOF
	}
	return fmt.Errorf("mp3: %s: %s", C.GoString(C.mp3g_status_string(st)), C.GoString(C.mp3g_last_error()))
}

// Decoder is a MP3-decoded stream (decode.go:34-43). Not safe for concurrent use.
type Decoder struct {
	d  *C.mp3g_decoder
	h  cgo.Handle   // the reader state the C callbacks reach (0 for NewDecoderBytes)
	rs *readerState // nil for NewDecoderBytes
}

// readerState is what the library's callbacks reach through the handle: the
// caller's reader and the error a failed Read / Seek returned, handed back
// from the decoder call that ran into it (decode.go:48-63 passes a reader's
// error through).
type readerState struct {
	r    io.Reader
	s    io.Seeker // nil: not an io.Seeker (Length() = -1)
	err  error     // the reader's last error
	pend error     // an error Read returned together with data: reported by the next call
}

//export mp3gGoRead
func mp3gGoRead(h C.uintptr_t, buf *C.uint8_t, n C.size_t) C.int64_t {
	rs := cgo.Handle(h).Value().(*readerState)
	if e := rs.pend; e != nil {
		rs.pend = nil
		if e == io.EOF || e == io.ErrUnexpectedEOF {
			return 0
		}
		rs.err = e
		return -1
	}
	p := unsafe.Slice((*byte)(unsafe.Pointer(buf)), int(n))
	for { // io.ReadFull's loop: (0, nil) asks again
		k, err := rs.r.Read(p)
		if k > 0 {
			rs.pend = err
			return C.int64_t(k)
		}
		if err == io.EOF || err == io.ErrUnexpectedEOF { // source.go:112-118
			return 0
		}
		if err != nil {
			rs.err = err
			return -1
		}
	}
}

//export mp3gGoSeek
func mp3gGoSeek(h C.uintptr_t, off C.int64_t, whence C.int) C.int64_t {
	rs := cgo.Handle(h).Value().(*readerState)
	n, err := rs.s.Seek(int64(off), int(whence))
	if err != nil {
		rs.err = err
		return -1
	}
	return C.int64_t(n)
}

// NewDecoder decodes the given io.Reader (decode.go:361-388), streaming it:
// the library calls back into r as it needs bytes and never retains a Go
// pointer (the callbacks get a cgo.Handle).
func NewDecoder(r io.Reader) (*Decoder, error) {
	if err := checkABI(); err != nil {
		return nil, err
	}
	rs := &readerState{r: r}
	seekable := C.int(0)
	if s, ok := r.(io.Seeker); ok {
		rs.s = s
		seekable = 1
	}
	h := cgo.NewHandle(rs)
	var d *C.mp3g_decoder
	if st := C.goreader_decoder_new(C.uintptr_t(h), seekable, 0, Mode, &d); st != C.MP3G_OK {
		err := rs.statusError(st)
		h.Delete()
		return nil, err
	}
	return track(&Decoder{d: d, h: h, rs: rs}), nil
}

// track: the reference's Decoder has no Close (decode.go:34-43), so a drop-in
// caller never calls it -- a finalizer releases the library decoder (its
// pinned host and device buffers) and the handle that pins the caller's
// reader once the Decoder is unreachable.  Close stays idempotent.
func track(d *Decoder) *Decoder {
	runtime.SetFinalizer(d, func(d *Decoder) { d.Close() })
	return d
}

// NewDecoderBytes decodes a complete stream already in memory (the library
// copies it; no callbacks): seekable as for a bytes.Reader.
func NewDecoderBytes(data []byte, seekable bool) (*Decoder, error) {
	if err := checkABI(); err != nil {
		return nil, err
	}
	var p *C.uint8_t
	if len(data) > 0 {
		p = (*C.uint8_t)(unsafe.Pointer(&data[0]))
	}
	s := C.int(0)
	if seekable {
		s = 1
	}
	var d *C.mp3g_decoder
	if st := C.mp3g_decoder_new(p, C.size_t(len(data)), s, 0, Mode, &d); st != C.MP3G_OK {
		return nil, statusError(st)
	}
	return track(&Decoder{d: d}), nil
}

// statusError with the reader's own error for MP3G_ERR_READ.
func (rs *readerState) statusError(st C.int) error {
	if st == C.MP3G_ERR_READ && rs != nil && rs.err != nil {
		return rs.err
	}
	return statusError(st)
}

func (d *Decoder) statusError(st C.int) error { return d.rs.statusError(st) }

// Close releases the decoder's host and device memory (idempotent; the
// finalizer calls it too).
func (d *Decoder) Close() error {
	runtime.SetFinalizer(d, nil)
	if d.d != nil {
		C.mp3g_decoder_free(d.d)
		d.d = nil
	}
	if d.h != 0 {
		d.h.Delete()
		d.h = 0
	}
	return nil
}

// Read is io.Reader's Read (decode.go:70-80): at most the rest of one frame.
//
// Every method that passes d.d to the library keeps d reachable until the
// call has returned (defer runtime.KeepAlive(d)): without it d can become
// unreachable once d.d is loaded -- the last Read of an io.ReadAll(dec) --
// and in reader mode the library calls back into Go during the call, where
// a GC can run the finalizer: Close would free the decoder under the call and
// delete the cgo.Handle its callbacks use.
func (d *Decoder) Read(buf []byte) (int, error) {
	defer runtime.KeepAlive(d)
	if len(buf) == 0 {
		return 0, nil
	}
	var n C.size_t
	st := C.mp3g_decoder_read(d.d, (*C.uint8_t)(unsafe.Pointer(&buf[0])), C.size_t(len(buf)), &n)
	if st != C.MP3G_OK {
		return int(n), d.statusError(st)
	}
	return int(n), nil
}

// ReadFull is io.ReadFull(d, buf) in one cgo call.
func (d *Decoder) ReadFull(buf []byte) (int, error) {
	defer runtime.KeepAlive(d)
	if len(buf) == 0 {
		return 0, nil
	}
	var n C.size_t
	st := C.mp3g_decoder_read_full(d.d, (*C.uint8_t)(unsafe.Pointer(&buf[0])), C.size_t(len(buf)), &n)
	switch {
	case st == C.MP3G_OK:
		return int(n), nil
	case st == C.MP3G_EOF && n == 0:
		return 0, io.EOF
	case st == C.MP3G_EOF:
		return int(n), io.ErrUnexpectedEOF
	}
	return int(n), d.statusError(st)
}

// Seek is io.Seeker's Seek (decode.go:89-145), with the reference's warm-up.
func (d *Decoder) Seek(offset int64, whence int) (int64, error) {
	defer runtime.KeepAlive(d)
	var np C.int64_t
	if st := C.mp3g_decoder_seek(d.d, C.int64_t(offset), C.int(whence), &np); st != C.MP3G_OK {
		return 0, d.statusError(st)
	}
	return int64(np), nil
}

func (d *Decoder) info() (sr int, length, bpf, pos int64) {
	defer runtime.KeepAlive(d)
	var s C.int
	var l, b, p C.int64_t
	C.mp3g_decoder_info(d.d, &s, &l, &b, &p)
	return int(s), int64(l), int64(b), int64(p)
}

// SampleRate (decode.go:147-150).
func (d *Decoder) SampleRate() int { sr, _, _, _ := d.info(); return sr }

// Length in bytes, -1 when the reader is not an io.Seeker (decode.go:218-224).
func (d *Decoder) Length() int64 { _, l, _, _ := d.info(); return l }

// BytesPerFrame (decode.go:226-230).
func (d *Decoder) BytesPerFrame() int64 { _, _, b, _ := d.info(); return b }

// Duration, Position, Remaining, Progress, SamplePosition, SampleCount,
// SeekToSample, Skip, SeekToTime: the time API (decode.go:232-354).
func (d *Decoder) Duration() time.Duration {
	defer runtime.KeepAlive(d)
	return time.Duration(C.mp3g_decoder_duration_ns(d.d))
}

func (d *Decoder) Position() time.Duration {
	defer runtime.KeepAlive(d)
	return time.Duration(C.mp3g_decoder_position_ns(d.d))
}

func (d *Decoder) Remaining() time.Duration {
	defer runtime.KeepAlive(d)
	return time.Duration(C.mp3g_decoder_remaining_ns(d.d))
}

func (d *Decoder) Progress() float64 {
	defer runtime.KeepAlive(d)
	return float64(C.mp3g_decoder_progress(d.d))
}

func (d *Decoder) SamplePosition() int64 {
	defer runtime.KeepAlive(d)
	return int64(C.mp3g_decoder_sample_position(d.d))
}

func (d *Decoder) SampleCount() int64 {
	defer runtime.KeepAlive(d)
	return int64(C.mp3g_decoder_sample_count(d.d))
}

func (d *Decoder) SeekToSample(s int64) error {
	defer runtime.KeepAlive(d)
	return d.statusError(C.mp3g_decoder_seek_to_sample(d.d, C.int64_t(s)))
}

func (d *Decoder) SeekToTime(t time.Duration) error {
	defer runtime.KeepAlive(d)
	return d.statusError(C.mp3g_decoder_seek_to_time_ns(d.d, C.int64_t(t)))
}

func (d *Decoder) Skip(dt time.Duration) error {
	defer runtime.KeepAlive(d)
	return d.statusError(C.mp3g_decoder_skip_ns(d.d, C.int64_t(dt)))
}

// DecodeMany decodes complete MP3 files on the GPU, the main data included:
// pcm[i] is what io.ReadAll(NewDecoder(file i)) returns, errs[i] the error
// that ended file i after its PCM (nil for io.EOF).
func DecodeMany(files [][]byte) ([][]byte, []error) {
	n := len(files)
	out, errs := make([][]byte, n), make([]error, n)
	if n == 0 {
		return out, errs
	}
	if err := checkABI(); err != nil {
		for i := range errs {
			errs[i] = err
		}
		return out, errs
	}
	datas := (*[1 << 30]*C.uint8_t)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:n:n]
	defer C.free(unsafe.Pointer(&datas[0]))
	lens := make([]C.size_t, n)
	for i, f := range files { // C memory: the call reads it, nothing is retained
		datas[i] = (*C.uint8_t)(C.CBytes(f))
		lens[i] = C.size_t(len(f))
		defer C.free(unsafe.Pointer(datas[i]))
	}
	streams := make([]C.mp3g_stream, n)
	status := make([]C.int, n)
	var pcm *C.int16_t
	var ng C.uint64_t
	st := C.mp3g_decode_streams(0, C.uint32_t(n), &datas[0], &lens[0], 0, Mode, &pcm, &ng,
		&streams[0], &status[0])
	if st != C.MP3G_OK {
		e := statusError(st)
		for i := range errs {
			errs[i] = e
		}
		return out, errs
	}
	defer C.mp3g_free(unsafe.Pointer(pcm))
	all := unsafe.Slice((*byte)(unsafe.Pointer(pcm)), int(ng)*C.MP3G_PCM_BYTES_PER_GRANULE)
	for i := range files {
		s := streams[i]
		lo := int(s.first_granule) * C.MP3G_PCM_BYTES_PER_GRANULE
		hi := lo + int(s.n_granules)*C.MP3G_PCM_BYTES_PER_GRANULE
		out[i] = append([]byte(nil), all[lo:hi]...)
		if e := statusError(status[i]); !errors.Is(e, io.EOF) {
			errs[i] = e
		}
	}
	return out, errs
}
