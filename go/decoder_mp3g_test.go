//go:build mp3g

// GC stress of the decoder shim (decoder_mp3g.go): the library calls back into
// Go (mp3gGoRead / mp3gGoSeek) in the middle of a cgo call, and the Decoder's
// finalizer frees the library decoder and deletes the cgo.Handle those
// callbacks use.  A reader that collects garbage and runs finalizers inside
// every callback makes a Decoder that is unreachable during its own call --
// the last Read of io.ReadAll(dec) -- fail loudly (invalid handle panic or
// freed decoder) unless every method keeps its receiver alive
// (runtime.KeepAlive).  The PCM is compared with the in-memory entry of the
// same library (NewDecoderBytes, no callbacks).  Names carry the MP3G prefix:
// this file sits beside the reference's own tests in package mp3.
package mp3

import (
	"bytes"
	"io"
	"os"
	"runtime"
	"testing"
)

type mp3gGCReader struct{ r io.Reader }

func (g *mp3gGCReader) Read(p []byte) (int, error) {
	runtime.GC()
	runtime.Gosched() // let the finalizer goroutine run
	return g.r.Read(p)
}

type mp3gGCSeeker struct{ r *bytes.Reader }

func (g *mp3gGCSeeker) Read(p []byte) (int, error) {
	runtime.GC()
	runtime.Gosched()
	return g.r.Read(p)
}

func (g *mp3gGCSeeker) Seek(off int64, whence int) (int64, error) {
	runtime.GC()
	runtime.Gosched()
	return g.r.Seek(off, whence)
}

func mp3gWant(t *testing.T, data []byte) []byte {
	t.Helper()
	d, err := NewDecoderBytes(data, true)
	if err != nil {
		t.Fatal(err)
	}
	defer d.Close()
	want, err := io.ReadAll(d)
	if err != nil {
		t.Fatal(err)
	}
	return want
}

func mp3gReadAllFresh(t *testing.T, r io.Reader) []byte {
	t.Helper()
	d, err := NewDecoder(r)
	if err != nil {
		t.Fatal(err)
	}
	// d is not used after this line: only the receivers of its methods keep it alive
	got, err := io.ReadAll(d)
	if err != nil {
		t.Fatal(err)
	}
	return got
}

func TestMP3G_GCInsideReaderCallbacks(t *testing.T) {
	for _, name := range []string{"example/classic_lame.mp3", "example/mpeg2.mp3"} {
		data, err := os.ReadFile(name)
		if err != nil {
			t.Fatal(err)
		}
		want := mp3gWant(t, data)
		for i := 0; i < 4; i++ {
			if got := mp3gReadAllFresh(t, &mp3gGCReader{bytes.NewReader(data)}); !bytes.Equal(got, want) {
				t.Fatalf("%s: streaming (non-seekable) decode differs: %d vs %d bytes", name, len(got), len(want))
			}
			if got := mp3gReadAllFresh(t, &mp3gGCSeeker{bytes.NewReader(data)}); !bytes.Equal(got, want) {
				t.Fatalf("%s: streaming (seekable) decode differs: %d vs %d bytes", name, len(got), len(want))
			}
		}
	}
}

func TestMP3G_GCDuringTimeAPI(t *testing.T) {
	data, err := os.ReadFile("example/classic_lame.mp3")
	if err != nil {
		t.Fatal(err)
	}
	d, err := NewDecoder(&mp3gGCSeeker{bytes.NewReader(data)})
	if err != nil {
		t.Fatal(err)
	}
	dur := d.Duration()
	if err := d.SeekToTime(dur / 2); err != nil {
		t.Fatal(err)
	}
	buf := make([]byte, 4096)
	if _, err := io.ReadFull(d, buf); err != nil {
		t.Fatal(err)
	}
	if p := d.Position(); p <= 0 || p > dur {
		t.Fatalf("Position %v after a seek to %v and a read", p, dur/2)
	}
}
