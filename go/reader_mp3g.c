//go:build mp3g

// reader_mp3g.c -- the C half of decoder_mp3g.go's streaming NewDecoder: an
// mp3g_reader (include/mp3g.h, ABI 3) whose callbacks call the Go functions
// exported there, passing the cgo.Handle of the decoder's reader state as the
// opaque user value (no Go pointer crosses into C).  In a .c file because a
// Go file with //export may only declare C functions in its preamble.
#include <stdint.h>

#include "mp3g.h"
#include "_cgo_export.h"

static int64_t goreader_read(void* user, uint8_t* buf, size_t cap) {
  return mp3gGoRead((uintptr_t)user, buf, cap);
}

static int64_t goreader_seek(void* user, int64_t offset, int whence) {
  return mp3gGoSeek((uintptr_t)user, offset, whence);
}

int goreader_decoder_new(uintptr_t h, int seekable, int device, uint32_t mode, mp3g_decoder** out) {
  mp3g_reader r = {goreader_read, seekable ? goreader_seek : 0, (void*)h};
  return mp3g_decoder_new_reader(&r, device, mode, out);
}
