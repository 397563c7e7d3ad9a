/* mp3g_decode.c -- a plain C consumer of the C-ABI (include/mp3g.h): what the
 * reference's example/main.go does with mp3.NewDecoder before it hands the
 * PCM to an audio device (example/main.go; decode.go:361-388), minus the
 * device: the file is STREAMED into the decoder through mp3g_reader callbacks
 * on a FILE* (the same shape the cgo shim uses with a cgo.Handle,
 * go/reader_mp3g.c), the PCM (s16le stereo, as Decoder.Read gives it) goes to
 * a file or stdout in io.ReadFull-sized blocks.
 *
 *   mp3g_decode [-f] [-n] in.mp3 [out.pcm]
 *     -f  fast mode (within 1 LSB of the reference; default: bit-exact)
 *     -n  present the input as a non-seekable reader (Length() = -1)
 * Prints sample rate, length, duration and the PCM bytes written to stderr.
 * Build: cc -std=c99 -I include examples/mp3g_decode.c -L go-mp3_amd/mp3g -lmp3g
 */
#include <errno.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mp3g.h"

/* io.Reader.Read over a FILE*: the count, 0 at EOF, -1 on an error */
static int64_t file_read(void* user, uint8_t* buf, size_t cap) {
  FILE* f = (FILE*)user;
  const size_t n = fread(buf, 1, cap, f);
  if (n == 0 && ferror(f)) return -1;
  return (int64_t)n;
}

/* io.Seeker.Seek: the new offset, -1 on an error */
static int64_t file_seek(void* user, int64_t offset, int whence) {
  FILE* f = (FILE*)user;
  const int w = whence == 0 ? SEEK_SET : whence == 1 ? SEEK_CUR : SEEK_END;
  if (fseek(f, (long)offset, w) != 0) return -1;
  return (int64_t)ftell(f);
}

static int fail(const char* what, int st) {
  fprintf(stderr, "mp3g_decode: %s: %s (%s)\n", what, mp3g_status_string(st), mp3g_last_error());
  return 1;
}

int main(int argc, char** argv) {
  uint32_t mode = MP3G_MODE_EXACT;
  int seekable = 1, a = 1;
  for (; a < argc && argv[a][0] == '-' && argv[a][1]; a++) {
    if (!strcmp(argv[a], "-f")) mode = MP3G_MODE_FAST;
    else if (!strcmp(argv[a], "-n")) seekable = 0;
    else break;
  }
  if (a >= argc) {
    fprintf(stderr, "usage: %s [-f] [-n] in.mp3 [out.pcm]\n", argv[0]);
    return 2;
  }
  if (mp3g_abi_version() != MP3G_ABI_VERSION) {
    fprintf(stderr, "mp3g_decode: built for ABI %d, library has %d\n", MP3G_ABI_VERSION, mp3g_abi_version());
    return 1;
  }
  FILE* in = fopen(argv[a], "rb");
  if (!in) {
    fprintf(stderr, "mp3g_decode: %s: %s\n", argv[a], strerror(errno));
    return 1;
  }
  FILE* out = a + 1 < argc ? fopen(argv[a + 1], "wb") : stdout;
  if (!out) {
    fprintf(stderr, "mp3g_decode: %s: %s\n", argv[a + 1], strerror(errno));
    fclose(in);
    return 1;
  }
  mp3g_reader r = {file_read, seekable ? file_seek : NULL, in};
  mp3g_decoder* dec = NULL;
  int st = mp3g_decoder_new_reader(&r, 0, mode, &dec);
  if (st != MP3G_OK) return fail("NewDecoder", st);
  int sample_rate = 0;
  int64_t length = 0, bpf = 0, pos = 0;
  mp3g_decoder_info(dec, &sample_rate, &length, &bpf, &pos);
  /* io.ReadFull in 1 MiB blocks until io.EOF (a short last block is the end) */
  const size_t cap = 1u << 20;
  uint8_t* buf = (uint8_t*)malloc(cap);
  uint64_t total = 0;
  int rc = 0;
  for (;;) {
    size_t n = 0;
    st = mp3g_decoder_read_full(dec, buf, cap, &n);
    if (n && fwrite(buf, 1, n, out) != n) {
      fprintf(stderr, "mp3g_decode: write: %s\n", strerror(errno));
      rc = 1;
      break;
    }
    total += n;
    if (st == MP3G_EOF) break;
    if (st != MP3G_OK) {
      rc = fail("Read", st);
      break;
    }
  }
  fprintf(stderr, "sample_rate %d length %" PRId64 " bytes_per_frame %" PRId64 " duration_ns %" PRId64
                  " pcm_bytes %" PRIu64 " mode %s\n",
          sample_rate, length, bpf, mp3g_decoder_duration_ns(dec), total,
          mode == MP3G_MODE_FAST ? "fast" : "exact");
  free(buf);
  mp3g_decoder_free(dec);
  fclose(in);
  if (out != stdout) fclose(out);
  return rc;
}
