#!/bin/sh
# apply_mp3g.sh -- the integration recipe of the GPU decoder into a checkout
# of llehouerou/go-mp3 ("Applying the shims").
#
#   go/apply_mp3g.sh <go-mp3 checkout> [<libmp3g.so>]
#
# 1. decode.go gets the build constraint `//go:build !mp3g`: with the tag
#    mp3g the package's Decoder, NewDecoder and the Decoder methods come from
#    decoder_mp3g.go instead (the two declare the same identifiers in package
#    mp3, so exactly one of them may be compiled).  source.go stays: nothing
#    in decoder_mp3g.go redeclares its identifiers and the reference's own
#    tests use its `source` type (time_seek_test.go).
# 2. decoder_mp3g.go + reader_mp3g.c (+ the GC-stress test) go next to
#    decode.go, frame_mp3g.go next to internal/frame/frame.go.
# 3. include/mp3g.h and the library go to third_party/mp3g/{include,lib},
#    where the shims' #cgo lines look.
#
# Then `go test -tags mp3g ./...` runs the reference's own test suite against
# the GPU decoder, and `go test ./...` (no tag) the pure-Go one, unchanged.
# tests/test_cgo_shim_cpu.py applies this recipe to a scratch copy of the
# reference's package declarations and checks that each build has every
# identifier exactly once.  Idempotent.
set -eu
[ $# -ge 1 ] || { echo "usage: $0 <go-mp3 checkout> [libmp3g.so]" >&2; exit 2; }
DST=$1
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(dirname "$HERE")
LIB=${2:-$REPO/go-mp3_amd/mp3g/libmp3g.so}
[ -f "$DST/decode.go" ] && [ -f "$DST/internal/frame/frame.go" ] || {
  echo "$0: $DST is not a go-mp3 checkout (decode.go, internal/frame/frame.go)" >&2; exit 2; }

# 1. the gate (a first line //go:build must be followed by a blank line)
if head -n 1 "$DST/decode.go" | grep -q '^//go:build'; then
  head -n 1 "$DST/decode.go" | grep -q '^//go:build !mp3g$' || {
    echo "$0: decode.go already has another build constraint: merge '!mp3g' into it by hand" >&2; exit 1; }
else
  tmp=$(mktemp)
  { printf '//go:build !mp3g\n\n'; cat "$DST/decode.go"; } > "$tmp"
  mv "$tmp" "$DST/decode.go"
fi

# 2. the shims
cp "$HERE/decoder_mp3g.go" "$HERE/reader_mp3g.c" "$HERE/decoder_mp3g_test.go" "$DST/"
cp "$HERE/frame_mp3g.go" "$DST/internal/frame/"

# 3. header and library
mkdir -p "$DST/third_party/mp3g/include" "$DST/third_party/mp3g/lib"
cp "$REPO/include/mp3g.h" "$DST/third_party/mp3g/include/"
if [ -f "$LIB" ]; then
  cp "$LIB" "$DST/third_party/mp3g/lib/libmp3g.so"
else
  echo "$0: note: $LIB not built yet (make -C go-mp3_amd/csrc); copy it to third_party/mp3g/lib/" >&2
fi
echo "applied: go test -tags mp3g ./... decodes on the GPU, go test ./... stays pure Go"
