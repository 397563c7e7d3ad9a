"""The committed cgo shim (go/*.go, build tag mp3g) against include/mp3g.h.

There is no Go toolchain in this image, so the shim cannot be compiled here;
this test does the mechanical part of that check: every C identifier the Go
files use exists in the header (functions, types, constants), every C call
passes as many arguments as the prototype declares, and every struct field
the shim writes is a field of that struct.  Reference seams: frame.go:121
(Frame.Decode) and decode.go:65 (its only call site).
"""
import os
import re

from conftest import REPO

HEADER = open(os.path.join(REPO, "include", "mp3g.h")).read()
GO = {f: open(os.path.join(REPO, "go", f)).read() for f in sorted(os.listdir(os.path.join(REPO, "go")))
      if f.endswith(".go")}
CGO_BUILTINS = {"malloc", "free", "CBytes", "GoString", "CString", "GoBytes"}
C_SCALARS = {"int", "uint", "size_t", "uintptr_t", "int16_t", "uint8_t", "uint16_t", "uint32_t", "uint64_t", "int64_t",
             "double", "float", "char"}


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def prototypes():
    """name -> parameter count of every function the header declares."""
    out = {}
    for m in re.finditer(r"\b(?:int|void|double|int64_t|const char\*)\s+\**(mp3g_\w+)\(([^;{]*?)\);",
                         _strip_comments(HEADER), flags=re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def struct_fields(name):
    m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), _strip_comments(HEADER), flags=re.S)
    assert m, name
    return set(re.findall(r"(\w+)\s*(?:\[[^\]]*\])*\s*;", m.group(1)))


def call_args(src, start):
    """Number of top-level arguments of the call whose '(' is at src[start]."""
    depth, n, seen = 0, 0, False
    for ch in src[start:]:
        if ch == "(":
            depth += 1
            if depth == 1:
                continue
        elif ch == ")":
            depth -= 1
            if depth == 0:
                return n + 1 if seen else 0
        elif ch == "," and depth == 1:
            n += 1
        if depth >= 1 and not ch.isspace():
            seen = True
    raise AssertionError("unbalanced call")


def test_go_shim_files_present():
    assert "frame_mp3g.go" in GO and "decoder_mp3g.go" in GO
    for f, src in GO.items():
        assert src.startswith("//go:build mp3g"), f
        assert 'import "C"' in src and '#include "mp3g.h"' in src, f


def preamble_functions(src):
    """name -> parameter count of the C functions a Go file's cgo preamble
    declares itself (helpers defined in the package's .c files)."""
    pre = src.split('import "C"', 1)[0]
    out = {}
    for m in re.finditer(r"^\s*(?://\s*)?(?:int|void|int64_t)\s+\**(\w+)\(([^;{]*?)\);", pre, flags=re.M):
        if m.group(0).lstrip().startswith("//"):
            continue
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_c_identifiers_and_call_arity_match_the_header():
    protos = prototypes()
    hdr = _strip_comments(HEADER)
    for f, src in GO.items():
        code = _strip_comments(src.split('import "C"', 1)[1])
        local = preamble_functions(src)
        for m in re.finditer(r"\bC\.(\w+)", code):
            name = m.group(1)
            after = code[m.end():m.end() + 1]
            if name in CGO_BUILTINS or name in C_SCALARS:
                continue
            if name in local:
                got = call_args(code, m.end())
                assert got == local[name], f"{f}: C.{name} called with {got} args, preamble declares {local[name]}"
                continue
            if name.startswith("mp3g_") and after == "(" and name in protos:
                got = call_args(code, m.end())
                assert got == protos[name], f"{f}: C.{name} called with {got} args, header declares {protos[name]}"
            elif name.startswith("mp3g_"):
                assert re.search(r"\b%s\b" % name, hdr), f"{f}: C.{name} not in mp3g.h"
                if after == "(":  # a conversion to a header type, e.g. (*C.mp3g_granule)(...)
                    assert re.search(r"typedef struct %s\b" % name, hdr), f"{f}: C.{name}(...) unknown"
            elif name.startswith("MP3G_"):
                assert re.search(r"(#define\s+%s\b|\b%s\s*=)" % (name, name), hdr), f"{f}: C.{name} not in mp3g.h"
            else:
                raise AssertionError(f"{f}: unexpected C.{name}")


def test_struct_fields_written_by_the_shim_exist():
    ch = struct_fields("mp3g_channel")
    gr = struct_fields("mp3g_granule")
    st = struct_fields("mp3g_stream")
    src = _strip_comments(GO["frame_mp3g.go"])
    for fld in re.findall(r"\bc\.(\w+)", src):
        assert fld in ch, f"mp3g_channel has no field {fld}"
    for fld in re.findall(r"\bg\.(\w+)\s*=", src):
        assert fld in gr, f"mp3g_granule has no field {fld}"
    for go in GO.values():
        for lit in re.findall(r"C\.mp3g_stream\{([^}]*)\}", go):
            for fld in re.findall(r"(\w+)\s*:", lit):
                assert fld in st, f"mp3g_stream has no field {fld}"
        for fld in re.findall(r"\bs\.(first_granule|n_granules|flags)\b", go):
            assert fld in st
    # the fields Decode reads are all copied
    for fld in ("count1", "global_gain", "scalefac_scale", "preflag", "win_switch_flag", "block_type",
                "mixed_block_flag", "subblock_gain", "scalefac_l", "scalefac_s"):
        assert re.search(r"\bc\.%s\b" % fld, src), f"frame_mp3g.go does not copy {fld}"


def test_abi_version_matches():
    v = int(re.search(r"#define MP3G_ABI_VERSION (\d+)", HEADER).group(1))
    for f in ("frame_mp3g.go", "decoder_mp3g.go"):
        assert f"const ABIVersion = {v}" in GO[f], f
        assert f"ABI version {v}" in GO[f], f  # the header comment
    # both shims check the loaded library's version before using it
    assert "C.mp3g_abi_version()" in GO["frame_mp3g.go"]
    go = GO["decoder_mp3g.go"]
    assert re.search(r"C\.mp3g_abi_version\(\)\); v != ABIVersion", go)
    for fn in ("func NewDecoder(", "func NewDecoderBytes(", "func DecodeMany("):
        body = go[go.index(fn):]
        body = body[:body.index("\n}\n")]
        assert "checkABI()" in body, fn


def test_decoder_finalizer():
    """The reference Decoder has no Close (decode.go:34-43): the shim's
    decoders are released by a finalizer; Close clears it (idempotent)."""
    go = GO["decoder_mp3g.go"]
    assert "runtime.SetFinalizer(d, func(d *Decoder) { d.Close() })" in go
    assert go.count("return track(&Decoder{") == 2
    close_body = go[go.index("func (d *Decoder) Close() error {"):]
    assert "runtime.SetFinalizer(d, nil)" in close_body[:close_body.index("\n}\n")]


def test_streaming_reader_trampolines():
    """decoder_mp3g.go streams its io.Reader (ABI 3): the .c trampolines call
    exactly the Go functions the Go file exports, with the mp3g_reader
    callback signatures of the header, and hand the library the handle as the
    user value; NewDecoder no longer reads the whole input first."""
    csrc = open(os.path.join(REPO, "go", "reader_mp3g.c")).read()
    go = GO["decoder_mp3g.go"]
    assert csrc.startswith("//go:build mp3g")
    exported = set(re.findall(r"^//export (\w+)", go, flags=re.M))
    assert exported == {"mp3gGoRead", "mp3gGoSeek"}
    for fn in exported:
        assert re.search(r"\b%s\(\(uintptr_t\)user," % fn, csrc), fn
    # the callback shapes of mp3g_reader
    rd = re.search(r"typedef struct mp3g_reader \{(.*?)\} mp3g_reader;", _strip_comments(HEADER), flags=re.S).group(1)
    assert "int64_t (*read)(void* user, uint8_t* buf, size_t cap);" in rd
    assert "int64_t (*seek)(void* user, int64_t offset, int whence);" in rd
    assert "static int64_t goreader_read(void* user, uint8_t* buf, size_t cap)" in csrc
    assert "static int64_t goreader_seek(void* user, int64_t offset, int whence)" in csrc
    assert "mp3g_decoder_new_reader(&r, device, mode, out)" in csrc
    decl = re.search(r"int goreader_decoder_new\(([^)]*)\)", go).group(1)
    assert decl == re.search(r"int goreader_decoder_new\(([^)]*)\)", csrc).group(1)
    body = go[go.index("func NewDecoder("):go.index("func NewDecoderBytes(")]
    assert "io.ReadAll" not in body and "cgo.NewHandle" in body
