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
      if f.endswith(".go") and not f.endswith("_test.go")}  # (cgo is not allowed in _test.go files)
GO_TESTS = {f: open(os.path.join(REPO, "go", f)).read() for f in sorted(os.listdir(os.path.join(REPO, "go")))
            if f.endswith("_test.go")}
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


# ---------------------------------------------------------------------------
# The drop-in inside the reference package (Missing 1).
#
# decoder_mp3g.go is package mp3 and declares Decoder, NewDecoder and the
# Decoder methods that the reference's decode.go declares too; the recipe
# (go/apply_mp3g.sh) gates decode.go with `//go:build !mp3g`, so each build
# compiles exactly one of them.  Without a Go toolchain the check is done on
# the declarations (tests/goparse.py): the recipe is applied to a scratch copy
# of the reference's package files, and each build's package scope -- tests
# included, since `go test` compiles them into the package -- must declare
# every identifier once.
import shutil  # noqa: E402
import subprocess  # noqa: E402

import pytest  # noqa: E402

import goparse  # noqa: E402

REF = "/root/reference"
needs_ref = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "decode.go")),
                               reason="the reference checkout is not on this machine")
TAGS = {"linux", "amd64", "cgo", "gc"}


def _pkg_files(root, sub=""):
    d = os.path.join(root, sub)
    return {f: open(os.path.join(d, f)).read() for f in sorted(os.listdir(d)) if f.endswith(".go")}


def _applied(tmp_path):
    """The recipe run on a scratch checkout holding the reference's package
    mp3 and internal/frame files (read from /root/reference, written to tmp)."""
    dst = tmp_path / "go-mp3"
    (dst / "internal" / "frame").mkdir(parents=True)
    for f in os.listdir(REF):
        if f.endswith(".go"):
            shutil.copy(os.path.join(REF, f), dst / f)
    for f in os.listdir(os.path.join(REF, "internal", "frame")):
        shutil.copy(os.path.join(REF, "internal", "frame", f), dst / "internal" / "frame" / f)
    r = subprocess.run(["sh", os.path.join(REPO, "go", "apply_mp3g.sh"), str(dst), "/nonexistent.so"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return dst


def _duplicates(files, tags):
    scope, methods = goparse.package_scope(files, tags)
    dup = {k: v for k, v in scope.items() if len(v) > 1}
    dup.update({f"{k[0]}.{k[1]}": v for k, v in methods.items() if len(v) > 1})
    return dup


@needs_ref
def test_recipe_gates_decode_go_and_every_build_declares_each_identifier_once(tmp_path):
    dst = _applied(tmp_path)
    mp3 = _pkg_files(dst)
    frame = _pkg_files(dst, "internal/frame")
    assert goparse.build_constraint(mp3["decode.go"]) == "!mp3g"
    assert {"decoder_mp3g.go", "decoder_mp3g_test.go"} <= set(mp3) and "frame_mp3g.go" in frame
    assert os.path.isfile(dst / "reader_mp3g.c") and os.path.isfile(dst / "third_party/mp3g/include/mp3g.h")
    for tags in (TAGS | {"mp3g"}, TAGS):
        for name, files in (("mp3", mp3), ("frame", frame)):
            assert _duplicates(files, tags) == {}, (name, sorted(tags))
            pk = {goparse.declarations(src)["package"] for f, src in files.items()
                  if goparse.build_ok(goparse.declarations(src)["build"], tags)}
            assert pk == {name}
    # with the tag the Decoder is the shim's; without it the reference's
    scope, _ = goparse.package_scope(mp3, TAGS | {"mp3g"})
    assert scope["Decoder"] == ["decoder_mp3g.go"] and scope["NewDecoder"] == ["decoder_mp3g.go"]
    assert scope["source"] == ["source.go"]  # kept: time_seek_test.go uses it
    scope, _ = goparse.package_scope(mp3, TAGS)
    assert scope["Decoder"] == ["decode.go"] and "readerState" not in scope
    # idempotent: a second run leaves decode.go with one gate
    r = subprocess.run(["sh", os.path.join(REPO, "go", "apply_mp3g.sh"), str(dst), "/nonexistent.so"],
                       capture_output=True, text=True)
    assert r.returncode == 0 and open(dst / "decode.go").read().count("//go:build") == 1


@needs_ref
def test_without_the_gate_the_collision_is_found(tmp_path):
    """The check above has teeth: decode.go without its gate redeclares the
    shim's identifiers under the mp3g tag (what `go build -tags mp3g` reports
    as "Decoder redeclared in this block")."""
    dst = _applied(tmp_path)
    src = open(dst / "decode.go").read()
    open(dst / "decode.go", "w").write(src.split("\n", 2)[2])  # drop the gate line and its blank line
    dup = _duplicates(_pkg_files(dst), TAGS | {"mp3g"})
    assert {"Decoder", "NewDecoder", "Decoder.Read", "Decoder.Seek"} <= set(dup)


def _exported_methods(src, recv):
    return {f["name"]: (f["params"], f["results"]) for f in goparse.declarations(src)["funcs"]
            if f["recv"] == recv and f["name"][0].isupper()}


@needs_ref
def test_shim_decoder_api_equals_the_reference():
    """The exported API of package mp3 (decode.go:70-361) with the same
    parameter and result types; the shim adds only Close, ReadFull (methods)
    and NewDecoderBytes, DecodeMany, Mode, ABIVersion (package scope)."""
    ref = open(os.path.join(REF, "decode.go")).read()
    shim = GO["decoder_mp3g.go"]
    rm, sm = _exported_methods(ref, "Decoder"), _exported_methods(shim, "Decoder")
    assert len(rm) == 14
    assert set(sm) - set(rm) == {"Close", "ReadFull"}
    for name, sig in rm.items():
        assert sm.get(name) == sig, (name, sig, sm.get(name))
    rf = {f["name"]: (f["params"], f["results"]) for f in goparse.declarations(ref)["funcs"] if f["recv"] is None}
    sf = {f["name"]: (f["params"], f["results"]) for f in goparse.declarations(shim)["funcs"] if f["recv"] is None}
    assert rf["NewDecoder"] == sf["NewDecoder"] == (["io.Reader"], ["*Decoder", "error"])
    ref_scope, _ = goparse.package_scope({"decode.go": ref}, TAGS)
    shim_scope, _ = goparse.package_scope({"d.go": shim}, TAGS | {"mp3g"})
    exported = lambda sc: {k for k in sc if k[0].isupper()}  # noqa: E731
    assert exported(shim_scope) - exported(ref_scope) == {"NewDecoderBytes", "DecodeMany", "Mode", "ABIVersion"}
    assert exported(ref_scope) <= exported(shim_scope)


@needs_ref
def test_reference_tests_use_only_what_the_shim_declares():
    """`go test -tags mp3g` compiles the reference's own tests against the
    shim: they may use no unexported identifier of decode.go (its Decoder
    fields and helpers, invalidLength) -- checked on every variable bound to
    a NewDecoder result and on package-scope names."""
    ref = open(os.path.join(REF, "decode.go")).read()
    d = goparse.declarations(ref)
    private_methods = {f["name"] for f in d["funcs"] if f["recv"] == "Decoder" and not f["name"][0].isupper()}
    body = re.search(r"type Decoder struct \{(.*?)\n\}", ref, flags=re.S).group(1)
    fields = set(re.findall(r"^\s*(\w+)\s", body, flags=re.M))
    assert {"readFrame", "bytesToDuration"} <= private_methods and {"frame", "buf", "pos"} <= fields
    private_scope = {n for n in d["values"] + d["types"] if not n[0].isupper()}
    shim_scope, shim_methods = goparse.package_scope({"d.go": GO["decoder_mp3g.go"]}, TAGS | {"mp3g"})
    n_tests = 0
    for f, src in _pkg_files(REF).items():
        if not f.endswith("_test.go"):
            continue
        n_tests += 1
        code = goparse.tokens(src)
        idents = {t[1] for t in code if t[0] == "ident"}
        for nm in private_scope:
            assert nm not in idents or nm in shim_scope, (f, nm)
        decs = set(re.findall(r"(\w+)\s*,\s*\w+\s*:?=\s*NewDecoder\(", src))
        for i in range(len(code) - 2):
            if code[i][1] in decs and code[i + 1][1] == ".":
                sel = code[i + 2][1]
                if not sel[0].isupper():
                    assert sel not in private_methods | fields or ("Decoder", sel) in shim_methods, (f, sel)
    assert n_tests == 5


def test_go_imports_are_used():
    """`imported and not used` is a compile error in Go."""
    for f, src in {**GO, **GO_TESTS}.items():
        imp = re.search(r'^import \((.*?)^\)', src, flags=re.S | re.M).group(1)
        code = _strip_comments(src.split(imp, 1)[1])
        for path in re.findall(r'"([^"]+)"', imp):
            name = path.rsplit("/", 1)[-1]
            assert re.search(r"\b%s\." % name, code), (f, path)


def test_reference_fields_read_by_the_frame_shim_exist():
    """frame_mp3g.go (package frame) reads Frame's header / sideInfo /
    mainData and the SideInfo / MainData fields Decode reads."""
    if not os.path.isdir(os.path.join(REF, "internal")):
        pytest.skip("the reference checkout is not on this machine")
    src = _strip_comments(GO["frame_mp3g.go"])

    def fields(path, typ):
        t = open(os.path.join(REF, path)).read()
        body = re.search(r"type %s struct \{(.*?)\n\}" % typ, t, flags=re.S).group(1)
        return set(re.findall(r"^\s*(\w+)\s", body, flags=re.M))
    assert set(re.findall(r"\bf\.(\w+)", src)) <= fields("internal/frame/frame.go", "Frame")
    assert set(re.findall(r"\bsi\.(\w+)", src)) <= fields("internal/sideinfo/sideinfo.go", "SideInfo")
    assert set(re.findall(r"\bf\.mainData\.(\w+)", src)) <= fields("internal/maindata/maindata.go", "MainData")


def test_decoder_methods_keep_the_receiver_alive():
    """a method that passes d.d to the library keeps d reachable
    until the call returns, or the finalizer can free the decoder (and delete
    the callbacks' cgo.Handle) during a GC inside a reader callback."""
    d = goparse.declarations(GO["decoder_mp3g.go"])
    n = 0
    for fn in d["funcs"]:
        if fn["recv"] == "Decoder" and fn["body"] and re.search(r"C \. mp3g_decoder_\w+ \(.*\bd \. d\b", fn["body"]):
            if fn["name"] == "Close":  # clears the finalizer before the call
                assert fn["body"].startswith("{ runtime . SetFinalizer ( d , nil )")
                continue
            assert fn["body"].startswith("{ defer runtime . KeepAlive ( d )"), fn["name"]
            n += 1
    assert n == 13
    t = GO_TESTS["decoder_mp3g_test.go"]
    assert t.startswith("//go:build mp3g") and "runtime.GC()" in t and "package mp3" in t
    # its helpers do not collide with the reference's tests (same package)
    names = {f["name"] for f in goparse.declarations(t)["funcs"] if f["recv"] is None} | \
        set(goparse.declarations(t)["types"])
    assert all(n.startswith(("mp3g", "TestMP3G_")) for n in names), names


def _integration_go_blocks():
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    assert doc.count("```") % 2 == 0, "unbalanced code fence in INTEGRATION.md"
    return re.findall(r"```go\n(.*?)```", doc, flags=re.S)


def test_integration_md_go_blocks_match_the_shims():
    """Every function INTEGRATION.md shows in a Go block is the shim's own:
    same receiver, parameter and result types, and the same body token for
    token (so the document cannot drift from the code it describes)."""
    shim = {}
    for f, src in GO.items():
        for fn in goparse.declarations(src)["funcs"]:
            shim[(fn["recv"], fn["name"])] = fn
    blocks = _integration_go_blocks()
    assert len(blocks) >= 3
    shown = 0
    for b in blocks:
        if b.startswith("// (fragment"):
            continue  # statements, not declarations
        src = b if re.match(r"\s*(//go:build[^\n]*\n\s*)?package ", b) else "package x\n" + b
        for fn in goparse.declarations(src)["funcs"]:
            key = (fn["recv"], fn["name"])
            assert key in shim, f"INTEGRATION.md shows {key}, which no shim declares"
            s = shim[key]
            assert (fn["params"], fn["results"]) == (s["params"], s["results"]), key
            assert fn["body"] == s["body"], f"INTEGRATION.md's {key} differs from the shim's"
            shown += 1
    assert shown >= 8
