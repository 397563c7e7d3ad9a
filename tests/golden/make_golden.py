#!/usr/bin/env python3
"""Generate the committed golden fixtures (run in the build container).

Inputs come from the reference's own test data (read-only at
/root/reference): the two sample streams under example/ and the regression
crasher corpus of fuzzing_test.go:22-107 (Go string literals decoded to their
bytes).  Expected outputs come from the oracle (oracle/, a C restatement of
the reference -- Go is not installed, so the reference itself cannot run).

Outputs (all under tests/golden/):
  classic_lame.mp3, mpeg2.mp3      copies of reference example/ data files
  fuzz/crasher_XX.bin              fuzzing_test.go inputs
  golden.json                      oracle PCM SHA-256 / lengths / properties
"""
import hashlib
import json
import os
import re
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402


def go_string_bytes(lit: str) -> bytes:
    """Decode the body of a Go interpreted string literal."""
    out = bytearray()
    i = 0
    while i < len(lit):
        ch = lit[i]
        if ch == "\\":
            e = lit[i + 1]
            if e == "x":
                out.append(int(lit[i + 2:i + 4], 16))
                i += 4
                continue
            if e == "u":
                out += chr(int(lit[i + 2:i + 6], 16)).encode("utf-8")
                i += 6
                continue
            simple = {"n": 10, "t": 9, "r": 13, "\\": 92, '"': 34, "0": 0}
            out.append(simple[e])
            i += 2
            continue
        out += ch.encode("utf-8")
        i += 1
    return bytes(out)


def fuzz_inputs():
    src = open(os.path.join(REF, "fuzzing_test.go")).read()
    body = src[src.index("inputs := []string{"):src.index("for _, input := range inputs")]
    body = re.sub(r"//[^\n]*", "", body)
    items = []
    for expr in body.split('",\n'):
        parts = re.findall(r'"((?:[^"\\]|\\.)*)"', expr)
        if parts:
            items.append(b"".join(go_string_bytes(p) for p in parts))
    return items


def main():
    os.makedirs(os.path.join(HERE, "fuzz"), exist_ok=True)
    for f in ("classic_lame.mp3", "mpeg2.mp3"):
        shutil.copyfile(os.path.join(REF, "example", f), os.path.join(HERE, f))
    crashers = fuzz_inputs()
    for k, b in enumerate(crashers):
        open(os.path.join(HERE, "fuzz", f"crasher_{k:02d}.bin"), "wb").write(b)
    gold = {"generator": "tests/golden/make_golden.py (oracle = C restatement; parity unpinned)",
            "files": {}, "fuzz": {}}
    for f in ("classic_lame.mp3", "mpeg2.mp3"):
        data = open(os.path.join(HERE, f), "rb").read()
        st, pcm, g, c = oracle.decode_all_capture(data)
        dec = oracle.Decoder(data)
        gold["files"][f] = {
            "status": st, "pcm_bytes": len(pcm), "pcm_sha256": hashlib.sha256(pcm).hexdigest(),
            "granules": int(len(g)), "frames": int(dec.n_frames), "sample_rate": int(dec.sample_rate),
            "length": int(dec.length), "duration_ns": int(dec.duration_ns),
            "descriptor_sha256": hashlib.sha256(g.tobytes()).hexdigest(),
            "coeff_sha256": hashlib.sha256(c.tobytes()).hexdigest(),
        }
    for k, b in enumerate(crashers):
        st, pcm = oracle.decode_all(b)
        gold["fuzz"][f"crasher_{k:02d}.bin"] = {"status": st, "pcm_bytes": len(pcm)}
    json.dump(gold, open(os.path.join(HERE, "golden.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(gold, indent=1)[:2000])


if __name__ == "__main__":
    main()
