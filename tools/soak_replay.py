#!/usr/bin/env python3
"""Replays a decoder case saved by tools/soak.py (gpurun_out/soak_fail/dec_*.{mp3,json})
on the product's decoder and the oracle's, printing every operation's results
side by side.  python tools/soak_replay.py gpurun_out/soak_fail/dec_4_0"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("go-mp3_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    import mp3g
    import oracle
    base = sys.argv[1]
    data = open(base + ".mp3", "rb").read()
    meta = json.load(open(base + ".json"))
    ops = meta["ops"]
    _, seekable, mode = ops[0][:3]
    if len(ops[0]) > 3 and ops[0][3]:
        print("(recorded on the streaming reader; replayed in memory)")
    o = oracle.Decoder(data, seekable=seekable)
    d = mp3g.Decoder(data, seekable=seekable, mode=mode)
    print(f"len {len(data)} seekable {seekable} mode {mode} length {d.length} / {o.length} "
          f"duration {getattr(d, 'duration_ns', None)} / {o.duration_ns}")
    for op in ops[1:]:
        if op[0] == "read":
            p, p2 = d.pos, o.pos
            st, b = d.read(op[1])
            st2, b2 = o.read(op[1])
            first = next((i for i in range(min(len(b), len(b2))) if b[i] != b2[i]), None)
            print(f"read {op[1]} at {p}/{p2}: status {st}/{st2} bytes {len(b)}/{len(b2)} first diff {first}"
                  + (f" ({b[first]:#04x} vs {b2[first]:#04x})" if first is not None else ""))
            if first is not None:
                import numpy as np
                a0 = p % 2
                m = (min(len(b), len(b2)) - a0) // 2 * 2
                x = np.frombuffer(b[a0:a0 + m], np.int16).astype(np.int32)
                y = np.frombuffer(b2[a0:a0 + m], np.int16).astype(np.int32)
                dd = np.abs(x - y)
                i = int(np.argmax(dd))
                print(f"   samples: max |diff| {int(dd.max())} at sample {i} (stream byte {p + a0 + 2 * i}), "
                      f"{int((dd > 0).sum())} differ; product {x[max(0, i - 2):i + 3].tolist()} "
                      f"oracle {y[max(0, i - 2):i + 3].tolist()}")
        elif op[0] == "seek":
            print(f"seek {op[1]} {op[2]}: {d.seek(op[1], op[2])} / {o.seek(op[1], op[2])}")
        elif op[0] == "seek_to_time_ns":
            print(f"seek_to_time_ns {op[1]}: {d.seek_to_time_ns(op[1])} / {o.seek_to_time_ns(op[1])}")
        else:
            print(f"seek_to_sample {op[1]}: {d.seek_to_sample(op[1])} / {o.seek_to_sample(op[1])}")
        print(f"   pos {d.pos}/{o.pos} position_ns {d.position_ns}/{o.position_ns}")


if __name__ == "__main__":
    main()
