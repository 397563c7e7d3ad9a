#!/usr/bin/env python3
"""Timeline of the pipelined batch drop-in (mp3g_decode_streams_into) from a
rocprofv3 --kernel-trace --memory-copy-trace run of tools/pipe_time.py, as a
small JSON under profiles/ (the raw traces stay in gpurun_out/).

  tools/summarize_pipe.py <trace dir> <out.json> [calls]

The trace holds `calls` (default 3) decode_streams_into calls with the same
number of main-data launches each; the last call runs from the first event
after the previous call's last PCM copy-out kernel to the end.  Within it, the
busy time of each kind of
work (host->device copies, main-data kernels, DSP kernels incl. the zone
launch, PCM copy-out kernels, device->host DMA copies) and how much of the span
has two or more of them running at once.
"""
import csv
import json
import os
import sys


def intervals(rows, key):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if key(r))


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in union(iv))


def main():
    src, dst = sys.argv[1:3]
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ker = list(csv.DictReader(open(os.path.join(src, "run_kernel_trace.csv"))))
    cpy = list(csv.DictReader(open(os.path.join(src, "run_memory_copy_trace.csv"))))
    kinds = {
        "main_data_kernel": intervals(ker, lambda r: "huffman" in r["Kernel_Name"]),
        "dsp_kernel": intervals(ker, lambda r: "granule_" in r["Kernel_Name"]),
        "copy_out_kernel": intervals(ker, lambda r: "copy_out" in r["Kernel_Name"]),
        "h2d_copy": intervals(cpy, lambda r: r["Direction"].endswith("HOST_TO_DEVICE")),
        "d2h_copy": intervals(cpy, lambda r: r["Direction"].endswith("DEVICE_TO_HOST")),
    }
    # the last call: everything after the previous call's last copy-out kernel
    # (a time gap does not separate calls: the next call's uploads can start
    # while the host is still draining the previous one)
    outs = kinds["copy_out_kernel"]
    per = len(outs) // calls
    if per * calls != len(outs) or len(kinds["main_data_kernel"]) != calls * (len(kinds["main_data_kernel"]) // calls):
        sys.exit(f"launch counts do not split into {calls} equal calls")
    prev_end = max(b for a, b in outs[: per * (calls - 1)]) if calls > 1 else 0
    allv = union([iv for v in kinds.values() for iv in v if iv[0] >= prev_end])
    start = allv[0][0]
    end = max(b for a, b in allv)
    clip = {k: [(max(a, start), min(b, end)) for a, b in v if a >= start] for k, v in kinds.items()}
    # time with >= 2 kinds active
    ev = []
    for k, v in clip.items():
        for a, b in union(v):
            ev += [(a, 1), (b, -1)]
    ev.sort()
    active, last, multi = 0, start, 0
    for t, d in ev:
        if active >= 2:
            multi += t - last
        active += d
        last = t
    span = end - start
    out = {
        "source": src, "span_ms": round(span / 1e6, 2),
        "busy_ms": {k: round(length(v) / 1e6, 2) for k, v in clip.items()},
        "launches": {k: len(v) for k, v in clip.items()},
        "two_or_more_active_ms": round(multi / 1e6, 2),
        "note": "the last mp3g_decode_streams_into call of tools/pipe_time.py (c3: 1,024 streams x 1,024 frames, "
                "fast mode); busy = union of each kind's intervals within the call",
    }
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
