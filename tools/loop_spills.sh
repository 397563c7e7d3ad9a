# Spill instructions inside the fast kernel's granule loop (the loop holding
# s_setprio 0) of build/kernels_fast.s: must print 0.
set -eu
F=${1:-go-mp3_amd/csrc/build/kernels_fast.s}
K=${2:-_ZN4mp3g2v319granule_fast_kernelILb0E}  # (a mangled-name prefix)
python3 - "$F" "$K" <<'PY'
import re, sys
f, k = sys.argv[1], sys.argv[2]
lines = open(f).read().split("\n")
i0 = next(i for i, l in enumerate(lines) if l.startswith(k) and l.split(";")[0].rstrip().endswith(":"))
i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[i0:i1]
sp = next(i for i, l in enumerate(body) if "s_setprio 0" in l)
# the innermost loop header before it, and its label (on that line or the one above)
h = max(i for i in range(sp) if "Loop Header" in body[i])
lab = next(re.match(r"^(\.LBB\w+):", body[j]).group(1) for j in (h, h - 1) if re.match(r"^\.LBB\w+:", body[j]))
e = max(i for i, l in enumerate(body) if re.search(r"s_(c?branch\w*) %s$" % re.escape(lab), l.strip()))
seg = body[h:e + 1]
spills = sum(bool(re.search(r"scratch_|v_readlane|v_writelane", l)) for l in seg)
instr = sum(bool(re.match(r"\s*(s_|v_|ds_|buffer_|global_)", l)) for l in seg)
print(f"loop {lab} lines {h}..{e}: {spills} spill ops, {instr} instructions")
PY
