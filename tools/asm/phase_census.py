"""Static instruction census of rollout_kernel between the MPCR_PROFILE phase
stamps (s_memtime).  Diagnostic: tells which code a phase's dynamic count
comes from (loops are counted once).

    hipcc --offload-arch=gfx950 --cuda-device-only -S -O3 ... -DMPCR_PROFILE -o prof.s rollout.hip
    python tools/asm/phase_census.py prof.s [narrow|wide]
"""
import re
import sys
import collections

path = sys.argv[1]
which = sys.argv[2] if len(sys.argv) > 2 else "narrow"
tag = "ILi16ELi16ELi24ELb0E" if which == "narrow" else "ILi32ELi32ELi72ELb1E"
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith("_ZN4mpcr14rollout_kernel" + tag) and l.rstrip().endswith(":") or
             (l.startswith("_ZN4mpcr14rollout_kernel" + tag) and ": ;" in l))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]
seg, segs = collections.Counter(), []
for l in body:
    s = l.strip()
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        continue
    op = s.split()[0]
    if op == "s_memtime":
        segs.append(seg)
        seg = collections.Counter()
        continue
    cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith("s_load") and not
           op.startswith("s_waitcnt") and not op.startswith("s_cbranch") and not op.startswith("s_branch") else
           "smem" if op.startswith("s_load") else "lds" if op.startswith("ds_") else
           "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "ctl")
    seg[cls] += 1
    seg["all"] += 1
segs.append(seg)
for i, c in enumerate(segs):
    print(f"seg {i:2d}: " + " ".join(f"{k}={c[k]}" for k in ("all", "valu", "salu", "smem", "lds", "vmem", "ctl")))
