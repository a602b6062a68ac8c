"""Static instruction census of rollout_kernel by source region (diagnostic).

Compile the device code with line tables, e.g.
    hipcc --offload-arch=gfx950 --cuda-device-only -S -O3 -gline-tables-only <FLAGS> -o ship.s csrc/rollout.hip
    python tools/asm/line_census.py ship.s [narrow|wide]
Each instruction is charged to the last rollout.hip line (.loc file 0) seen
before it; lines are grouped into the enclosing __device__ helper, or, inside
the kernel body, into the phase between two STAMP(k) markers.  Loop bodies
count once (static), so multiply by trip counts when reading.
"""
import collections
import os
import re
import sys

path = sys.argv[1]
which = sys.argv[2] if len(sys.argv) > 2 else "narrow"
tag = "ILi16ELi16ELi24ELb0E" if which == "narrow" else "ILi32ELi32ELi72ELb1E"
src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "manipulator_mujoco_amd", "csrc",
                        "rollout.hip")).read().splitlines()
# regions: helper functions (by signature line) and kernel phases (by STAMP)
regions = []  # (start_line, name)
kern = None
for i, l in enumerate(src, 1):
    m = re.match(r"^(?:template <[^>]*>\s*)?__(?:device|global)__[^(]*?\b(\w+)\s*\(", l)
    if m:
        regions.append((i, m.group(1)))
        if "__global__" in l:
            kern = i
    m = re.search(r"STAMP\((\d+)\);", l)
    if m and kern and i > kern:
        regions.append((i, f"kernel@after-STAMP{m.group(1)}"))
    if re.match(r"^template <", l) and i + 1 <= len(src) and "__device__" in src[i]:
        pass
regions.sort()


def region(line):
    name = "?"
    for s, n in regions:
        if s <= line:
            name = n
        else:
            break
    return name


lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith("_ZN4mpcr14rollout_kernel" + tag) and ":" in l)
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
cur = 0
per = collections.defaultdict(collections.Counter)
for l in lines[start:end]:
    s = l.strip()
    if s.startswith(".loc"):
        f = s.split()
        if f[1] == "0":
            cur = int(f[2])
        continue
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        continue
    op = s.split()[0]
    cls = ("valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else
           "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "smem" if op.startswith("s_load") else
           "ctl" if op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_barrier", "s_nop")) else "salu")
    r = region(cur)
    per[r][cls] += 1
    per[r]["all"] += 1
tot = collections.Counter()
for r, c in sorted(per.items(), key=lambda kv: -kv[1]["all"]):
    tot.update(c)
    print(f"{r:34s} " + " ".join(f"{k}={c[k]:5d}" for k in ("all", "valu", "salu", "lds", "vmem", "smem", "ctl")))
print(f"{'TOTAL':34s} " + " ".join(f"{k}={tot[k]:5d}" for k in ("all", "valu", "salu", "lds", "vmem", "smem", "ctl")))
