#!/bin/bash
# Device assembly of the rollout kernels (CPU container) and, per function,
# the flat / global / scratch memory instruction counts:  tools/kasm.sh [-D...]
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 --cuda-device-only -S -O3 -std=c++17 -fno-hip-fp32-correctly-rounded-divide-sqrt \
  -freciprocal-math -fapprox-func -mllvm -simplifycfg-sink-common=false -fno-slp-vectorize -fassociative-math \
  -fno-signed-zeros -fno-trapping-math "$@" -o /tmp/rollout.s manipulator_mujoco_amd/csrc/rollout.hip 2>/dev/null || exit 1
python3 - <<'PY'
import re
lines = open("/tmp/rollout.s").read().split("\n")
funcs = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)] + [(len(lines), "END")]
pats = {"flat ld": r"\bflat_load", "st": r"\bflat_store", "| global ld": r"\bglobal_load", "st ": r"\bglobal_store",
        "| scratch ld": r"\bscratch_load", " st": r"\bscratch_store", "| ds": r"\bds_"}
for (i, name), (j, _) in zip(funcs, funcs[1:]):
    b = lines[i:j]
    cnt = {k: sum(1 for l in b if re.search(p, l)) for k, p in pats.items()}
    print(f"{name[14:58]:44s} " + " ".join(f"{k} {v:4d}" for k, v in cnt.items()))
PY
