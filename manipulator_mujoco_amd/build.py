"""Build libmpcr.so in-tree for gfx950 (hipcc, no JIT caches).

    python -m manipulator_mujoco_amd.build
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# translation units and their own device flags: the rollout kernel is built
# without SLP vectorisation (packing scalar fp32 ops into v_pk_* pairs cost
# more register-pair v_movs than it saved there: 1328 -> 649 static v_mov,
# 126 -> 104 VGPRs, C3 2.59 -> 2.35 ms), the CEM step kernels keep it
# (sample_project 0.38 -> 0.30 ms with it)
# and is allowed to reassociate fp32 (-fassociative-math needs no signed zeros
# and no trapping; NaN / Inf semantics stay): 2.29 -> 2.25 ms, parity unchanged.
# The CEM TU does not get it (top-k orders -0 before +0 like the reference).
# rollout.hip is compiled twice: MPCR_TU=1, the single-arm kernels and the
# launch logic, with those flags; MPCR_TU=2, the dual-arm kernels, with the
# fast-math device flags dropped (_drop_fast: IEEE division / square root, no
# reassociation) -- the latency-bound dual arm pays ~5 % (C4 45.9 -> 48.3 ms)
# and its rollouts keep within the fp32 restatement's drift (C4 shard
# well-conditioned misses 22 -> 8); the VALU-bound C3 would pay 16 %.
_ROLLOUT_FLAGS = ["-Xarch_device", "-fno-slp-vectorize", "-Xarch_device", "-fassociative-math",
                  "-Xarch_device", "-fno-signed-zeros", "-Xarch_device", "-fno-trapping-math"]
UNITS = [(os.path.join(CSRC, "engine.hip"), []),
         (os.path.join(CSRC, "rollout.hip"), _ROLLOUT_FLAGS + ["-DMPCR_TU=1"]),
         (os.path.join(CSRC, "rollout.hip"), ["PRECISE"] + _ROLLOUT_FLAGS + ["-DMPCR_TU=2"])]
SRC = sorted({u for u, _ in UNITS})
DEPS = SRC + [os.path.join(CSRC, f) for f in ("rollout.h", "cem.hip", "comm.hip", "mpcr_device.h")] + [
    os.path.join(os.path.dirname(HERE), "include", f) for f in ("mpcr.h", "mpcr_model.h")]
OUT = os.path.join(HERE, "libmpcr.so")
ARCH = os.environ.get("MPCR_OFFLOAD_ARCH", "gfx950")
# fp32 '/' and sqrtf map to the 1-ulp hardware v_rcp/v_sqrt (not the ~10-op
# IEEE sequences); device code may also use a*rcp(b) without the frexp/ldexp
# range scaling (operands here are guarded away from denormals; 3.91 -> 3.67 ms
# on C3).  Every other fp semantic (NaN/Inf, no reassociation) stays, and the
# host's fp64 code (KKT inverse, model constants) is untouched.
# simplifycfg-sink-common=false: sinking the narrow phase's per-geometry-type
# slot stores into one store with a phi'd index forced the slot arrays into
# scratch (32 B/lane); without it they stay in registers (205 -> 179 VGPRs).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-pass-failed",
         "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-Xarch_device", "-freciprocal-math",
         "-Xarch_device", "-fapprox-func", "-mllvm", "-simplifycfg-sink-common=false"]


def source_hash() -> str:
    """sha256 over libmpcr.so's sources and compile flags: identifies the build
    a committed counter profile was taken from (bench.py attaches committed
    rocprof counters only to a run of the same build)."""
    import hashlib
    h = hashlib.sha256()
    for d in DEPS:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    h.update(repr((FLAGS, [f for _, f in UNITS])).encode())
    return h.hexdigest()[:16]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


# the fast-math device flags above, dropped by compile_lib(precise=True) for
# accuracy experiments (tools/build_variant.py --precise)
FAST_MATH = {"-freciprocal-math", "-fapprox-func", "-fassociative-math", "-fno-signed-zeros", "-fno-trapping-math"}


def _drop_fast(flags):
    out, skip = [], False
    for i, f in enumerate(flags):
        if skip:
            skip = False
            continue
        if f == "-Xarch_device" and i + 1 < len(flags) and flags[i + 1] in FAST_MATH:
            skip = True
            continue
        if f == "-fno-hip-fp32-correctly-rounded-divide-sqrt":
            continue
        out.append(f)
    return out


def compile_lib(out: str, extra=(), verbose: bool = False, precise: bool = False) -> str:
    """Compile every unit (FLAGS + its own + extra) and link the shared library.
    precise: without the fast-math device flags (IEEE division / sqrt, no
    reassociation) -- accuracy experiments only."""
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        objs = []
        for i, (src, unit_flags) in enumerate(UNITS):
            obj = os.path.join(tmp, f"{os.path.basename(src)}.{i}.o")
            fl = FLAGS + [f for f in unit_flags if f != "PRECISE"]
            if precise or "PRECISE" in unit_flags:
                fl = _drop_fast(fl)
            cmd = [hipcc(), f"--offload-arch={ARCH}", "-c"] + fl + list(extra) + ["-o", obj, src]
            if verbose:
                cmd.append("-Rpass-analysis=kernel-resource-usage")
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
            objs.append(obj)
        subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs, check=True)
    os.replace(out + ".tmp", out)
    return out


MJCF_SRC = os.path.join(CSRC, "mjcf_embed.cpp")
MJCF_OUT = os.path.join(HERE, "libmpcr_mjcf.so")


def compile_mjcf_lib(out: str = MJCF_OUT) -> str:
    """libmpcr_mjcf.so: the MJCF compiler (mjcf.py) in an embedded CPython,
    host C++ only (g++), dlopened by libmpcr.so for .xml model paths."""
    import sysconfig
    inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    cmd = [shutil.which("g++") or "g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{inc}", MJCF_SRC,
           f"-L{libdir}", f"-Wl,-rpath,{libdir}", f"-lpython{ver}", "-ldl", "-o", out + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if force or not os.path.exists(MJCF_OUT) or os.path.getmtime(MJCF_OUT) < os.path.getmtime(MJCF_SRC):
        # optional: libmpcr.so dlopens it only for .xml model paths and reports
        # "MJCF compiler unavailable" at run time when it is missing (a host
        # without Python headers or a shared libpython still builds the engine)
        try:
            compile_mjcf_lib()
        except (subprocess.CalledProcessError, OSError) as e:
            print(f"warning: libmpcr_mjcf.so not built ({e}); mpcr_model_load of .xml paths will be unavailable",
                  file=sys.stderr)
    if not force and os.path.exists(OUT):
        mt = os.path.getmtime(OUT)
        if all(os.path.getmtime(d) <= mt for d in DEPS):
            return OUT
    return compile_lib(OUT, verbose=verbose)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
