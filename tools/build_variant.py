"""Build libmpcr.so with extra compiler flags into build_variants/<name>.so
(for tools/ab_session.sh interleaved timing).

    python tools/build_variant.py NAME [--precise] [extra hipcc flags...]
--precise drops the fast-math device flags (IEEE division / sqrt, no reassociation).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from manipulator_mujoco_amd import build  # noqa: E402

name, extra = sys.argv[1], [a for a in sys.argv[2:] if a != "--precise"]
precise = "--precise" in sys.argv
out = os.path.join(ROOT, "build_variants", name + ".so")
os.makedirs(os.path.dirname(out), exist_ok=True)
build.compile_lib(out, extra, precise=precise)
print(out)
