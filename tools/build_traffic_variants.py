"""Build the traffic-attribution variants of libmpcr.so into build_variants/
(CPU container; the GPU session's `traffic` step runs FETCH_SIZE / WRITE_SIZE
passes on each).  Diagnostic builds only, never shipped:
  t_ship   the shipped flags
  t_jl96   every J row of the narrow image in LDS (no HBM J slab)
  t_cprev  the previous-step slot distances in LDS (no HBM slot history)
  t_both   both (LDS images over the 16-blocks budget: fewer blocks per CU,
           so only the counters, not the times, mean anything)
  t_nopace pacing off (its slot table's loads and stores)"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from manipulator_mujoco_amd import build  # noqa: E402

VARIANTS = {
    "t_ship": [],
    "t_jl96": ["-DMPCR_N_JL=96", "-DMPCR_N_LDS_UNCHECKED"],
    "t_cprev": ["-DMPCR_N_CPREV_GLOBAL=0", "-DMPCR_N_LDS_UNCHECKED"],
    "t_both": ["-DMPCR_N_JL=96", "-DMPCR_N_CPREV_GLOBAL=0", "-DMPCR_N_LDS_UNCHECKED"],
    "t_nopace": ["-DMPCR_PACE=0"],
}

if __name__ == "__main__":
    os.makedirs(os.path.join(ROOT, "build_variants"), exist_ok=True)
    names = sys.argv[1:] or list(VARIANTS)
    with ThreadPoolExecutor(4) as ex:
        for out in ex.map(lambda v: build.compile_lib(os.path.join(ROOT, "build_variants", v + ".so"), VARIANTS[v]),
                          names):
            print(out)
