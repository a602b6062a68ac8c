"""ctypes binding of libmpcr (include/mpcr.h).

The shared library is built in-tree by ``__graft_entry__.build()`` /
``python -m manipulator_mujoco_amd.build``.  There is deliberately no CPU
fallback: if the library or a gfx950 device is missing, every entry point
raises.
"""

from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPCR_LIB") or os.path.join(_HERE, "libmpcr.so")  # MPCR_LIB: A/B builds (tools/)

MPCR_LAYOUT_XI = 0
MPCR_LAYOUT_THETADOT = 1
MPCR_F_DEVICE_PTRS = 1
MPCR_F_RESET_BEST = 2
MPCR_F_SYNC = 4

# every symbol include/mpcr.h declares (tests check the exports)
EXPORTS = (
    "mpcr_last_error", "mpcr_abi_version", "mpcr_device_arch", "mpcr_model_from_blob", "mpcr_model_load",
    "mpcr_model_set_timestep", "mpcr_model_info", "mpcr_model_free", "mpcr_engine_create", "mpcr_engine_free",
    "mpcr_rollout_cost", "mpcr_argmin", "mpcr_best_key_decode", "mpcr_topk", "mpcr_cem_create", "mpcr_cem_free",
    "mpcr_cem_factor", "mpcr_cem_sample_project", "mpcr_project", "mpcr_cem_update", "mpcr_rollout_cost_dp",
    "mpcr_plant_create", "mpcr_plant_free", "mpcr_plant_set_state", "mpcr_plant_get_state", "mpcr_plant_step",
    "mpcr_rollout_occupancy", "mpcr_set_two_wave_max_n", "mpcr_engine_dispatches", "mpcr_comm_unique_id", "mpcr_comm_init", "mpcr_comm_free", "mpcr_comm_allreduce_key",
    "mpcr_comm_allgather", "mpcr_comm_gather_elites", "mpcr_model_hull_starts", "mpcr_set_hull_start_scramble",
)
_VOID = ("mpcr_last_error", "mpcr_model_free", "mpcr_engine_free", "mpcr_best_key_decode", "mpcr_cem_free",
         "mpcr_plant_free", "mpcr_comm_free")

_lib = None


class MpcrError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpcrError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    # torch's HIP runtime first: torch links an unversioned libamdhip64.so of
    # its own, libmpcr the system's libamdhip64.so.7 (the same SONAME).  Loaded
    # in this order libmpcr binds to torch's copy; the other way round the
    # process holds two HIP runtimes and libmpcr's finds no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    vp, i, d, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_float
    P = ctypes.POINTER
    lib.mpcr_last_error.restype = ctypes.c_char_p
    lib.mpcr_abi_version.restype = i
    lib.mpcr_device_arch.argtypes = [i, ctypes.c_char_p, i]
    lib.mpcr_model_from_blob.argtypes = [vp, ctypes.c_size_t, P(vp)]
    lib.mpcr_model_load.argtypes = [ctypes.c_char_p, d, P(vp)]
    lib.mpcr_model_set_timestep.argtypes = [vp, d]
    lib.mpcr_model_info.argtypes = [vp, P(i), P(i), P(i), P(i), P(i)]
    lib.mpcr_model_free.argtypes = [vp]
    lib.mpcr_model_free.restype = None
    lib.mpcr_engine_create.argtypes = [vp, i, i, i, vp, i, P(vp)]
    lib.mpcr_engine_free.argtypes = [vp]
    lib.mpcr_engine_free.restype = None
    lib.mpcr_rollout_cost.argtypes = [vp, vp, i, i, P(d), P(f), P(f), P(f), vp, vp, vp, vp, i, vp, i, vp]
    lib.mpcr_rollout_trace.argtypes = [vp, vp, i, i, P(d), P(f), P(f), P(f), vp, vp, vp, vp]
    lib.mpcr_argmin.argtypes = [vp, vp, i, i, i, vp, P(i), P(f), i, vp]
    lib.mpcr_best_key_decode.argtypes = [ctypes.c_uint64, P(i), P(f)]
    lib.mpcr_best_key_decode.restype = None
    lib.mpcr_topk.argtypes = [vp, vp, i, i, i, vp, i, vp]
    u64 = ctypes.c_uint64
    lib.mpcr_cem_create.argtypes = [i, i, i, i, vp, vp, vp, vp, i, P(vp)]
    lib.mpcr_cem_free.argtypes = [vp]
    lib.mpcr_cem_free.restype = None
    lib.mpcr_cem_factor.argtypes = [vp, vp, f, i, vp]
    lib.mpcr_cem_sample_project.argtypes = [vp, i, vp, u64, u64, i, vp, vp, vp, i, i, P(f), f, vp, i, vp]
    lib.mpcr_project.argtypes = [vp, vp, vp, i, i, i, P(f), f, vp, i, vp]
    lib.mpcr_cem_update.argtypes = [vp, vp, i, vp, i, vp, i, f, f, f, f, vp, vp, i, vp]
    lib.mpcr_rollout_cost_dp.argtypes = [vp, vp, i, i, vp, vp, vp, vp, vp, i, vp, i, vp]
    lib.mpcr_plant_create.argtypes = [vp, i, P(vp)]
    lib.mpcr_plant_free.argtypes = [vp]
    lib.mpcr_plant_free.restype = None
    lib.mpcr_plant_set_state.argtypes = [vp, P(d), P(d), P(d)]
    lib.mpcr_plant_get_state.argtypes = [vp, P(d), P(d), P(d), P(d)]
    lib.mpcr_plant_step.argtypes = [vp, P(d), i, vp]
    lib.mpcr_rollout_occupancy.argtypes = [i, P(i)]
    lib.mpcr_set_two_wave_max_n.argtypes = [i]
    lib.mpcr_engine_dispatches.argtypes = [vp, i, P(i)]
    lib.mpcr_plant_step_debug.argtypes = [vp, P(d), vp, i]
    lib.mpcr_plant_dbg_size.argtypes = []
    lib.mpcr_comm_unique_id.argtypes = [ctypes.c_char_p]
    lib.mpcr_comm_init.argtypes = [i, i, ctypes.c_char_p, i, P(vp)]
    lib.mpcr_comm_free.argtypes = [vp]
    lib.mpcr_comm_free.restype = None
    lib.mpcr_comm_allreduce_key.argtypes = [vp, vp, i, vp]
    lib.mpcr_comm_allgather.argtypes = [vp, vp, vp, ctypes.c_size_t, vp]
    lib.mpcr_comm_gather_elites.argtypes = [vp, vp, vp, i, i, i, vp, vp, vp]
    lib.mpcr_model_hull_starts.argtypes = [vp, i, P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_uint8), ctypes.c_int64]
    lib.mpcr_set_hull_start_scramble.argtypes = [u64]
    for name in EXPORTS + ("mpcr_rollout_trace", "mpcr_plant_step_debug", "mpcr_plant_dbg_size"):
        if name not in _VOID:
            getattr(lib, name).restype = i
    lib.mpcr_model_hull_starts.restype = ctypes.c_int64
    lib.mpcr_set_hull_start_scramble.restype = u64
    _lib = lib
    return lib


def check(rc: int):
    if rc != 0:
        msg = load().mpcr_last_error().decode(errors="replace")
        raise MpcrError(f"libmpcr error {rc}: {msg}")


def decode_key(key: int):
    idx = ctypes.c_int()
    val = ctypes.c_float()
    load().mpcr_best_key_decode(ctypes.c_uint64(key), ctypes.byref(idx), ctypes.byref(val))
    return idx.value, val.value
