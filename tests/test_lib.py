"""The C ABI library: loads here (no GPU), exports every symbol include/mpcr.h
declares, validates model blobs, and fails loudly without a gfx950 device."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from manipulator_mujoco_amd import _lib, models


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "mpcr.h")).read()
    decl = r"^(?:int|void|const char\*)\s+(mpcr_[a-z_]+)\s*\("
    return sorted(set(re.findall(decl, src, flags=re.M)))


def test_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_symbols()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(_lib.EXPORTS) <= set(names)
    assert lib.mpcr_abi_version() == 1


def test_model_blob_roundtrip_and_rejects_garbage():
    lib = _lib.load()
    m = models.load("scene_mjx", 0.05)
    blob = m.to_blob()
    h = ctypes.c_void_p()
    assert lib.mpcr_model_from_blob(blob, len(blob), ctypes.byref(h)) == 0
    nq, nv, ns, nc, npair = (ctypes.c_int() for _ in range(5))
    assert lib.mpcr_model_info(h, *(ctypes.byref(x) for x in (nq, nv, ns, nc, npair))) == 0
    assert (nq.value, nv.value, ns.value, nc.value, npair.value) == (15, 14, 87, 6, 59)
    lib.mpcr_model_free(h)
    bad = bytearray(blob)
    bad[0] ^= 0xFF
    assert lib.mpcr_model_from_blob(bytes(bad), len(bad), ctypes.byref(h)) == -2
    assert b"magic" in lib.mpcr_last_error()
    assert lib.mpcr_model_from_blob(blob[:-8], len(blob) - 8, ctypes.byref(h)) == -2


def test_model_file_load(tmp_path):
    lib = _lib.load()
    p = tmp_path / "m.mpcrm"
    models.load("planner_scene").save(str(p))
    h = ctypes.c_void_p()
    assert lib.mpcr_model_load(str(p).encode(), 0.05, ctypes.byref(h)) == 0
    lib.mpcr_model_free(h)


def test_key_decode_roundtrip():
    from manipulator_mujoco_amd import dist
    for c, i in ((1.5, 3), (-2.0, 7), (0.0, 0), (float("inf"), 12), (float("nan"), 5)):
        k = dist.ordered_key(c, i)
        idx, val = _lib.decode_key(k)
        assert idx == i
        assert (np.isnan(val) and np.isnan(c)) or val == np.float32(c)
        assert dist.decode_key(k)[0] == i
    keys = [dist.ordered_key(c, i) for i, c in enumerate([3.0, -1.0, float("nan"), -1.0, 2.0])]
    assert min(keys) == keys[2]          # NaN wins (argmin semantics)
    keys[2] = dist.ordered_key(5.0, 2)
    assert min(keys) == keys[1]          # ties -> first index


def test_engine_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from manipulator_mujoco_amd import basis
    from manipulator_mujoco_amd.engine import Engine
    _, _, Pd, _ = basis.planner_basis(20, 0.05)
    with pytest.raises(_lib.MpcrError):
        Engine(models.load("planner_scene", 0.05), 20, 8, Pd)
