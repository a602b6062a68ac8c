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
    decl = r"^(?:int|void|const char\*|u?int64_t)\s+(mpcr_[a-z_]+)\s*\("
    return sorted(set(re.findall(decl, src, flags=re.M)))


def test_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_symbols()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(_lib.EXPORTS) <= set(names)
    assert lib.mpcr_abi_version() == 4  # v4: engine-built hull start tables (include/mpcr.h)


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


def test_c_host_loads_mjcf(tmp_path):
    """§8b: a host with no Python of its own loads a scene from its MJCF
    through the C ABI (mpcr_model_load on an .xml path -> the embedded
    compiler of libmpcr_mjcf.so), replacing MjModel.from_xml_path
    (SBP/mjx_planner.py:100-103).  The sizes match the Python compiler's."""
    import shutil
    import subprocess

    from manipulator_mujoco_amd import mjcf
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no C compiler")
    exe = tmp_path / "mjcf_host"
    subprocess.run([gcc, "-O1", "-o", str(exe), os.path.join(ROOT, "tests", "c_host", "mjcf_host.c"), "-ldl"],
                   check=True)
    xml = tmp_path / "scene.xml"
    xml.write_text("""<mujoco><option timestep="0.01"/><worldbody>
      <geom name="floor" type="plane" size="1 1 0.1"/>
      <body name="a" pos="0 0 0.5"><joint type="hinge" axis="0 1 0"/><geom type="capsule" size="0.05 0.2"/>
        <body name="b" pos="0 0 0.4"><joint type="slide" axis="1 0 0" range="-0.1 0.1"/><geom type="box" size="0.05 0.05 0.05"/></body>
      </body></worldbody></mujoco>""")
    libpath = os.path.join(ROOT, "manipulator_mujoco_amd", "libmpcr.so")
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    r = subprocess.run([str(exe), libpath, str(xml), "0.05"], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    m = mjcf.compile_mjcf(str(xml), 0.05)
    assert r.stdout.strip() == f"nq={m.nq} nv={m.nv} nslot={m.nslot} nctrl={m.nctrl} npair={m.npair}"
    # a broken file comes back as an error code, not a crash
    bad = tmp_path / "bad.xml"
    bad.write_text("<mujoco><worldbody><body></mujoco>")
    r = subprocess.run([str(exe), libpath, str(bad), "0.05"], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 5 and "MJCF" in r.stderr


def test_mjcf_load_through_ctypes(tmp_path):
    """The same entry from a Python host (ctypes): the blob the embedded
    compiler returns equals the Python compiler's struct byte for byte."""
    from manipulator_mujoco_amd import mjcf
    xml = tmp_path / "s.xml"
    xml.write_text('<mujoco><worldbody><body pos="0 0 1"><freejoint/><geom type="sphere" size="0.1"/></body>'
                   '</worldbody></mujoco>')
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.mpcr_model_load(str(xml).encode(), 0.02, ctypes.byref(h)))
    info = [ctypes.c_int() for _ in range(5)]
    _lib.check(lib.mpcr_model_info(h, *(ctypes.byref(x) for x in info)))
    m = mjcf.compile_mjcf(str(xml), 0.02)
    assert [x.value for x in info] == [m.nq, m.nv, m.nslot, m.nctrl, m.npair]
    lib.mpcr_model_free(h)
    assert mjcf.compile_blob(str(xml), 0.02) == bytes(m.to_struct())


def test_mjcf_library_exports_its_header():
    src = open(os.path.join(ROOT, "include", "mpcr_mjcf.h")).read()
    names = re.findall(r"^(?:int|void)\s+(mpcr_[a-z_]+)\s*\(", src, flags=re.M)
    so = ctypes.CDLL(os.path.join(ROOT, "manipulator_mujoco_amd", "libmpcr_mjcf.so"))
    assert names == ["mpcr_mjcf_compile", "mpcr_mjcf_free"]
    for n in names:
        assert hasattr(so, n), n


def test_comm_entry_points_fail_cleanly():
    """mpcr_comm_*: argument errors are EINVAL with a message; creating an id
    either works (GPU host) or reports RCCL's error (no GPU) -- no crash."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(128)
    assert lib.mpcr_comm_init(2, 2, uid, 0, ctypes.byref(h)) == -1
    assert b"bad comm arguments" in lib.mpcr_last_error()
    assert lib.mpcr_comm_unique_id(None) == -1
    rc = lib.mpcr_comm_unique_id(uid)
    assert rc == 0 or (rc == -3 and lib.mpcr_last_error())
    lib.mpcr_comm_free(None)
