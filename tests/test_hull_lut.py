"""The hull support start table the engine builds (model format v9 dropped it
from the blob; engine.hip hull_start_table, read back through
mpcr_model_hull_starts) and the cube-map cell mapping the oracle and the
kernel share (oracle lut_cell / rollout.hip lut_cell): every cell names a
vertex of its own hull that is extreme along the cell centre.  Host only --
the table is built on the CPU at engine creation (tests/test_oracle.py
covers the rollouts, tests/test_hull_ties.py the start independence)."""
import numpy as np
import pytest

from manipulator_mujoco_amd import cmodel, models
from manipulator_mujoco_amd.engine import Model

R = 32  # any resolution builds the same way; the library's own (MPCR_LUT_R) is checked for shape


def cell_dirs(R):
    """Cell-centre directions, cell order (2 axis + negative) R^2 + iu R + iv
    with u, v the components (axis + 1) % 3, (axis + 2) % 3."""
    c = -1.0 + (2.0 * np.arange(R) + 1.0) / R
    out = np.zeros((6, R, R, 3))
    for f in range(6):
        ax, neg = f // 2, f % 2
        out[f, :, :, ax] = -1.0 if neg else 1.0
        out[f, :, :, (ax + 1) % 3] = c[:, None]
        out[f, :, :, (ax + 2) % 3] = c[None, :]
    return out.reshape(-1, 3)


def lut_cell(l, R):
    """numpy restatement of the oracle's lut_cell (major axis lowest on ties)."""
    a = np.abs(l)
    ax = 0 if (a[0] >= a[1] and a[0] >= a[2]) else (1 if a[1] >= a[2] else 2)
    la = a[ax]
    if not la > 0:
        return 0
    iu = int(np.floor((l[(ax + 1) % 3] / la + 1.0) * 0.5 * R))
    iv = int(np.floor((l[(ax + 2) % 3] / la + 1.0) * 0.5 * R))
    iu, iv = min(max(iu, 0), R - 1), min(max(iv, 0), R - 1)
    return (2 * ax + (1 if l[ax] < 0 else 0)) * R * R + iu * R + iv


@pytest.fixture(scope="module")
def dual_arm():
    return models.load("dual_arm", 0.05)


def test_cell_dirs_map_to_their_own_cells():
    for r in (R, 256):
        dirs = cell_dirs(r)
        for c in range(0, len(dirs), 7):
            assert lut_cell(dirs[c], r) == c


def test_table_layout_and_extremes(dual_arm):
    m = dual_arm
    adr, lut = Model(m).hull_starts(R)
    hulls = np.where((np.asarray(m.geom_hulladr) >= 0) & (np.asarray(m.geom_hullnum) > 0))[0]
    assert len(hulls) == 14
    ncell = 6 * R ** 2
    assert lut.size == ncell * len(hulls)
    verts = np.asarray(m.hull_vert).reshape(-1, 3)
    dirs = cell_dirs(R)
    for g in hulls:
        a, n = int(m.geom_hulladr[g]), int(m.geom_hullnum[g])
        cells = lut[adr[g]:adr[g] + ncell]
        assert ((cells >= a) & (cells < a + n)).all()  # the geom's own hull
        vals = dirs @ verts[a:a + n].T
        best = vals.max(axis=1)
        got = np.einsum("ij,ij->i", dirs, verts[cells])
        assert np.allclose(got, best, rtol=0, atol=1e-12)  # extreme along the cell centre
        # a clear maximum is the table's vertex (ties: any of them, the kernel's walk is start-independent)
        clear = (vals >= best[:, None] - 1e-12).sum(axis=1) == 1
        assert (cells[clear] == np.argmax(vals, axis=1)[clear] + a).all()
    for g in range(int(m.ngeom)):
        if g not in hulls:
            assert adr[g] == -1


def test_library_resolution(dual_arm):
    adr, lut = Model(dual_arm).hull_starts()
    r = int(round(np.sqrt(lut.size / 14 / 6)))
    assert lut.size == 14 * 6 * r * r and r >= 128  # MPCR_LUT_R


def test_blob_carries_no_table(dual_arm):
    s = dual_arm.to_struct()
    assert s.version == cmodel.VERSION == 9  # v9: the engine builds the table
    names = {n for n, _ in cmodel.mpcr_model_t._fields_}
    assert "hull_lut" not in names and "geom_lutadr" not in names


def test_models_without_hulls_have_no_table():
    m = models.load("scene_mjx", 0.05)
    adr, lut = Model(m).hull_starts()
    assert lut.size == 0 and (adr == -1).all()
