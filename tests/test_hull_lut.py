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


def _kernel_dot(x, d):
    """x . d in fp32 as the kernel forms it (products and sums in float)."""
    x, d = x.astype(np.float32), d.astype(np.float32)
    return (x[..., 0] * d[..., 0] + x[..., 1] * d[..., 1]) + x[..., 2] * d[..., 2]


@pytest.mark.parametrize("scale", [1.0, 40.0])
def test_exact_cells_hold_along_sampled_directions(dual_arm, scale):
    """a cell the engine marks exact skips the climb, so its start
    vertex must beat every neighbour along every direction in the cell as the
    kernel computes the projections (fp32).  Checked on the dual arm's hulls
    and on the same hulls scaled to metres (scale 40: the 2691-vertex hull
    spans ~4 m, where a fixed 1e-6 m margin would be below fp32 rounding):
    the cell corners and random interior directions of every 5th exact cell,
    normalised in fp32 as the kernel's local direction is."""
    import copy
    m = copy.copy(dual_arm)
    m.hull_vert = np.asarray(dual_arm.hull_vert, dtype=np.float64) * scale
    adr, lut, exact = Model(m).hull_starts(R, exact=True)
    assert exact.mean() > 0.3  # many cells skip the climb (more at the library's finer cells)
    verts = np.asarray(m.hull_vert).reshape(-1, 3)
    adjadr, adjnum, adj = (np.asarray(m.hull_adjadr), np.asarray(m.hull_adjnum), np.asarray(m.hull_adj))
    rng = np.random.default_rng(3)
    c = -1.0 + 2.0 * np.arange(R + 1) / R  # cell edges
    checked = 0
    for g in np.where(adr >= 0)[0]:
        cells = np.where(exact[adr[g]:adr[g] + 6 * R * R])[0][::5]
        for cc in cells:
            f, iu, iv = cc // (R * R), (cc // R) % R, cc % R
            ax = f // 2
            t = np.concatenate([np.array([[0, 0], [0, 1], [1, 0], [1, 1]], float), rng.random((4, 2))])
            d = np.zeros((len(t), 3))
            d[:, ax] = -1.0 if f % 2 else 1.0
            d[:, (ax + 1) % 3] = c[iu] + (c[iu + 1] - c[iu]) * t[:, 0]
            d[:, (ax + 2) % 3] = c[iv] + (c[iv + 1] - c[iv]) * t[:, 1]
            d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
            v = int(lut[adr[g] + cc])
            nb = adj[adjadr[v]:adjadr[v] + adjnum[v]]
            best = _kernel_dot(verts[v][None, :], d)  # (dirs,)
            other = _kernel_dot(verts[nb][None, :, :], d[:, None, :])  # (dirs, nb)
            assert (other <= best[:, None]).all(), (g, cc, v, float((other - best[:, None]).max()))
            checked += 1
    assert checked > 1000
