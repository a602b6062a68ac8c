"""GPU parity gates: the HIP path through the C ABI vs the fp64 CPU oracle on
identical inputs (cost within 1e-4 relative, the north-star tolerance), plus
size-independent properties at the full BASELINE sizes."""
import numpy as np
import pytest

import oracle
import parity_util as pu
from manipulator_mujoco_amd import basis, models
from manipulator_mujoco_amd.engine import MPCR_LAYOUT_THETADOT, MPCR_LAYOUT_XI, Engine

pytestmark = pytest.mark.gpu

Q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
W = np.array([20.0, 3.0, 80.0])
PT = np.array([-0.3, -0.3, 0.5])
QT = np.array([0.0, 1.0, 0.0, 0.0])
TOL = pu.TOL  # north star: costs within 1e-4 relative fp32


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


def assert_no_sync_loss(st):
    """No candidate lost a two-wave handshake (status bit 10,
    MPCR_STATUS_SYNC in include/mpcr.h: its outputs would be void)."""
    s = st.cpu().numpy() if hasattr(st, "cpu") else np.asarray(st)
    assert int(((s >> 10) & 1).sum()) == 0, "two-wave handshake lost"


def projected_xi(n, H, seed, device):
    """BASELINE.md synthetic inputs: xi ~ N(0, 10.003 I) projected with 10 ADMM iterations."""
    import torch

    from manipulator_mujoco_amd.projection import ProjectionFilter
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    f = ProjectionFilter(P, Pd, Pdd, 6, device)
    rng = np.random.default_rng(seed)
    xi = torch.tensor(rng.normal(0, np.sqrt(10.003), (n, 66)).astype(np.float32), device=device)
    return f(xi, f.boundary(Q0, np.zeros(6), np.zeros(6), n), 10)


def compare(m, g, o, H):
    gc, oc = g["cost4"].astype(np.float64), o["cost4"]
    rel = np.abs(gc[:, 0] - oc[:, 0]) / np.maximum(np.abs(oc[:, 0]), 1e-6)
    # candidates grazing a contact (|dist| < 1e-5 somewhere) can flip the
    # integer #{c < 0} term between fp32 and fp64: reported separately
    if m.nslot:
        graze = (np.abs(o["slots"]) < 1e-5).any(axis=(1, 2))
    else:
        graze = np.zeros(len(rel), bool)
    return rel, graze


@pytest.mark.parametrize("name", models.PLANNER_SCENES)
@pytest.mark.parametrize("layout", [MPCR_LAYOUT_XI, MPCR_LAYOUT_THETADOT])
def test_parity_small(torch_cuda, name, layout):
    n, H = 64, 20
    m = models.load(name, 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    rng = np.random.default_rng(11)
    if layout == MPCR_LAYOUT_XI:
        inp = rng.normal(0, 0.05, (n, 66)).astype(np.float32)
        td = np.einsum("tk,njk->njt", Pd, inp.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
    else:
        t = np.arange(H) * 0.05
        inp = (rng.uniform(-0.7, 0.7, (n, 6, 1)) * np.sin(rng.uniform(0.2, 2, (n, 6, 1)) * t)).reshape(n, 6 * H)
        inp = inp.astype(np.float32)
        td = inp.astype(np.float64)
    e = Engine(m, H, n, Pd)
    g = e.trace(inp, layout, Q0, W, PT, QT)
    o = oracle.rollout(m, td, Q0, W, PT, QT, want_slots=True, want_eef=True)
    rel, graze = compare(m, g, o, H)
    assert rel[~graze].max() < TOL, rel.max()
    assert graze.mean() < 0.1
    # trajectories agree to fp32 rounding (sub-millimetre / sub-milliradian)
    assert np.abs(g["theta"] - o["theta"]).max() < 1e-3
    assert np.abs(g["eef"][..., :3] - o["eef"][..., :3]).max() < 1e-3
    if m.nslot:
        assert np.abs(g["slots"] - o["slots"]).max() < 1e-3


def _td(Pd, xi_h, H):
    n = xi_h.shape[0]
    return np.einsum("tk,njk->njt", Pd, xi_h.reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)


@pytest.mark.parametrize("name", ["planner_scene", "scene_mjx", "ur5e_hande_mjx"])
def test_parity_projected_h50(torch_cuda, name):
    """Realistic samples (projected to |thetadot| <= 0.8): arm/table/box
    contacts occur.  Bar: tests/parity_util.py (per-candidate conditioning,
    no allowance on well-conditioned candidates, the selection)."""
    torch = torch_cuda
    n, H = 256, 50
    m = models.load(name, 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 3, torch.device("cuda:0"))
    xi_h = xi.cpu().numpy()
    e = Engine(m, H, n, Pd)
    g = e.trace(xi_h, MPCR_LAYOUT_XI, Q0, W, PT, QT)
    o, sens = pu.conditioning(m, _td(Pd, xi_h, H))
    st = pu.check(m, g["cost4"][:, 0], o, sens, name)
    assert st["median_rel"] < 1e-5 and st["well"] >= 0.5 * n, st
    pu.check_components(m, g["cost4"], o, name, g_slots=g["slots"])


def test_parity_c2_full(torch_cuda):
    """C2 at its BASELINE size (ur5e_1_robotiq_hande_mjx.xml, 1024 x 50): every
    candidate against the oracle, the selection.  SURVEY §8d asks whether any
    contact activates on C2 ("no contacts"): it does -- the model has no
    gravcomp, the arm sags and the hand / wrist capsules (robot_5..9) reach
    the table (table_geom_1) after ~1.2 s in almost every candidate; the
    count is printed and the masked-slot distances must agree with the
    oracle's sign where they are not grazing."""
    torch = torch_cuda
    n, H = 1024, 50
    m = models.load("ur5e_hande_mjx", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 2, torch.device("cuda:0"))
    xi_h = xi.cpu().numpy()
    e = Engine(m, H, n, Pd)
    g = e.trace(xi_h, MPCR_LAYOUT_XI, Q0, W, PT, QT)
    o, sens = pu.conditioning(m, _td(Pd, xi_h, H))
    st = pu.check(m, g["cost4"][:, 0], o, sens, "C2")
    comp = pu.check_components(m, g["cost4"], o, "C2", g_slots=g["slots"])
    print(f"C2 components: {comp}")
    act_g = (g["slots"] < 0).any(axis=(1, 2))
    act_o = (o["slots"] < 0).any(axis=(1, 2))
    print(f"C2 contacts: {int(act_g.sum())}/{n} candidates with an active robot contact (oracle {int(act_o.sum())}); {st}")
    keep = ~pu.grazing(m, o) & (sens < pu.TOL / 10)
    assert (act_g[keep] == act_o[keep]).all()


def test_parity_c3_full(torch_cuda):
    """C3 at the BASELINE size (scene_mjx, 4096 x 50), the bench workload:
    all 4096 candidates against the oracle, the selection.  Includes the
    candidates whose busiest step needs more constraint rows than the LDS
    keeps (J rows >= 36 live in the per-candidate HBM slab): they are held
    to the same bar and counted."""
    torch = torch_cuda
    n, H = 4096, 50
    m = models.load("scene_mjx", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 3, torch.device("cuda:0"))
    xi_h = xi.cpu().numpy()
    e = Engine(m, H, n, Pd)
    st_ = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    key = torch.empty(1, dtype=torch.int64, device="cuda:0")
    a = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, best_key=key, status=st_).cpu().numpy()
    o, sens = pu.conditioning(m, _td(Pd, xi_h, H))
    stats = pu.check(m, a[:, 0], o, sens, "C3")
    # components and the integer count, from the traced slots (the trace is the
    # same kernel: its costs are the launch's bit for bit)
    tr = e.trace(xi_h, MPCR_LAYOUT_XI, Q0, W, PT, QT)
    assert np.array_equal(tr["cost4"], a)
    comp = pu.check_components(m, a, o, "C3", g_slots=tr["slots"])
    print(f"C3 components: {comp}")
    from manipulator_mujoco_amd import _lib
    idx, _ = _lib.decode_key(int(key.item()) & 0xFFFFFFFFFFFFFFFF)
    assert idx == stats["sel_gpu"]
    rows = (st_.cpu().numpy() >> 2) & 255
    slab = rows > 36
    rel = np.abs(a[:, 0] - o["cost4"][:, 0]) / np.abs(o["cost4"][:, 0])
    well = (sens < pu.TOL / 10) & ~pu.grazing(m, o)
    print(f"C3: {stats}; slab-path candidates {int(slab.sum())}, well-conditioned {int((slab & well).sum())}, "
          f"their max rel {rel[slab & well].max() if (slab & well).any() else 0:.2e}")
    assert (slab & well).sum() >= 100


def test_thetadot_and_theta_outputs(torch_cuda):
    torch = torch_cuda
    n, H = 128, 50
    m = models.load("scene_mjx", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 5, torch.device("cuda:0"))
    e = Engine(m, H, n, Pd)
    td = torch.empty((n, 6 * H), device="cuda:0")
    th = torch.empty((n, 6 * H), device="cuda:0")
    key = torch.empty(1, dtype=torch.int64, device="cuda:0")
    c4 = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, theta=th, thetadot=td, best_key=key)
    torch.cuda.synchronize()
    ref = np.einsum("tk,njk->njt", Pd, xi.cpu().numpy().reshape(n, 6, 11).astype(np.float64)).reshape(n, 6 * H)
    np.testing.assert_allclose(td.cpu().numpy(), ref, atol=2e-5)
    # first post-step theta = q0 + dt*thetadot_0 + dt^2*qacc_0; C3 has no
    # gravcomp, so gravity sags the arm by up to dt^2 * ~25 rad/s^2
    th0 = th.cpu().numpy()[:, ::H]
    assert np.abs(th0 - (Q0 + 0.05 * ref[:, ::H])).max() < 0.1
    from manipulator_mujoco_amd import _lib
    idx, val = _lib.decode_key(int(key.item()) & 0xFFFFFFFFFFFFFFFF)
    c = c4.cpu().numpy()
    assert idx == int(np.argmin(c[:, 0])) and val == c[idx, 0]


def test_argmin_nan_first_and_ties(torch_cuda):
    import ctypes
    torch = torch_cuda
    from manipulator_mujoco_amd import _lib
    _, P, Pd, _ = basis.planner_basis(20, 0.05)
    e = Engine(models.load("planner_scene", 0.05), 20, 4096, Pd)
    lib = _lib.load()
    c = np.random.default_rng(2).uniform(1, 9, (3000, 4)).astype(np.float32)
    c[1234, 0] = c[2345, 0] = -5.0
    idx, val = ctypes.c_int(), ctypes.c_float()
    assert lib.mpcr_argmin(e.handle, c.ctypes.data, 4, 3000, 0, None, ctypes.byref(idx), ctypes.byref(val), 0,
                           None) == 0
    assert idx.value == 1234 and val.value == -5.0
    c[2999, 0] = np.nan
    c[2000, 0] = np.nan
    assert lib.mpcr_argmin(e.handle, c.ctypes.data, 4, 3000, 100, None, ctypes.byref(idx), ctypes.byref(val), 0,
                           None) == 0
    assert idx.value == 2100 and np.isnan(val.value)


def test_full_size_properties(torch_cuda):
    """C3 at the BASELINE size (4096 x 50): finite, deterministic, sharding-invariant."""
    torch = torch_cuda
    n, H = 4096, 50
    m = models.load("scene_mjx", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 3, torch.device("cuda:0"))
    e = Engine(m, H, n, Pd)
    st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    key = torch.empty(1, dtype=torch.int64, device="cuda:0")
    a = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, best_key=key, status=st).clone()
    b = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b)  # bitwise deterministic
    assert torch.isfinite(a).all()
    assert int((st & 1).sum()) == 0  # no constraint-row truncation
    half = n // 2
    k2 = torch.empty(1, dtype=torch.int64, device="cuda:0")
    c1 = e.rollout_cost(xi[:half].contiguous(), MPCR_LAYOUT_XI, Q0, W, PT, QT).clone()
    c2 = e.rollout_cost(xi[half:].contiguous(), MPCR_LAYOUT_XI, Q0, W, PT, QT, best_key=k2, index_base=half).clone()
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([c1, c2]), a)
    from manipulator_mujoco_amd import _lib
    i_full, _ = _lib.decode_key(int(key.item()) & 0xFFFFFFFFFFFFFFFF)
    i_hi, _ = _lib.decode_key(int(k2.item()) & 0xFFFFFFFFFFFFFFFF)
    assert i_full == int(torch.argmin(a[:, 0]))
    assert i_hi == half + int(torch.argmin(a[half:, 0]))


@pytest.mark.parametrize("name,H,n", [("scene_mjx", 20, 4099), ("dual_arm", 10, 515)])
def test_ragged_batches_are_batch_independent(torch_cuda, name, H, n):
    """Ragged batch sizes (1, an odd handful, one past a wave of 64, a partial
    last launch round; small ones take the two-wave variant) give each
    candidate exactly the outputs it has inside the full batch, the best key
    names the prefix's own argmin, and an empty batch is a no-op."""
    torch = torch_cuda
    from manipulator_mujoco_amd import _lib
    m = models.load(name, 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 7, torch.device("cuda:0"))
    e = Engine(m, H, n, Pd)

    def run(k):
        c4 = torch.full((k, 4), float("nan"), device="cuda:0")
        th = torch.empty((k, 6 * H), device="cuda:0")
        st = torch.zeros(k, dtype=torch.int32, device="cuda:0")
        key = torch.empty(1, dtype=torch.int64, device="cuda:0")
        e.rollout_cost(xi[:k].contiguous(), MPCR_LAYOUT_XI, Q0, W, PT, QT, cost4=c4, theta=th, best_key=key,
                       status=st)
        torch.cuda.synchronize()
        return c4, th, st, key

    full = run(n)
    assert torch.isfinite(full[0]).all()
    for k in (1, 3, 65, n - 2):
        c4, th, st, key = run(k)
        assert torch.equal(c4, full[0][:k]), k
        assert torch.equal(th, full[1][:k]), k
        assert torch.equal(st, full[2][:k]), k
        idx, val = _lib.decode_key(int(key.item()) & 0xFFFFFFFFFFFFFFFF)
        assert idx == int(torch.argmin(c4[:, 0])) and val == float(c4[idx, 0]), k
    empty = torch.empty((0, 66), device="cuda:0")
    c0 = e.rollout_cost(empty, MPCR_LAYOUT_XI, Q0, W, PT, QT)
    torch.cuda.synchronize()
    assert c0.shape == (0, 4)


@pytest.mark.parametrize("name,H", [("scene_mjx", 50), ("dual_arm", 20)])
def test_c4_global_batch_on_one_gpu(torch_cuda, name, H):
    """The largest batch of BASELINE (C4's global 32768 candidates) on one
    GPU: eight launch rounds, the per-candidate HBM slabs at their largest.
    Each 4096-candidate shard equals its own launch bitwise (the shards the
    8-GPU run hands to its ranks) and the best key names the global argmin."""
    torch = torch_cuda
    from manipulator_mujoco_amd import _lib
    n, shard = 32768, 4096
    m = models.load(name, 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 8, torch.device("cuda:0"))
    e = Engine(m, H, n, Pd)
    st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    key = torch.empty(1, dtype=torch.int64, device="cuda:0")
    a = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, best_key=key, status=st).clone()
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    assert int((st & 1).sum()) == 0  # no constraint-row truncation
    for r in (0, 3, 7):
        lo = r * shard
        c = e.rollout_cost(xi[lo:lo + shard].contiguous(), MPCR_LAYOUT_XI, Q0, W, PT, QT, index_base=lo).clone()
        torch.cuda.synchronize()
        assert torch.equal(c, a[lo:lo + shard]), r
    idx, val = _lib.decode_key(int(key.item()) & 0xFFFFFFFFFFFFFFFF)
    assert idx == int(torch.argmin(a[:, 0])) and val == float(a[idx, 0])


def test_compute_cem_dropin(torch_cuda):
    from manipulator_mujoco_amd.planner import cem_planner
    p = cem_planner(num_dof=6, num_batch=256, num_steps=16, timestep=0.05, maxiter_cem=3, num_elite=0.05,
                    w_pos=20.0, w_rot=3.0, w_col=80.0, maxiter_projection=10, verbose=False)
    out = p.compute_cem(np.zeros(p.nvar), Q0, np.zeros(6), np.zeros(6), PT, QT)
    cost, cg, cr, cc, best_vels, best_traj, xi_mean, thetadot, theta = out
    assert cost.shape == (3,) and best_vels.shape == (16, 6) and best_traj.shape == (16, 6)
    assert xi_mean.shape == (66,) and thetadot.shape == (3, 256, 96) and theta.shape == (3, 256, 96)
    assert np.isfinite(cost).all() and cost[-1] <= cost[0] * 1.5
    # best_vels is the argmin row of the last iteration's thetadot
    k = np.where((thetadot[-1] == best_vels.T.reshape(-1)).all(axis=1))[0]
    assert k.size >= 1
    # the same call is deterministic (fixed key, SBP/mjx_planner.py:388)
    out2 = p.compute_cem(np.zeros(p.nvar), Q0, np.zeros(6), np.zeros(6), PT, QT)
    np.testing.assert_array_equal(out2[0], cost)


@pytest.mark.parametrize("H", [50, 100])
def test_dual_arm_parity_to_conditioning(torch_cuda, H):
    """Dual arm (C4/C5 scene) on realistic projected samples.  Its costs are
    chaotic even in fp64 (the 2F-85 linkage sits in permanent mesh contact and
    the Newton line search couples it to arm 1): 1e-7 input noise moves a
    share of the candidates by more than 1e-4.  The per-candidate bar of
    tests/parity_util.py takes that into account."""
    torch = torch_cuda
    n = 256
    m = models.load("dual_arm", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 4, torch.device("cuda:0"))
    xi_h = xi.cpu().numpy()
    e = Engine(m, H, n, Pd)
    st = np.zeros(n, dtype=np.int32)
    g = e.rollout_cost(xi_h, MPCR_LAYOUT_XI, Q0, W, PT, QT, status=st).astype(np.float64)
    assert_no_sync_loss(st)
    o, sens = pu.conditioning(m, _td(Pd, xi_h, H), seed=H)
    st = pu.check(m, g[:, 0], o, sens, f"dual arm H={H}")
    comp = pu.check_components(m, g, o, f"dual arm H={H}")
    print(f"dual arm H={H}: {st}; components {comp}")
    assert st["median_rel"] < 1e-5


def test_dual_arm_c4_properties(torch_cuda):
    """C4's per-GPU shard (4096 x 100, dual arm: implicitfast, actuators,
    connect equalities, convex-hull contacts): finite, deterministic,
    shard-invariant, the gripper's permanently touching linkage contacts are
    found (constraint rows every step), no row truncation."""
    torch = torch_cuda
    n, H = 4096, 100
    m = models.load("dual_arm", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 4, torch.device("cuda:0"))
    e = Engine(m, H, n, Pd)
    st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    a = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, status=st).clone()
    b = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT).clone()
    half = n // 2
    c2 = e.rollout_cost(xi[half:].contiguous(), MPCR_LAYOUT_XI, Q0, W, PT, QT, index_base=half).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.isfinite(a).all() and torch.equal(c2, a[half:])
    s_ = st.cpu().numpy()
    assert int((s_ & 1).sum()) == 0
    assert_no_sync_loss(s_)
    rows_per_step = (s_ >> 11) / H
    assert rows_per_step.min() >= 8  # 8 equality rows + the linkage contacts
    # the busiest step's rows (status bits 2-9, no longer saturating at 63):
    # below the wide image's 8 + 4 x 48 = 200-row cap (measured p50 / p99 /
    # max 76 / 160 / 184 on this shard, round 4)
    max_rows = (s_ >> 2) & 255
    print(f"C4 max rows per step p50/p99/max {np.percentile(max_rows, 50):.0f}/{np.percentile(max_rows, 99):.0f}/"
          f"{max_rows.max()}")
    assert max_rows.max() < 8 + 4 * 48  # no step reached the cap (status bit 0 is the truncation flag)
    # the whole shard against the oracle: conditioning bar and the selection
    o, sens = pu.conditioning(m, _td(Pd, xi.cpu().numpy(), H), seed=7)
    assert int(o["maxcon"].max()) <= 48 and int(o["maxrows"].max()) <= 8 + 4 * 48  # the wide image's caps
    # the whole bar, well-conditioned candidates included
    a4 = a.cpu().numpy()
    st_ = pu.check(m, a4[:, 0], o, sens, "C4 shard")
    comp = pu.check_components(m, a4, o, "C4 shard")
    print(f"C4 shard: {st_}; components {comp}")


def test_kernel_occupancy_budget(torch_cuda):
    """The LDS images and register budgets the performance rests on (DESIGN.md
    §LDS capacity): 16 narrow blocks per CU (<= 9520 B each, 4 waves/SIMD),
    the dual-arm image at <= 20448 B (the compact mass matrix in LDS; 8 blocks
    per CU measured up to that size, 7 at 20960 B) with a 2-waves/SIMD register
    budget: 8 blocks per CU."""
    import ctypes

    from manipulator_mujoco_amd import _lib
    info = (ctypes.c_int * 6)()
    _lib.check(_lib.load().mpcr_rollout_occupancy(0, info))
    nb, nlds, nreg, wb, wlds, wreg = list(info)
    assert nlds <= 9520 and nreg <= 128 and nb >= 16, list(info)
    assert wlds <= 20448 and wreg <= 256 and wb >= 8, list(info)


@pytest.mark.parametrize("name,n", [("ur5e_hande_mjx", 1024), ("scene_mjx", 512), ("dual_arm", 1024)])
def test_two_wave_variant_is_bitwise_one_wave(torch_cuda, name, n):
    """Small batches may run two waves per candidate (collision beside the
    dynamics, mpcr_set_two_wave_max_n): the same instructions on the same data,
    so cost4, theta, thetadot and status equal the one-wave kernel's bit for
    bit."""
    torch = torch_cuda
    from manipulator_mujoco_amd import _lib
    lib = _lib.load()
    H = 50
    m = models.load(name, 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 2, torch.device("cuda:0"))
    e = Engine(m, H, n, Pd)
    outs = []
    prev = lib.mpcr_set_two_wave_max_n(-1)
    try:
        for thr in (0, n):
            lib.mpcr_set_two_wave_max_n(thr)
            c4 = torch.empty((n, 4), device="cuda:0")
            th = torch.empty((n, 6 * H), device="cuda:0")
            td = torch.empty((n, 6 * H), device="cuda:0")
            st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
            e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, cost4=c4, theta=th, thetadot=td, status=st)
            torch.cuda.synchronize()
            outs.append((c4, th, td, st))
    finally:
        lib.mpcr_set_two_wave_max_n(prev)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert_no_sync_loss(outs[1][3])


@pytest.mark.parametrize("lead_max", [-1, 0, 6])
def test_two_wave_dual_arm_flush_paths_bitwise(torch_cuda, monkeypatch, lead_max):
    """The two-wave dual-arm kernel's convex flush has two paths: the lead
    flush (swap mode: the collision wave runs every pair's MPR beside wave 0's
    dynamics, a manifold queue over both waves) for steps with at most
    DevModel::w2_lead_max listed pairs, else the dealt flush (item i on wave
    i & 1).  MPCR_W2_LEAD_MAX lowers the limit: -1 sends every step to the
    dealt flush (no pair list is ever that short), 0 only the pair-free steps
    to the lead path, 6 mixes them within each rollout.  Every mix is bitwise
    the one-wave kernel."""
    torch = torch_cuda
    from manipulator_mujoco_amd import _lib
    lib = _lib.load()
    n, H = 512, 50
    m = models.load("dual_arm", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 6, torch.device("cuda:0"))
    monkeypatch.setenv("MPCR_W2_LEAD_MAX", str(lead_max))
    e = Engine(m, H, n, Pd)
    outs = []
    prev = lib.mpcr_set_two_wave_max_n(-1)
    try:
        for thr in (0, n):
            lib.mpcr_set_two_wave_max_n(thr)
            c4 = torch.empty((n, 4), device="cuda:0")
            th = torch.empty((n, 6 * H), device="cuda:0")
            td = torch.empty((n, 6 * H), device="cuda:0")
            st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
            e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, cost4=c4, theta=th, thetadot=td, status=st)
            torch.cuda.synchronize()
            outs.append((c4, th, td, st))
    finally:
        lib.mpcr_set_two_wave_max_n(prev)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert_no_sync_loss(outs[1][3])


@pytest.mark.parametrize("seg,groups", [(25, 1), (50, 2), (20, 4)])
def test_dual_arm_horizon_segments_bitwise(torch_cuda, monkeypatch, seg, groups):
    """Dual-arm rollouts as horizon segments (rollout_launch: each segment
    resumes from the state the previous one saved, candidate groups on their
    own streams) are bitwise the one-launch rollouts: costs, theta, thetadot,
    status and the fused best key."""
    torch = torch_cuda
    n, H = 2048 + 37, 100  # ragged: groups of unequal size
    m = models.load("dual_arm", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 4, torch.device("cuda:0"))
    out = []
    for steps, g in ((0, 1), (seg, groups)):
        monkeypatch.setenv("MPCR_SEG_STEPS", str(steps))
        monkeypatch.setenv("MPCR_SEG_GROUPS", str(g))
        e = Engine(m, H, n, Pd)
        # one dispatch, or one per segment and group (mpcr_engine_dispatches;
        # the batch is above the 2048 resident blocks, so it is segmented)
        assert e.dispatches(n) == (1 if steps == 0 else g * -(-H // steps)), (steps, g)
        assert e.dispatches(1024) == 1  # the two-wave variant: one round
        st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
        th = torch.empty((n, 6 * H), device="cuda:0")
        td = torch.empty((n, 6 * H), device="cuda:0")
        key = torch.empty(1, dtype=torch.int64, device="cuda:0")
        c = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, theta=th, thetadot=td, best_key=key, status=st,
                           index_base=5).clone()
        torch.cuda.synchronize()
        out.append((c, th, td, st, key))
        del e
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
    assert_no_sync_loss(out[1][3])


def test_dual_arm_compact_mass_matrix_bitwise_slab(torch_cuda, monkeypatch):
    """The dual-arm mass matrix kept compact in LDS (16-column tree windows,
    DevModel::mc_c0) gives bitwise the costs, theta, thetadot and status of
    the dense per-candidate HBM slab (MPCR_M_SLAB=1, the path for models whose
    trees do not fit the window): the window leaves out exact zeros only."""
    torch = torch_cuda
    n, H = 1536, 40
    m = models.load("dual_arm", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 9, torch.device("cuda:0"))
    out = []
    for slab in ("0", "1"):
        monkeypatch.setenv("MPCR_M_SLAB", slab)
        e = Engine(m, H, n, Pd)
        st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
        th = torch.empty((n, 6 * H), device="cuda:0")
        td = torch.empty((n, 6 * H), device="cuda:0")
        c = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, theta=th, thetadot=td, status=st).clone()
        torch.cuda.synchronize()
        out.append((c, th, td, st))
        del e
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
    assert_no_sync_loss(out[1][3])


def test_kernel_support_is_start_independent(torch_cuda):
    """The kernel's hull supports do not depend on where a climb starts
    (the tie walk of sup_finish / tie_round): the dual arm
    rolled out with a support start table whose every cell points at a hashed
    vertex of its hull (mpcr_set_hull_start_scramble; the engine marks such a
    cell exact only when that vertex is its support) gives the same status
    words and, but for the SAT's value-only queries, bitwise the same costs
    and theta as with the extreme-vertex table -- a table resolution is a
    performance choice, not a parity change.  The SAT's separations skip the
    tie walk (any tied vertex gives the value to within kHullTie, 1e-7 m), so
    a start can move a separation in its last bits: over seeds 1..3 at
    1024 x 50 and 4096 x 100 that left 0-2 and 9 candidates a cost ulp apart
    (tools/scramble_check.py, profiles/r06_scramble_check.txt); the
    -DMPCR_SAT_TIES=1 build walks those too and is bitwise for all of them,
    at +5 % kernel time.  The bar: statuses equal, at most 1 % of the
    candidates not bitwise, none off by more than 1e-6 relative cost."""
    torch = torch_cuda
    from manipulator_mujoco_amd import _lib
    lib = _lib.load()
    n, H = 1024, 50
    m = models.load("dual_arm", 0.05)
    _, P, Pd, _ = basis.planner_basis(H, 0.05)
    xi = projected_xi(n, H, 20250629 + 4, torch.device("cuda:0"))
    out = []
    for scr in (0, 1):
        prev = lib.mpcr_set_hull_start_scramble(scr)  # engines created now start at hashed vertices
        try:
            e = Engine(m, H, n, Pd)
        finally:
            lib.mpcr_set_hull_start_scramble(prev)
        st = torch.zeros(n, dtype=torch.int32, device="cuda:0")
        th = torch.empty((n, 6 * H), device="cuda:0")
        c = e.rollout_cost(xi, MPCR_LAYOUT_XI, Q0, W, PT, QT, theta=th, status=st).clone()
        torch.cuda.synchronize()
        out.append((c.cpu().numpy(), th.cpu().numpy(), st.cpu().numpy()))
        del e
    (ca, ta, sa), (cb, tb, sb) = out
    diff = (ca != cb).any(axis=1) | (ta != tb).any(axis=1)
    rel = np.abs(ca[:, 0].astype(np.float64) - cb[:, 0]) / np.abs(ca[:, 0])
    print(f"start table scrambled: {int(diff.sum())}/{n} candidates differ, worst cost rel {rel.max():.1e}")
    assert np.array_equal(sa, sb)
    assert diff.sum() <= n // 100 and rel.max() <= 1e-6
