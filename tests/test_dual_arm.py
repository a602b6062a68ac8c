"""Dual-arm class on the CPU: the compiled
bundle's structure, and analytic pins of the oracle's new physics
(oracle/mpcr_oracle.c: MPR convex collision, plane-convex, actuators,
implicitfast) on small synthetic scenes whose answers are known in closed form.
The GPU kernel is checked against this oracle in tests/test_gpu_parity.py."""
import os
import struct

import numpy as np
import pytest

import oracle
from conftest import REFERENCE, has_reference
from manipulator_mujoco_amd import basis, cmodel, mjcf, models


@pytest.fixture(scope="module")
def dual():
    return models.load("dual_arm", 0.05)


def test_dual_arm_structure(dual):
    m = dual
    assert (m.nv, m.nq, m.nu, m.neq, m.npair, m.nslot) == (22, 22, 14, 4, 662, 0)
    assert m.integrator == cmodel.INT_IMPLICITFAST and m.iterations == 100 and m.ls_iterations == 50
    assert sorted(m.eq_type.tolist()) == [0, 0, 2, 2]  # 2 connect, 2 joint
    funcs = m.pair_func.tolist()
    assert funcs.count(cmodel.COL_CONVEX) == 424 and funcs.count(cmodel.COL_PLANE_CONVEX) == 16
    assert funcs == sorted(funcs)  # convex pairs last (the kernel compacts them in order)
    assert int((m.body_weldid != 0).sum()) == 29
    # arm 1 is the planner's: the first 6 dofs, hande + tcp present
    assert m.names["body"][m.hande_body] == "hande" and m.names["site"][m.tcp_site] == "tcp"
    # the two grippers' tendon actuators spread over their two finger / driver joints
    tendon = [a for a in range(m.nu) if m.act_ntrn[a] == 2]
    assert len(tendon) == 2
    for a in tendon:
        np.testing.assert_allclose(m.act_moment[a], [0.5, 0.5])


def test_hull_graphs(dual):
    """Every hull vertex graph is symmetric and hill climbing from the first
    vertex reaches the true support point (what the kernel and oracle rely on)."""
    m = dual
    rng = np.random.default_rng(0)
    adj = [set(m.hull_adj[m.hull_adjadr[v]:m.hull_adjadr[v] + m.hull_adjnum[v]].tolist()) for v in range(m.nhullv)]
    corners = {int(c) + k for c in m.geom_cornadr if c >= 0 for k in range(8)}  # box corners: faces only
    for v, nb in enumerate(adj):
        if v in corners:
            assert not nb
            continue
        assert len(nb) >= 3 and v not in nb
        for u in nb:
            assert v in adj[u]
    for g in np.where(m.geom_hulladr >= 0)[0]:
        a, n = m.geom_hulladr[g], m.geom_hullnum[g]
        V = m.hull_vert[a:a + n]
        assert np.linalg.norm(V.mean(axis=0)) < 1e-9  # recentred: the portal starts inside
        for d in rng.normal(size=(20, 3)):
            v = a
            while True:
                best = max(adj[v], key=lambda u: m.hull_vert[u] @ d)
                if m.hull_vert[best] @ d <= m.hull_vert[v] @ d:
                    break
                v = best
            assert abs(m.hull_vert[v] @ d - (V @ d).max()) < 1e-12


def test_connect_anchors_coincide_at_qpos0(dual):
    m = dual
    k = mjcf.kinematics0(m, m.qpos0)
    for e in np.where(m.eq_type == cmodel.EQ_CONNECT)[0]:
        b1, b2 = m.eq_obj1[e], m.eq_obj2[e]
        p1 = k["xpos"][b1] + k["xmat"][b1] @ m.eq_data[e, :3]
        p2 = k["xpos"][b2] + k["xmat"][b2] @ m.eq_data[e, 3:6]
        np.testing.assert_allclose(p1, p2, atol=1e-12)


@pytest.mark.skipif(not has_reference(), reason="needs /root/reference MJCF")
def test_dual_bundle_is_current():
    m = mjcf.compile_mjcf(os.path.join(REFERENCE, "universal_robots_ur5e/dual_arm_gripper_scene.xml"), 0.05)
    assert m.to_blob() == models.load("dual_arm", 0.05).to_blob()


def test_dual_arm_rollout_is_finite_and_holds_arm2(dual):
    """Planner semantics on the dual arm: finite costs; arm 2 (position servos
    at ctrl 0, its home pose) stays within a few centiradians of home."""
    H, n = 30, 4
    rng = np.random.default_rng(1)
    td = rng.uniform(-0.4, 0.4, (n, 6 * H))
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    o = oracle.rollout(dual, td, q0, np.array([20.0, 3.0, 80.0]), np.array([-0.3, -0.3, 0.5]),
                       np.array([0.0, 1.0, 0.0, 0.0]), want_theta=True)
    assert np.isfinite(o["cost4"]).all() and o["status"] == 0
    qpos = dual.qpos_init[:dual.nq].copy()
    qpos[:6] = q0
    qvel, qws = np.zeros(dual.nv), np.zeros(dual.nv)
    for _ in range(H):
        r = oracle.step(dual, qpos, qvel, qws)
        qpos, qvel, qws = r["qpos"], r["qvel"], r["qacc_warmstart"]
    assert np.abs(qpos[8:14]).max() < 0.05


# ---------------------------------------------------------------------------
# analytic pins on synthetic scenes


def _cube_stl(path, h):
    """Binary STL of an axis-aligned cube with half size h (12 triangles)."""
    c = np.array([[x, y, z] for x in (-h, h) for y in (-h, h) for z in (-h, h)])
    faces = [(0, 1, 3), (0, 3, 2), (4, 6, 7), (4, 7, 5), (0, 4, 5), (0, 5, 1),
             (2, 3, 7), (2, 7, 6), (0, 2, 6), (0, 6, 4), (1, 5, 7), (1, 7, 3)]
    with open(path, "wb") as f:
        f.write(b"\0" * 80 + struct.pack("<I", len(faces)))
        for t in faces:
            f.write(struct.pack("<3f", 0, 0, 0))
            for i in t:
                f.write(struct.pack("<3f", *c[i]))
            f.write(b"\0\0")


def _scene(tmp_path, body_xml, extra="", option='<option timestep="0.01" gravity="0 0 0"/>'):
    _cube_stl(tmp_path / "cube.stl", 0.05)
    xml = f"""<mujoco>
  <compiler angle="radian" autolimits="true"/>
  {option}
  <asset><mesh name="cube" file="cube.stl"/></asset>
  <worldbody>
    <geom name="floor" type="plane" size="0 0 0.05"/>
    {body_xml}
  </worldbody>
  {extra}
</mujoco>"""
    p = tmp_path / "s.xml"
    p.write_text(xml)
    return mjcf.compile_mjcf(str(p))


def _dists(m):
    """First contact slot of every pair, keyed by both geom-name orders."""
    r = oracle.step(m, m.qpos_init[:m.nq].copy(), np.zeros(m.nv), np.zeros(m.nv))
    d = {}
    for p in range(m.npair):
        a, b = m.names["geom"][m.pair_geom1[p]], m.names["geom"][m.pair_geom2[p]]
        d[(a, b)] = d[(b, a)] = r["dist"][m.pair_conadr[p]]
    return r, d


def test_mpr_sphere_sphere_depth(tmp_path):
    m = _scene(tmp_path, """
    <body name="a" pos="0 0 1"><freejoint/><geom name="a" type="sphere" size="0.1"/></body>
    <body name="b" pos="0.03 0.04 1.13"><freejoint/><geom name="b" type="sphere" size="0.1"/></body>""")
    # sphere-sphere has no primitive function here: the general convex (MPR) path
    assert cmodel.COL_CONVEX in m.pair_func.tolist()
    _, d = _dists(m)
    depth = 0.2 - np.sqrt(0.03 ** 2 + 0.04 ** 2 + 0.13 ** 2)
    assert abs(d[("a", "b")] + depth) < 1e-6


def test_mpr_mesh_cube_on_box_and_plane(tmp_path):
    m = _scene(tmp_path, """
    <body name="c" pos="0 0 0.04"><freejoint/><geom name="c" type="mesh" mesh="cube"/></body>
    <body name="k" pos="0.3 0 0.03"><freejoint/><geom name="k" type="mesh" mesh="cube"/></body>
    <body name="t" pos="0.3 0 -0.015"><geom name="t" type="box" size="0.2 0.2 0.01"/></body>""")
    _, d = _dists(m)
    assert abs(d[("floor", "c")] - (0.04 - 0.05)) < 1e-9    # plane-convex: deepest hull vertex
    assert abs(d[("t", "k")] - ((0.03 - 0.05) - (-0.005))) < 1e-6  # box top at -0.005, cube bottom at -0.02


def test_mpr_cylinder_and_capsule_on_box(tmp_path):
    m = _scene(tmp_path, """
    <body name="t" pos="0 0 -0.5"><geom name="t" type="box" size="1 1 0.5"/></body>
    <body name="y" pos="0 0 0.097"><freejoint/><geom name="y" type="cylinder" size="0.05 0.1"/></body>
    <body name="p" pos="0.5 0 0.015" euler="0 1.5707963267948966 0"><freejoint/>
      <geom name="p" type="capsule" size="0.02 0.1"/></body>""")
    _, d = _dists(m)
    assert abs(d[("t", "y")] + 0.003) < 1e-6   # cylinder end face 3 mm into the box top (MPR)
    assert abs(d[("t", "p")] + 0.005) < 1e-6   # capsule-box keeps its primitive function


def test_actuator_implicitfast_slide(tmp_path):
    """Position servo (kp, kv) on a slide joint of mass `mass`, no gravity: the
    actuator force is -kp q - kv v, and implicitfast advances the velocity with
    (mass + dt kv) a = -kp q - kv v."""
    kp, kv, mass, dt, q = 100.0, 10.0, 2.0, 0.01, 0.1
    m = _scene(tmp_path, f"""
    <body name="s" pos="0 0 1"><joint name="x" type="slide" axis="1 0 0"/>
      <geom name="s" type="sphere" size="0.01" mass="{mass}" contype="0" conaffinity="0"/></body>""",
               extra=f'<actuator><position joint="x" kp="{kp}" kv="{kv}"/></actuator>',
               option=f'<option timestep="{dt}" gravity="0 0 0" integrator="implicitfast"/>')
    assert m.nu == 1 and m.integrator == cmodel.INT_IMPLICITFAST
    r = oracle.step(m, np.array([q]), np.zeros(1), np.zeros(1))
    np.testing.assert_allclose(r["qacc"], [-kp * q / mass], rtol=1e-12)   # forward (explicit) acceleration
    a_impl = -kp * q / (mass + dt * kv)
    np.testing.assert_allclose(r["qvel"], [dt * a_impl], rtol=1e-12)
    np.testing.assert_allclose(r["qpos"], [q + dt * dt * a_impl], rtol=1e-12)


def test_actuator_force_and_joint_clamps(tmp_path):
    """General affine actuator with forcerange, on a joint with actuatorfrcrange."""
    m = _scene(tmp_path, """
    <body name="s" pos="0 0 1"><joint name="x" type="slide" axis="1 0 0" actuatorfrcrange="-3 3"/>
      <geom name="s" type="sphere" size="0.01" mass="1" contype="0" conaffinity="0"/></body>""",
               extra='<actuator><general joint="x" gaintype="fixed" biastype="affine" gainprm="2" '
                     'biasprm="1 -50 0" ctrlrange="-1 1" forcerange="-5 5"/></actuator>')
    for q, expect in ((0.0, 1.0), (0.05, -1.5), (0.2, -3.0), (-0.2, 3.0)):  # ctrl 0: f = 1 - 50 q
        r = oracle.step(m, np.array([q]), np.zeros(1), np.zeros(1))
        np.testing.assert_allclose(r["qacc"], [expect], rtol=1e-12, atol=1e-12)


def test_ctrl_zero_servos_pull_arm1_home(dual):
    """The C5 closed loop's drift (profiles/r01_c4_c5.json: eef_dist grows) is
    the reference's own semantics, not a plant error.  The dual-arm MJCF gives
    arm 1 position servos (URD/ur5e_1_robotiq_hande.xml:10,169-174: gain 2000,
    bias 0 -2000 -400) and the planner never writes ctrl, so MjData's default
    ctrl = 0 holds (SBP/mjx_planner.py:102-107; the keyframe at
    URD/dual_arm_gripper_scene.xml:30 is ctrl 0 too).  Each step the override
    qvel[:6] = thetadot (SBP/mjx_planner.py:254) meets the servo's implicit
    damping (implicitfast) and its position term: most of the commanded
    velocity is absorbed and the joints creep toward q = 0 whatever the plan.
    Without the actuators the commanded velocity passes through."""
    m = dual
    qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    cmd = np.array([0.5, 0, 0, 0, 0, 0])

    def run(model, steps=5):
        qpos = np.array(model.qpos_init[:model.nq])
        qpos[qa] = q0
        qvel, ws = np.zeros(model.nv), np.zeros(model.nv)
        for _ in range(steps):
            qv = qvel.copy()
            qv[da] = cmd
            o = oracle.step(model, qpos, qv, ws)
            qpos, qvel, ws = o["qpos"], o["qvel"], o["qacc_warmstart"]
        return qpos[qa], qvel[da]

    q, v = run(m)
    assert v[0] < 0.4 * cmd[0]  # the commanded joint keeps < 40 % of its velocity
    moved = q[1:5] - q0[1:5]
    assert (np.sign(moved) == -np.sign(q0[1:5])).all() and (np.abs(moved) > 0.05).all()  # toward 0
    free = models.load("dual_arm", 0.05)
    free.nu = 0
    q, v = run(free)
    assert v[0] > 0.8 * cmd[0]  # (the other joints then sag under gravity: no gravcomp here)


def test_polyhedron_faces(dual):
    """The faces of the polyhedron-pair hulls / boxes (model v7): unit outward
    normals, every kept vertex on its face plane, counter-clockwise about the
    normal, the hull inside every face plane, each vertex listed by its faces."""
    m = dual
    assert m.nface > 0
    for g in np.where(m.geom_faceadr >= 0)[0]:
        f0, nf = m.geom_faceadr[g], m.geom_facenum[g]
        if m.geom_type[g] == 7:
            V = m.hull_vert[m.geom_hulladr[g]:m.geom_hulladr[g] + m.geom_hullnum[g]]
        else:
            V = m.hull_vert[m.geom_cornadr[g]:m.geom_cornadr[g] + 8]
        for f in range(f0, f0 + nf):
            n, off = m.face_plane[f, :3], m.face_plane[f, 3]
            assert abs(np.linalg.norm(n) - 1) < 1e-9
            assert (V @ n).max() <= off + 1e-6 * max(1.0, abs(off))  # the hull lies inside
            P = m.hull_vert[m.face_vert[m.face_vadr[f]:m.face_vadr[f] + m.face_vnum[f]]]
            assert 3 <= len(P) <= 16
            assert np.abs(P @ n - off).max() < 1e-5
            c = P.mean(axis=0)
            area = sum(np.cross(P[k] - c, P[(k + 1) % len(P)] - c) @ n for k in range(len(P)))
            assert area > 0  # counter-clockwise
            for v in m.face_vert[m.face_vadr[f]:m.face_vadr[f] + m.face_vnum[f]]:
                assert f in m.vert_face[m.vert_faceadr[v]:m.vert_faceadr[v] + m.vert_facenum[v]]


def _active(m, qpos=None):
    r = oracle.step_debug(m, m.qpos_init[:m.nq].copy() if qpos is None else qpos, np.zeros(m.nv), np.zeros(m.nv))
    names = m.names["geom"]
    out = {}
    for k in range(r["ncon"]):
        p = r["con_pair"][k]
        key = (names[m.pair_geom1[p]], names[m.pair_geom2[p]])
        out.setdefault(key, []).append((r["con_dist"][k], r["con_pos"][k], r["con_normal"][k]))
    return out


def test_poly_manifold_cube_flat_on_box(tmp_path):
    """A mesh cube resting flat 15 mm deep in a box table: the polyhedron
    manifold (mjx convex_convex restated: reference face, clipped incident
    face, 4 picks) puts one contact under each bottom corner, all at the same
    depth, normal along z, half-way through the penetration."""
    m = _scene(tmp_path, """
    <body name="k" pos="0.3 0 0.03"><freejoint/><geom name="k" type="mesh" mesh="cube"/></body>
    <body name="t" pos="0.3 0 -0.015"><geom name="t" type="box" size="0.2 0.2 0.01"/></body>""")
    c = _active(m)
    key = ("t", "k") if ("t", "k") in c else ("k", "t")
    cs = c[key]
    assert len(cs) == 4
    for dist, pos, n in cs:
        assert abs(dist + 0.015) < 1e-9
        assert abs(abs(n[2]) - 1) < 1e-12
        assert abs(pos[2] - (-0.02 + 0.0075)) < 1e-9  # half-way between the cube bottom and the table top
    xy = sorted((round(p[0] - 0.3, 6), round(p[1], 6)) for _, p, _ in cs)
    assert xy == [(-0.05, -0.05), (-0.05, 0.05), (0.05, -0.05), (0.05, 0.05)]


def test_poly_manifold_clips_to_the_smaller_face(tmp_path):
    """Two mesh cubes, the upper one shifted by half a side: the contact
    polygon is the overlap of the faces (clipped), 4 corners of the 5 cm x
    10 cm overlap region; a cube tilted by 45 degrees onto its edge: the
    lower cube's top face is the reference, the edge's two ends the
    contacts."""
    m = _scene(tmp_path, """
    <body name="a" pos="0 0 0"><freejoint/><geom name="a" type="mesh" mesh="cube"/></body>
    <body name="b" pos="0.05 0 0.098"><freejoint/><geom name="b" type="mesh" mesh="cube"/></body>
    <body name="e" pos="1 0 0"><freejoint/><geom name="e" type="mesh" mesh="cube"/></body>
    <body name="f" pos="1 0 0.1157" euler="0.7853981633974483 0 0"><freejoint/><geom name="f" type="mesh" mesh="cube"/></body>""")
    c = _active(m)
    ab = c.get(("a", "b")) or c.get(("b", "a"))
    assert len(ab) == 4
    xs = sorted(round(p[0], 6) for _, p, _ in ab)
    ys = sorted(round(p[1], 6) for _, p, _ in ab)
    assert xs == [0.0, 0.0, 0.05, 0.05] and ys == [-0.05, -0.05, 0.05, 0.05]
    for dist, _, n in ab:
        assert abs(dist + 0.002) < 1e-8 and abs(abs(n[2]) - 1) < 1e-12  # (fp32 STL vertices)
    ef = c.get(("e", "f")) or c.get(("f", "e"))
    assert ef is not None and len(ef) == 2
    depth = 0.05 * np.sqrt(2) - (0.1157 - 0.05)
    assert sorted(round(p[0], 6) for _, p, _ in ef) == [0.95, 1.05]
    for dist, _, n in ef:
        assert abs(dist + depth) < 1e-8 and abs(abs(n[2]) - 1) < 1e-12


SHARED_MESH_DEEP = """
    <body name="a" pos="0 0 0.2" euler="0.3 0 0"><freejoint/><geom name="a" type="mesh" mesh="cube"/></body>
    <body name="b" pos="0.01 0 0.30454"><freejoint/><geom name="b" type="mesh" mesh="cube"/></body>"""


def test_poly_manifold_deep_pair_of_one_mesh(tmp_path):
    """Two geoms of one mesh share its face range (the compiler caches hulls
    per mesh), 8 mm deep, so the all-face SAT runs: the winning axis is g2's
    bottom face (b), not g1's face of the same index (the kernel
    credited it to g1 and fell back to MPR's single contact).  The tilted
    cube's top edge clipped to b's bottom face: two contacts, normal +z."""
    m = _scene(tmp_path, SHARED_MESH_DEEP)
    ga, gb = m.names["geom"].index("a"), m.names["geom"].index("b")
    assert m.geom_faceadr[ga] == m.geom_faceadr[gb] >= 0
    c = _active(m)
    ab = c.get(("a", "b")) or c.get(("b", "a"))
    assert ab is not None and len(ab) == 2
    depth = 0.05 * (np.cos(0.3) + np.sin(0.3)) + 0.05 - (0.30454 - 0.2)
    for dist, _, n in ab:
        assert abs(dist + depth) < 1e-6 and abs(abs(n[2]) - 1) < 1e-12
    assert sorted(round(p[0], 6) for _, p, _ in ab) == [-0.04, 0.05]  # the edge clipped to b's face


def test_plane_cylinder_four_points(tmp_path):
    """Plane-cylinder (MuJoCo's mjc_PlaneCylinder restated): an upright
    cylinder 3 mm into the floor gets the deepest rim point, the two rim points
    120 degrees either side of it (all three at the same depth, an equilateral
    triangle on the bottom cap); its top cap stays clear."""
    m = _scene(tmp_path, """
    <body name="y" pos="0 0 0.097"><freejoint/><geom name="y" type="cylinder" size="0.05 0.1"/></body>""")
    c = _active(m)
    cs = c.get(("floor", "y")) or c.get(("y", "floor"))
    assert len(cs) == 3
    for dist, pos, n in cs:
        assert abs(dist + 0.003) < 1e-9 and abs(n[2] - 1) < 1e-12
        assert abs(np.hypot(pos[0], pos[1]) - 0.05) < 1e-9
    ang = sorted(np.degrees(np.arctan2(p[1], p[0])) % 360 for _, p, _ in cs)
    gaps = np.diff(ang + [ang[0] + 360])
    assert np.allclose(gaps, 120, atol=1e-6)


def test_finger_hull_contact_is_precision_stable(dual):
    """The Hand-E's two finger hulls interpenetrate ~2 cm on C4's selected
    candidate (558 of the seed-4 shard): the SAT face picked
    for the polyhedron manifold can clip the incident face to nothing, and the
    pair then takes one contact at the incident support vertex along the
    reference normal -- not MPR's normal, whose portal path differed between
    fp32 and fp64 by 0.06 (the GPU-vs-oracle miss of 2.3e-4 on the selected
    cost).  At the traced steps the fp64 oracle and its fp32 build now agree
    on that contact's normal and depth."""
    import torch

    from manipulator_mujoco_amd.projection import ProjectionFilter
    m, H = dual, 100
    B, G = m.names["body"], m.geom_bodyid
    pair = next(p for p in range(m.npair)
                if {B[G[m.pair_geom1[p]]], B[G[m.pair_geom2[p]]]} == {"hande_left_finger", "hande_right_finger"})
    _, P, Pd, Pdd = basis.planner_basis(H, 0.05)
    f = ProjectionFilter(P, Pd, Pdd, 6, torch.device("cpu"))
    rng = np.random.default_rng(20250629 + 4)
    xi = torch.tensor(rng.normal(0, np.sqrt(10.003), (4096, 66)).astype(np.float32))[[558]]
    q0 = np.array([1.5, -1.8, 1.75, -1.25, -1.6, 0.0])
    xi = f(xi, f.boundary(q0, np.zeros(6), np.zeros(6), 1), 10).numpy()
    td = np.einsum("tk,njk->njt", Pd, xi.reshape(1, 6, 11).astype(np.float64)).reshape(6, H)
    qa, da = np.asarray(m.ctrl_qposadr[:6]), np.asarray(m.ctrl_dofadr[:6])
    qpos = np.array(m.qpos_init[:m.nq], dtype=np.float64)
    qpos[qa] = q0
    qvel, ws = np.array(m.qvel_init[:m.nv], dtype=np.float64), np.zeros(m.nv)
    checked = 0
    for t in range(66):
        qv = qvel.copy()
        qv[da] = td[:, t]
        if t in (30, 54, 65):
            o64 = oracle.step_debug(m, qpos, qv, ws)
            o32 = oracle.step_debug(m, qpos, qv, ws, precision="fp32")
            k64 = [k for k in range(o64["ncon"]) if o64["con_pair"][k] == pair]
            k32 = [k for k in range(o32["ncon"]) if o32["con_pair"][k] == pair]
            if k64 and k32:
                checked += 1
                assert np.abs(o64["con_normal"][k64[0]] - o32["con_normal"][k32[0]]).max() < 1e-3
                assert abs(min(o64["con_dist"][k] for k in k64) - min(o32["con_dist"][k] for k in k32)) < 1e-5
        st = oracle.step(m, qpos, qv, ws)
        qpos, qvel, ws = st["qpos"], st["qvel"], st["qacc_warmstart"]
    assert checked >= 2
