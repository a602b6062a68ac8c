"""Which part of the Newton solver makes fp32 lose parity?  (CPU experiment)

Builds variants of the fp32 oracle (oracle_f32.c) in which chosen parts of the
constraint solver (mpcr_oracle.c solve() and its helpers) run in fp64 from the
fp32 inputs (J, D, aref, M), and counts, on a batch of the parity tests, the
well-conditioned candidates (tests/parity_util.py) each variant moves by more
than 1e-4 against the fp64 oracle.  Parts (any '+'-joined subset; everything
else stays fp32):
  book   line-search point costs / derivatives, step sizes and bracket
         arithmetic (lspt), the Gauss-term quadratic sums, cost bookkeeping
  jar    J qacc - aref;  jv  J search;  mulM  M x;  grad  J^T f;  hess  J^T D J
  ls     the line search's row sums;  force  row forces / cone update
  cost   the solver cost;  chol  the Cholesky factor / solve;  upd  the qacc update
  all    the whole solver
The source is the oracle of git revision REV (default: before the round-4
change that made the fp32 build keep `book`'s line-search part in fp64).

    python tools/oracle_precision.py [model=dual_arm] [n=1024] [H=100] [seed=4] [variants=none,book,all]
Writes its sources and libraries to /tmp/oracle_precision/.
"""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

OUT = "/tmp/oracle_precision"
REV = os.environ.get("REV", "76a4230")


def _body_to_float(src, fname):
    m = re.search(r"\n(static [^\n]*\b%s\([^{]*\{)" % re.escape(fname), src)
    start = m.end()
    depth, j = 1, start
    while depth:
        depth += {"{": 1, "}": -1}.get(src[j], 0)
        j += 1
    body = src[start:j].replace("hpd", "float")
    # scratch arrays handed to fp64 callees stay fp64
    body = body.replace("memset(H, 0, 9 * sizeof(float));", "memset(H, 0, 9 * sizeof(hpd));")
    body = body.replace("float gauss = 0, f[MAXEFC];", "float gauss = 0; hpd f[MAXEFC];")
    body = body.replace("      float c[3];\n      ell_line_hp", "      hpd c[3];\n      ell_line_hp")
    body = body.replace("float H[3][3];\n      c += ell_update_hp", "hpd H[3][3];\n      c += ell_update_hp")
    return src[:start] + body + src[j:]


def variant_source(src, keep):
    """The oracle with solve() (and chol) duplicated as *_hp in fp64, then the
    parts not in `keep` turned back to fp32."""
    lines = src.split("\n")
    find = lambda pat, s=0: next(i for i in range(s, len(lines)) if re.match(pat, lines[i]))  # noqa: E731
    a = find(r"^typedef struct \{ double alpha, cost, d0, d1; \} lspt;")
    b = find(r"^/\* step = forward \+ Euler", a) - 2
    block = "\n".join(lines[a:b])
    for nm in ["mulM", "ell_update", "efc_cost_force", "solver_cost", "eval_jar", "ell_line", "ls_eval", "solve",
               "lspt", "chol", "chol_solve"]:
        block = re.sub(r"\b%s\b" % nm, nm + "_hp", block)
    block = re.sub(r"\bdouble\b", "hpd", block)
    rep = [("memcpy(d->qacc, d->qacc_smooth, sizeof(hpd) * nv);", "for (int i_ = 0; i_ < nv; i_++) d->qacc[i_] = d->qacc_smooth[i_];"),
           ("memcpy(qacc, cw < cs ? d->qacc_warmstart : d->qacc_smooth, sizeof(hpd) * nv);",
            "for (int i_ = 0; i_ < nv; i_++) qacc[i_] = cw < cs ? d->qacc_warmstart[i_] : d->qacc_smooth[i_];"),
           ("memcpy(qacc, d->qacc_smooth, sizeof(hpd) * nv);", "for (int i_ = 0; i_ < nv; i_++) qacc[i_] = d->qacc_smooth[i_];"),
           ("memcpy(d->qacc, qacc, sizeof(hpd) * nv);", "for (int i_ = 0; i_ < nv; i_++) d->qacc[i_] = qacc[i_];"),
           ("efc_cost_force_hp(d, jar, d->efc_force);",
            "{ hpd ff_[MAXEFC]; efc_cost_force_hp(d, jar, ff_); for (int r_ = 0; r_ < nefc; r_++) d->efc_force[r_] = ff_[r_]; }"),
           ("    hpd Mw[NV], jw[MAXEFC], Ms[NV], js[MAXEFC];",
            "    hpd Mw[NV], jw[MAXEFC], Ms[NV], js[MAXEFC], qw_[NV], qs_[NV];\n"
            "    for (int i_ = 0; i_ < nv; i_++) { qw_[i_] = d->qacc_warmstart[i_]; qs_[i_] = d->qacc_smooth[i_]; }"),
           ("mulM_hp(m, d, d->qacc_warmstart, Mw);", "mulM_hp(m, d, qw_, Mw);"),
           ("eval_jar_hp(m, d, d->qacc_warmstart, jw);", "eval_jar_hp(m, d, qw_, jw);"),
           ("mulM_hp(m, d, d->qacc_smooth, Ms);", "mulM_hp(m, d, qs_, Ms);"),
           ("eval_jar_hp(m, d, d->qacc_smooth, js);", "eval_jar_hp(m, d, qs_, js);"),
           ("solver_cost_hp(m, d, d->qacc_warmstart, Mw, jw), cs = solver_cost_hp(m, d, d->qacc_smooth, Ms, js);",
            "solver_cost_hp(m, d, qw_, Mw, jw), cs = solver_cost_hp(m, d, qs_, Ms, js);")]
    for x, y in rep:
        assert x in block, x
        block = block.replace(x, y)
    ca = find(r"^static int chol\(double L\[NV\]\[NV\]")
    cb = find(r"^/\* -{10,}", ca)
    chol = re.sub(r"\bchol_solve\b", "chol_solve_hp", re.sub(r"\bchol\b", "chol_hp", "\n".join(lines[ca:cb])))
    chol = re.sub(r"\bdouble\b", "hpd", chol)
    out = "\n".join(lines[:b]) + "\n" + chol + "\n" + block + "\n" + "\n".join(lines[b:])
    out = out.replace("  solve(m, d);\n}", "  solve_hp(m, d);\n}")
    if "all" in keep:
        return out
    parts = {"jar": ["eval_jar_hp"], "ls": ["ls_eval_hp", "ell_line_hp"], "force": ["efc_cost_force_hp", "ell_update_hp"],
             "mulM": ["mulM_hp"], "cost": ["solver_cost_hp"], "chol": ["chol_hp", "chol_solve_hp"]}
    for p, fs in parts.items():
        if p not in keep:
            for f in fs:
                out = _body_to_float(out, f)
    edits = {
        "hess": [("hpd h = d->M[i][j];", "float h = d->M[i][j];"), ("          hpd h = 0;", "          float h = 0;")],
        "grad": [("hpd qc = 0;\n      for (int r = 0; r < nefc; r++) qc += d->efc_J[r][i] * f[r];",
                  "float qc = 0;\n      for (int r = 0; r < nefc; r++) qc += (float)(d->efc_J[r][i] * (float)f[r]);")],
        "jv": [("      hpd s = 0;\n      for (int i = 0; i < nv; i++) s += d->efc_J[r][i] * search[i];",
                "      float s = 0;\n      for (int i = 0; i < nv; i++) s += d->efc_J[r][i] * (float)search[i];")],
        "upd": [("for (int i = 0; i < nv; i++) { qacc[i] += alpha * search[i]; Ma[i] += alpha * Mv[i]; }\n"
                 "      for (int r = 0; r < nefc; r++) jar[r] += alpha * jv[r];",
                 "for (int i = 0; i < nv; i++) { qacc[i] = (float)qacc[i] + (float)alpha * (float)search[i]; "
                 "Ma[i] = (float)Ma[i] + (float)alpha * (float)Mv[i]; }\n"
                 "      for (int r = 0; r < nefc; r++) jar[r] = (float)jar[r] + (float)alpha * (float)jv[r];")],
        "book": [("typedef struct { hpd alpha, cost, d0, d1; } lspt_hp;", "typedef struct { float alpha, cost, d0, d1; } lspt_hp;"),
                 ("    hpd gauss = 0, q1 = 0, q2 = 0;", "    float gauss = 0, q1 = 0, q2 = 0;"),
                 ("  hpd cost = solver_cost_hp(m, d, qacc, Ma, jar), prev_cost = 1e300;",
                  "  float cost = solver_cost_hp(m, d, qacc, Ma, jar), prev_cost = 1e30f;"),
                 ("    hpd gn = 0;", "    float gn = 0;"),
                 ("    hpd Mv[NV], jv[MAXEFC], sn = 0;", "    hpd Mv[NV], jv[MAXEFC]; float sn = 0;"),
                 ("    hpd alpha = lo.cost < hi.cost ? lo.alpha : hi.alpha;", "    float alpha = lo.cost < hi.cost ? lo.alpha : hi.alpha;")],
    }
    for p, reps in edits.items():
        if p not in keep:
            for x, y in reps:
                assert x in out, x
                out = out.replace(x, y)
    return out


def build(keep):
    os.makedirs(OUT, exist_ok=True)
    name = "_".join(sorted(keep)) or "none"
    src = subprocess.check_output(["git", "-C", ROOT, "show", f"{REV}:oracle/mpcr_oracle.c"], text=True)
    inc = os.path.join(ROOT, "include") + "/"
    with open(f"{OUT}/oracle_{name}.c", "w") as f:
        f.write(variant_source(src, keep).replace('"../include/', '"' + inc))
    f32 = open(os.path.join(ROOT, "oracle", "oracle_f32.c")).read()
    f32 = re.sub(r"typedef double mpcr_hp;[^\n]*\n#define MPCR_HP_DEFINED\n", "", f32)
    f32 = f32.replace('#include "mpcr_oracle.c"', f'#include "{OUT}/oracle_{name}.c"')
    f32 = f32.replace("#define double float", "typedef double hpd;\n#define double float").replace('"../include/', '"' + inc)
    with open(f"{OUT}/f32_{name}.c", "w") as f:
        f.write(f32)
    lib = f"{OUT}/lib_{name}.so"
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-fPIC", "-w", "-fsingle-precision-constant", "-shared", "-o", lib,
                           f"{OUT}/f32_{name}.c", "-lm"])
    return name, lib


def main():
    import oracle
    import parity_util as pu
    from diag_f32 import batch
    from manipulator_mujoco_amd import models
    a = sys.argv[1:]
    model = a[0] if a else "dual_arm"
    n = int(a[1]) if len(a) > 1 else 1024
    H = int(a[2]) if len(a) > 2 else 100
    seed = int(a[3]) if len(a) > 3 else 4
    variants = (a[4] if len(a) > 4 else "none,book,all").split(",")
    m = models.load(model, 0.05)
    td = batch(m, n, H, seed)
    with oracle.exact(4):
        o, sens = pu.conditioning(m, td)
    well = (sens < pu.TOL / 10) & ~pu.grazing(m, o)
    oc = o["cost4"][:, 0]
    print(f"{model} {n} x {H} seed {seed}: well {int(well.sum())}, probe B well-misses "
          f"{int((well & (o['probe_b'] >= pu.TOL)).sum())}")
    for v in variants:
        keep = set() if v == "none" else set(v.split("+"))
        name, path = build(keep)
        L = ctypes.CDLL(path)
        base = oracle.lib_f32()
        L.oracle_rollout.argtypes, L.oracle_rollout.restype = base.oracle_rollout.argtypes, ctypes.c_int
        L.oracle_set_exact(4)
        oracle._LIB32 = L
        run = oracle.Runner(m, pu.WORKERS, pu.Q0, pu.W, pu.PT, pu.QT, precision="fp32")
        c = run.rollout(td).astype(np.float64)[:, 0]
        run.close()
        oracle._LIB32 = None
        r = np.abs(c - oc) / np.abs(oc)
        print(f"  fp64 parts {v:28s} well-conditioned misses {int((well & (r >= pu.TOL)).sum()):4d}  "
              f"all misses {(r >= pu.TOL).mean():.3f}  worst well {r[well].max():.1e}")


if __name__ == "__main__":
    main()
