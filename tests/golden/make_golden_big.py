"""Golden Newton steps at the BASELINE sizes C2 (n=1024, m=2048) and C3 (n=4096, m=8192), from the CPU oracle.

The problem itself is NOT stored (A alone is 268 MB at C3): the GPU test regenerates it with
cvx_amd.problems.random_qp(n, m, instance) and first checks the fingerprint recorded here (SHA-256 of the
RNG-only arrays A and ub; sums of the BLAS-derived P and a0, which may differ in the last bit between BLAS
thread counts and are checked to 1e-12 relative).

The trajectory is the oracle's barrier t-loop (oracle.unconstrained_solve, warm start, t = 1, 10, ...) from
x0 = 0 up to the second step of the t = 1e4 centering, with H formed in BLAS order (t P + A' diag(1/d^2) A,
oracle._barrier_hessian_blas) and LAPACK substitutions: the per-constraint fold of n x n outer products
would take minutes per Hessian at C3.  At the recorded steps the direction is recomputed from the fixture's
(t, x, grad):
  * C2: with the reference's per-constraint fold (BarrierSolver.scala:303-315, oracle.barrier_hessian) and the
    scalar substitutions (MatrixUtils.scala:383-430) -- the literal restatement;
  * C3: with the BLAS-ordered H and dtrtrs (hess_form = "blas" in the fixture).
The line-search decisions (accepted step, both backtracking counters) are the reference's line search
(UnconstrainedSolver.scala:83-113, oracle.unconstrained_line_search) run on that direction from the
recorded (iteration, frozen trust radius).

Late in the path (t >= 1e6) H is ill-conditioned, so the test holds those steps to backward-error, decrement-side and
line-search-replay criteria instead of the 1e-8 direction bar.  C2 is also solved to the standard termination: its
final x, per-centering step counts and active sets (separated threshold and Constraint.isActive's 1e-12) are stored.

C3LATE (round 5) pins the late C3 path (t = 1e10 .. 1e12) at the engine's own states: see make_late.

Run:  python tests/golden/make_golden_big.py [C2] [C3] [C3LATE[=states.npz]]   (C3 takes several minutes and ~6 GB
of RAM)
"""
from __future__ import annotations

import hashlib
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from cvx_amd import problems as Z  # noqa: E402
from oracle import cvx_oracle as O  # noqa: E402

CONFIGS = {
    # name: (n, m, instance, recorded (t, iteration-within-centering) pairs, form of the recorded directions)
    "C2": (1024, 2048, 0, [(1.0, 0), (1.0, 1), (1e2, 0), (1e4, 0), (1e4, 1),
                           (1e6, 0), (1e6, 1), (1e8, 0), (1e8, 1), (1e11, 0), (1e11, 1)], "fold"),
    "C3": (4096, 8192, 0, [(1.0, 0), (1e2, 0), (1e4, 0), (1e4, 1), (1e6, 0), (1e6, 1), (1e8, 0), (1e8, 1)], "blas"),
}
# Newton steps per centering at most, for t above 1e4, on the way to the late recorded states (C3 only: there a
# centering from t = 1e7 on runs into maxIter = 1000 on the oracle's rounding noise, ~80 minutes each on the CPU).  A
# recorded state is a test input (t, x, grad) with the oracle's outputs at it, so an x reached after capped centerings
# is as good a late-path point as the fully centred one.
LATE_CAP = {"C3": 40}
# configurations whose whole barrier solve is run to the standard termination (gap < tolSolver): the final x, the
# per-centering Newton step counts and the active sets at the separated threshold and at Constraint.isActive's 1e-12
FULL = {"C2"}
ACTIVE_SEPARATED = 1e-6


def fingerprint(spec):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(spec["A"]).tobytes())
    h.update(np.ascontiguousarray(spec["ub"]).tobytes())
    return h.hexdigest(), float(np.sum(spec["P"])), float(np.sum(spec["a0"]))


def make(name):
    n, m, inst, want, form = CONFIGS[name]
    t0 = time.time()
    spec = Z.random_qp(n, m, instance=inst)
    pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
    pars = O.standard_params()
    sha, psum, a0sum = fingerprint(spec)
    t_last = max(t for t, _ in want)
    full = name in FULL
    x = spec["x0"].copy()
    t = 1.0
    states = []  # (t, it_n, radius, x, grad)
    per_centering = []  # Newton steps of each centering (full solves)
    gap = float("inf")
    # the reference's t-loop (BarrierSolver.scala:70-117): until gap = m/t < tolSolver (full) or past t_last
    while (gap >= pars.tolSolver) if full else (t <= t_last):
        max_steps = max(k for tt, k in want if tt == t) + 1 if (t == t_last and not full) else None
        if t > 1e4 and name in LATE_CAP and max_steps is None:
            max_steps = LATE_CAP[name]
        sol = O.unconstrained_solve(pb, t, x, pars, record=True, max_steps=max_steps, hess="blas", fast_subst=True)
        for rc in sol.records:
            if (t, rc.it_n) in want and rc.newton_decrement > pars.tolSolver:
                states.append((t, rc.it_n, rc.radius, rc.x.copy(), rc.grad.copy()))
        print(f"{name}: t={t:g} {sol.newton_steps} steps ({time.time() - t0:.0f} s)", flush=True)
        per_centering.append(sol.newton_steps)
        x = sol.x
        gap = m / t
        t *= 10.0
    x_final = x.copy()
    missing = [w for w in want if w not in [(s_[0], s_[1]) for s_ in states]]
    if missing:  # a centering that ends before its second step (or a final decrement below tol) has nothing there
        print(f"{name}: not recorded (no such moving step): {missing}", flush=True)
    out = {k: [] for k in ("t", "it_n", "radius", "x", "grad", "f", "dx", "q", "step", "kc", "ka", "ruiz", "reg",
                           "rel_err")}
    for (t, it_n, radius, x, g) in states:
        rec = O.NewtonStepRecord(x=x, grad=g, f=0.0, dx=None, q=0.0, newton_decrement=0.0)
        if form == "fold":
            d = O.newton_direction(pb, t, x, g, pars.tolEqSolve, rec)
        else:
            d = O.newton_direction(pb, t, x, g, pars.tolEqSolve, rec, fast_subst=True, hess="blas")
        assert rec.fallback == 0
        q = float(np.dot(d, g))
        if it_n == 0:
            radius = math.sqrt(-q)
        f = O.barrier_value(pb, t, x)
        _, st, k1, it = O.unconstrained_line_search(pb, t, x, d, q, f, it_n, radius, pars)
        for k, v in (("t", t), ("it_n", it_n), ("radius", radius), ("x", x), ("grad", g), ("f", f), ("dx", d),
                     ("q", q), ("step", st), ("kc", k1), ("ka", it - k1), ("ruiz", rec.ruiz_sweeps),
                     ("reg", rec.regularized), ("rel_err", rec.rel_err)):
            out[k].append(v)
        print(f"{name}: t={t:g} it={it_n} q={q:.6e} step={st:g} kc={k1} ka={it - k1} ruiz={rec.ruiz_sweeps} "
              f"reg={rec.regularized}", flush=True)
    arrays = {k: np.array(v) for k, v in out.items()}
    if full:  # the whole solve: final x, step counts per centering, active sets (Constraint.isActive, :26)
        x = x_final
        g = pb.r + pb.A @ x
        marg = np.abs(g - pb.ub)
        act_sep = np.nonzero(marg < ACTIVE_SEPARATED)[0]
        act_12 = np.nonzero(marg < 1e-12)[0]
        # separation of the threshold: no margin within a factor 100 of it
        near = np.sum((marg > ACTIVE_SEPARATED / 100) & (marg < ACTIVE_SEPARATED * 100))
        print(f"{name}: final gap {gap:.3e}, {sum(per_centering)} Newton steps {per_centering}, active "
              f"{len(act_sep)} (< {ACTIVE_SEPARATED:g}; {near} margins within 100x), {len(act_12)} (< 1e-12)")
        arrays.update(x_final=x, gap=np.array(gap), per_centering=np.array(per_centering),
                      active_sep=act_sep, active_1e12=act_12, active_threshold=np.array(ACTIVE_SEPARATED),
                      active_near=np.array(near))
    arrays.update(n=np.array(n), m=np.array(m), instance=np.array(inst), sha256=np.array(sha), P_sum=np.array(psum),
                  a0_sum=np.array(a0sum), hess_form=np.array(form))
    path = os.path.join(HERE, "big", f"{name}_n{n}_m{m}.npz")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.savez_compressed(path, **arrays)
    print(f"{name}: wrote {path} ({os.path.getsize(path) / 1e3:.0f} KB, {time.time() - t0:.0f} s)")


def make_late(states_path):
    """C3LATE: the late C3 path (t = 1e10 .. 1e12, where a full solve spends 96 % of its Newton steps) at states of the
    ENGINE's own C3 solve (scripts/c3_late_states.py on the GPU: the iterate entering inner iterations 0 and 1 of each
    late centering and its first regularized steps, with the centering's frozen trust radius).  At each state the
    oracle computes the gradient, the BLAS-ordered Hessian's Newton direction (Ruiz, regularizedCholesky, dtrtrs,
    MatrixUtils.scala:240-516), its backward error, the FIRST attempt's min diag(L) of chol(Q) (MatrixUtils.scala:456-458:
    <= 1e-7 sends the step to Q + 1e-10 I) and the reference's line search from the recorded (iteration, radius)
    (UnconstrainedSolver.scala:83-113).  The engine's own records ride along (engine_*)."""
    from scipy.linalg import lapack
    n, m, inst = 4096, 8192, 0
    t0 = time.time()
    st = dict(np.load(states_path))
    spec = Z.random_qp(n, m, instance=inst)
    pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
    pars = O.standard_params()
    sha, psum, a0sum = fingerprint(spec)
    out = {k: [] for k in ("t", "it_n", "radius", "x", "grad", "f", "dx", "q", "step", "kc", "ka", "ruiz", "reg",
                           "rel_err", "min_diag0", "info0", "rel_err_alt")}
    for k in range(st["t"].shape[0]):
        t, it_n, radius, x = float(st["t"][k]), int(st["it_n"][k]), float(st["radius"][k]), st["x"][k]
        g = O.barrier_gradient(pb, t, x)
        rec = O.NewtonStepRecord(x=x, grad=g, f=0.0, dx=None, q=0.0, newton_decrement=0.0)
        d = O.newton_direction(pb, t, x, g, pars.tolEqSolve, rec, fast_subst=True, hess="blas")
        assert rec.fallback == 0
        H = O.barrier_hessian(pb, t, x, literal="blas")
        dR, Q, _ = O.ruiz_equilibrate(H)
        L0, info0 = lapack.dpotrf(Q, lower=1, clean=1)
        mind0 = float(np.min(np.diag(L0))) if info0 == 0 else float("nan")
        # the other branch of regularizedCholesky at this state (its backward error): where the branch decision is below
        # FP64's resolution the engine may legitimately take it
        Qa = Q + np.eye(n) * 1e-10 if rec.regularized == 0 else Q
        La, infoa = lapack.dpotrf(Qa, lower=1, clean=1)
        rel_alt = float("nan")
        if infoa == 0:
            w_ = O.triangular_solve(La, "L", (dR * -g)[:, None])[:, 0]
            u_ = O.triangular_solve(La.T, "U", w_[:, None])[:, 0]
            rel_alt = O.relative_size(H @ (dR * u_) + g, -g, pars.tolEqSolve)
        del H, Q, L0, Qa, La
        q = float(np.dot(d, g))
        if it_n == 0:
            radius = math.sqrt(-q)
        f = O.barrier_value(pb, t, x)
        _, stp, k1, it = O.unconstrained_line_search(pb, t, x, d, q, f, it_n, radius, pars)
        for key, v in (("t", t), ("it_n", it_n), ("radius", radius), ("x", x), ("grad", g), ("f", f), ("dx", d),
                       ("q", q), ("step", stp), ("kc", k1), ("ka", it - k1), ("ruiz", rec.ruiz_sweeps),
                       ("reg", rec.regularized), ("rel_err", rec.rel_err), ("min_diag0", mind0), ("info0", info0),
                       ("rel_err_alt", rel_alt)):
            out[key].append(v)
        print(f"C3LATE: t={t:g} it={it_n} q={q:.6e} step={stp:g} kc={k1} ka={it - k1} ruiz={rec.ruiz_sweeps} "
              f"reg={rec.regularized} (first attempt min diag {mind0:.3e}, info {info0}; engine reg "
              f"{int(st['regularized'][k])} min diag {float(st['min_diag'][k]):.3e}) rel_err {rec.rel_err:.2e} (other "
              f"branch {rel_alt:.2e}) "
              f"({time.time() - t0:.0f} s)", flush=True)
    arrays = {k: np.array(v) for k, v in out.items()}
    for key in ("step", "backtracks_c", "backtracks_armijo", "ruiz_sweeps", "regularized", "min_diag", "rel_err", "q",
                "ls_ties", "small_pivot"):
        arrays["engine_" + key] = st[key]
    arrays.update(n=np.array(n), m=np.array(m), instance=np.array(inst), sha256=np.array(sha), P_sum=np.array(psum),
                  a0_sum=np.array(a0sum), hess_form=np.array("blas"), source=np.array("engine states"))
    path = os.path.join(HERE, "big", f"C3late_n{n}_m{m}.npz")
    np.savez_compressed(path, **arrays)
    print(f"C3LATE: wrote {path} ({os.path.getsize(path) / 1e3:.0f} KB, {time.time() - t0:.0f} s)")


def make_whole(threads=6):
    """C3WHOLE (round 6): the oracle's WHOLE C3 barrier solve with the standard parameters, the reference's t-loop
    (BarrierSolver.scala:70-117) around UnconstrainedSolver.solve (UnconstrainedSolver.scala:34-125), with the
    BLAS-ordered Hessian (a per-constraint fold would take minutes per step at n = 4096).  Stored: the per-centering
    Newton step counts, the x entering every centering, the final x and gap, and one scalar record per Newton step
    (t, iteration, q, step, both backtracking counters, Ruiz sweeps, regularization flag, fallback, backward error);
    plus the x and dx of the first two steps of each centering, so the engine's first steps from the oracle's
    centering start can be compared directly.  A partial file is rewritten after every centering (the three
    t = 1e10 .. 1e12 centerings run to maxIter, ~1000 steps each)."""
    from threadpoolctl import threadpool_limits
    n, m, inst = 4096, 8192, 0
    t0 = time.time()
    spec = Z.random_qp(n, m, instance=inst)
    pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
    pars = O.standard_params()
    sha, psum, a0sum = fingerprint(spec)
    keys = ("t", "it_n", "q", "f", "step", "kc", "ka", "ruiz", "reg", "fallback", "rel_err")
    steps = {k: [] for k in keys}
    first = {"t": [], "it_n": [], "x": [], "dx": []}
    x_start, per_centering, ts = [], [], []
    path = os.path.join(HERE, "big", f"C3whole_n{n}_m{m}.npz")

    def save(x, gap, done):
        arrays = {("step_" + k): np.array(v) for k, v in steps.items()}
        arrays.update({("first_" + k): np.array(v) for k, v in first.items()})
        arrays.update(x_start=np.array(x_start), per_centering=np.array(per_centering), t_centering=np.array(ts),
                      x_final=x, gap=np.array(gap), complete=np.array(done), n=np.array(n), m=np.array(m),
                      instance=np.array(inst), sha256=np.array(sha), P_sum=np.array(psum), a0_sum=np.array(a0sum),
                      hess_form=np.array("blas"), blas_threads=np.array(threads))
        np.savez_compressed(path, **arrays)

    cur = {"t": 1.0}

    def on_step(rc):
        for k, v in (("t", cur["t"]), ("it_n", rc.it_n), ("q", rc.q), ("f", rc.f), ("step", rc.step),
                     ("kc", rc.backtracks_c), ("ka", rc.backtracks_armijo), ("ruiz", rc.ruiz_sweeps),
                     ("reg", rc.regularized), ("fallback", rc.fallback), ("rel_err", rc.rel_err)):
            steps[k].append(v)
        if rc.it_n < 2:
            first["t"].append(cur["t"])
            first["it_n"].append(rc.it_n)
            first["x"].append(rc.x.copy())
            first["dx"].append(rc.dx.copy())
        if rc.it_n % 25 == 0:
            print(f"C3WHOLE: t={cur['t']:g} it={rc.it_n} q={rc.q:.3e} step={rc.step:g} reg={rc.regularized} "
                  f"({time.time() - t0:.0f} s)", flush=True)
        if rc.it_n % 25 == 24:  # a centering in progress: its steps so far, readable if the run is stopped
            np.savez_compressed(path.replace(".npz", "_inprogress.npz"), t=np.array(cur["t"]), x_start=x_start[-1],
                                **{("step_" + k): np.array(v) for k, v in steps.items()})

    x = spec["x0"].copy()
    t = 1.0
    gap = float("inf")
    if os.path.exists(path):  # resume after the last complete centering of a partial file
        old = dict(np.load(path))
        if not bool(old["complete"]) and str(old["sha256"]) == sha:
            for k in keys:
                steps[k] = list(old["step_" + k])
            for k in first:
                first[k] = list(old["first_" + k])
            x_start, per_centering, ts = list(old["x_start"]), list(old["per_centering"]), list(old["t_centering"])
            x, gap, t = old["x_final"].copy(), float(old["gap"]), float(ts[-1]) * 10.0
            print(f"C3WHOLE: resuming at t={t:g} after {per_centering}", flush=True)
    with threadpool_limits(threads):
        while gap >= pars.tolSolver and len(per_centering) < 100:
            cur["t"] = t
            x_start.append(x.copy())
            ts.append(t)
            sol = O.unconstrained_solve(pb, t, x, pars, hess="blas", fast_subst=True, on_step=on_step)
            per_centering.append(sol.newton_steps)
            x = sol.x
            gap = m / t
            print(f"C3WHOLE: t={t:g} {sol.newton_steps} steps, counts so far {per_centering} "
                  f"({time.time() - t0:.0f} s)", flush=True)
            save(x, gap, gap < pars.tolSolver)
            t *= 10.0
    print(f"C3WHOLE: wrote {path} ({os.path.getsize(path) / 1e3:.0f} KB, {time.time() - t0:.0f} s), "
          f"{sum(per_centering)} Newton steps {per_centering}, gap {gap:.3e}")


if __name__ == "__main__":
    for nm in (sys.argv[1:] or ["C2", "C3"]):
        if nm == "C3WHOLE":
            make_whole()
        elif nm.startswith("C3LATE"):  # C3LATE=<states.npz from scripts/c3_late_states.py>
            make_late(nm.split("=", 1)[1] if "=" in nm else os.path.join(HERE, "..", "..", "gpurun_out",
                                                                         "c3_late_states.npz"))
        else:
            make(nm)
