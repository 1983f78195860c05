"""Benchmark: Newton KKT solves/s of the MI355X barrier engine on the C3 random dense QP (n=4096, m=8192).

One "step" = one full inner Newton iteration of the barrier method on device-resident data: barrier
gradient (2 GEMV passes over A), Hessian assembly H = tP + A'diag(1/d^2)A (FP64 MFMA SYRK), Ruiz
equilibration, regularised blocked Cholesky with the fused forward solve, backward solve, residual check,
the backtracking line search and the iterate update (UnconstrainedSolver.scala:47-134).  The t-loop
(BarrierSolver.scala:70-117) advances t *= 10 when a centering terminates, as the reference does.

N > 1: one process per GPU, an independent instance per rank (config C5, seed 20261015 + rank), no
collective inside the timed region except the bracketing barrier; value = total steps / max-rank time;
one gather of the per-rank results to rank 0 afterwards.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Newton KKT solves/sec at n=4096 m=8192; % MFMA roofline on trailing SYRK"
FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix peak (spec)
HBM_PEAK_GBS = 8000.0


def _fold_sample(job):
    """One single-thread worker of the fold sample: the rank-1 fold of BarrierSolver.scala:303-315 (with the
    reference's n x n temporaries) over a contiguous run of constraints in list order, starting from t P; returns the
    per-constraint wall times (stops early at the time budget)."""
    P, A_rows, r_rows, ub_rows, x, budget = job
    from threadpoolctl import threadpool_limits
    n = P.shape[0]
    per = []
    with threadpool_limits(1):
        s = P * 1.0
        t0 = time.perf_counter()
        for k in range(A_rows.shape[0]):
            tk = time.perf_counter()
            d = ub_rows[k] - (r_rows[k] + float(np.dot(A_rows[k], x)))  # LinearConstraint.valueAt
            G = A_rows[k]
            s = s + np.outer(G, G) / (d * d) + np.zeros((n, n)) / d
            per.append(time.perf_counter() - tk)
            if time.perf_counter() - t0 > budget:
                break
    return per


def cpu_baseline(spec, seconds_budget: float = 30.0, fraction: float = 0.25, workers: int = 0):
    """Reference-faithful CPU port timed on this host (oracle/cvx_oracle.py = restatement of the Breeze path):
    the per-constraint rank-1 Hessian fold of BarrierSolver.scala:303-315 with all of its n x n temporaries,
    timed on `fraction` of the constraints and scaled to m, plus one Ruiz + regularizedCholesky + substitution solve
    (MatrixUtils.scala:240-516) at full n, plus m dot products per line-search trial.  The fold sample is split into
    contiguous runs over a few concurrent single-thread worker processes (spawned children that touch no GPU) so that
    a quarter of C3's 8192 constraints fits the time budget; each per-constraint time is a single-thread cost (the
    concurrent workers share memory bandwidth, which can only make them slower).  Every constraint of the fold does
    identical work (n x n temporaries), so the per-constraint time is shape-invariant; the sample string states the
    sample size and spread."""
    import multiprocessing as mp

    from threadpoolctl import threadpool_limits

    from oracle import cvx_oracle as O
    n, m = spec["A"].shape[1], spec["A"].shape[0]
    pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
    x = spec["x0"]
    nw = workers or max(1, min(4, cpu_threads() // 2))
    want = max(1, int(round(fraction * m)))
    runs = np.array_split(np.arange(want), nw)
    jobs = [(spec["P"], spec["A"][r], spec["r"][r], spec["ub"][r], x, seconds_budget) for r in runs]
    t_wall = time.perf_counter()
    with mp.get_context("spawn").Pool(nw) as pool:
        per = [t for part in pool.map(_fold_sample, jobs) for t in part]
    t_wall = time.perf_counter() - t_wall
    k = len(per)
    t_fold = float(np.mean(per)) * m
    cv = float(np.std(per) / np.mean(per)) if k > 1 else 0.0
    with threadpool_limits(1):
        # (2) equilibrate + factor + solve at full size
        dd = spec["ub"] - spec["A"] @ x
        H = spec["P"] + spec["A"].T @ (spec["A"] / (dd * dd)[:, None])
        y = O.barrier_gradient(pb, 1.0, x)
        t1 = time.perf_counter()
        O.cholesky_solve(H, -y, 0.1, fast_subst=True)
        t_solve = time.perf_counter() - t1
        # (3) one barrier value + feasibility sweep per line-search trial (m dots of length n)
        t2 = time.perf_counter()
        for i in range(min(m, 2048)):
            O.constraint_value(pb, i, x)
        t_trial = (time.perf_counter() - t2) / min(m, 2048) * m * 2
    t_step = t_fold + t_solve + t_trial
    return {"value": 1.0 / t_step, "unit": "Newton KKT solves/s", "cores": 1, "kind": "port",
            "sample": (f"reference-faithful numpy port (oracle/cvx_oracle.py), single-thread costs: rank-1 Hessian "
                       f"fold timed on {k} of {m} constraints ({100.0 * k / m:.1f} %, {nw} concurrent single-thread "
                       f"workers, {t_wall:.1f} s wall; per-constraint time spread {100 * cv:.1f} % CV) and scaled to m "
                       f"({t_fold:.1f} s/Hessian), Ruiz+regularizedCholesky+dtrtrs solve at n={n} ({t_solve:.2f} s), "
                       f"2 trial sweeps ({t_trial:.2f} s); projected {t_step:.1f} s per Newton step")}


def ruiz_blas(H, max_iter: int = 20, tol: float = 1e-6):
    """MatrixUtils.scala:240-268 (Jacobi Ruiz) in GEMV form for the BLAS leg: |Q_i|_2 = d_i sqrt((S d^2)_i) with
    S = H o H formed once, so each sweep is one dgemv instead of three n x n passes."""
    S = H * H
    d = np.ones(H.shape[0])
    for _ in range(max_iter):
        u = np.sqrt(d * np.sqrt(S @ (d * d)))
        rho = float(np.max(np.abs(1.0 - u)))
        if rho <= tol:
            break
        d = d / np.where(u == 0.0, 1.0, u)
    return d


def cpu_threads() -> int:
    """Host threads for the BLAS leg: the job's CPU share (OMP_NUM_THREADS on the GPU box, 16 there), else nproc."""
    try:
        return max(1, int(os.environ.get("OMP_NUM_THREADS", "")))
    except ValueError:
        return max(1, os.cpu_count() or 1)


def cpu_baseline_blas(spec, steps: int = 3):
    """SURVEY.md §8d baseline (2): the BLAS-backed CPU equivalent of one Newton step on all of the job's host
    threads — barrier gradient (dgemv), H = tP + (A/d)'(A/d) (OpenBLAS dsyrk, lower), Ruiz equilibration
    (MatrixUtils.scala:240-268, vectorized), dpotrf('L') with the reference's regularisation test, two dtrsv and
    the residual.  Median of `steps` steps after one warm-up; wall clock."""
    from scipy.linalg import blas, lapack
    from threadpoolctl import threadpool_limits

    from oracle import cvx_oracle as O
    A, P, ub, x = spec["A"], spec["P"], spec["ub"], spec["x0"]
    n, m = A.shape[1], A.shape[0]
    nt = cpu_threads()
    t = 1.0
    times = []
    with threadpool_limits(nt):
        for it in range(steps + 1):
            t0 = time.perf_counter()
            d = ub - (spec["r"] + A @ x)
            y = t * (spec["a0"] + P @ x) + A.T @ (1.0 / d)
            As = A / d[:, None]
            H = blas.dsyrk(1.0, As, beta=t, c=P, trans=1, lower=1)
            H = np.tril(H) + np.tril(H, -1).T
            dr = ruiz_blas(H)
            Q = H * dr[:, None] * dr[None, :]
            L, info = lapack.dpotrf(Q, lower=1, clean=1)
            if info != 0 or np.min(np.diag(L)) <= 1e-7:
                L, info = lapack.dpotrf(Q + 1e-10 * np.eye(n), lower=1, clean=1)
            w = blas.dtrsv(L, dr * -y, lower=1)
            u = blas.dtrsv(L, w, lower=1, trans=1)
            dx = dr * u
            _ = np.linalg.norm(H @ dx + y)
            if it > 0:
                times.append(time.perf_counter() - t0)
    ts = float(np.median(times))
    return {"value": 1.0 / ts, "unit": "Newton KKT solves/s", "cores": nt, "kind": "port",
            "sample": (f"BLAS-backed CPU equivalent (SURVEY.md §8d (2)): numpy/scipy OpenBLAS dgemv + dsyrk + "
                       f"Ruiz + dpotrf + 2 dtrsv + residual at n={n} m={m}, {nt} threads, median of {steps} "
                       f"steps ({ts:.3f} s/step)")}


def latest_profile(name):
    """The newest committed profile file of that name (profiles/r06, then r05, r04, r03, r02)."""
    for r in ("r06", "r05", "r04", "r03", "r02"):
        p = os.path.join(ROOT, "profiles", r, name)
        if os.path.exists(p):
            return p
    return os.path.join(ROOT, "profiles", "r05", name)


PMC_TRAFFIC = latest_profile("pmc_traffic.json")
# the same rooflines recomputed from the committed rocprofv3 kernel trace of `bench.py --steps 20 --warmup 5
# --no-cpu-baseline` (scripts/trace_roofline.py: sums of kernel durations over the timed steps)
TRACE_ROOFLINE = latest_profile("trace_roofline.json")


def committed_whole_solve():
    """The newest committed C3FULL line (one complete C3 barrier solve with the standard parameters, `bench.py
    --workload C3FULL`): the whole-job rate, regularized steps included, beside the t = 1 window `value` times."""
    path = latest_profile("bench_c3full.json")
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        return None
    return {"source": os.path.relpath(path, ROOT), "note": "a committed C3FULL line, not measured by this run",
            "steps_per_s": d.get("value"), "newton_steps": d.get("steps"),
            "steps_per_centering": d.get("steps_per_centering"),
            "regularized_refactorizations": d.get("regularized_refactorizations"),
            "cholesky_ms_per_step": (d.get("phases_ms_per_occurrence_timed_solve") or {}).get("cholesky_fused_fwd")}


def trace_roofline():
    try:
        d = json.load(open(TRACE_ROOFLINE))
        return d, os.path.relpath(TRACE_ROOFLINE, ROOT)
    except (OSError, ValueError):
        return None, None


def pmc_traffic(kernel_prefixes, exclude=()):
    """HBM bytes of one phase from the committed rocprofv3 PMC passes (scripts/pmc_traffic.py: FETCH_SIZE x2 +
    WRITE_SIZE, gfx950 corrections), summed over the launches the phase consists of (for the assembly: the main
    wave, the split-K tail and the ordered reduce, the same region the HIP events time); None if absent."""
    try:
        doc = json.load(open(PMC_TRAFFIC))
    except (OSError, ValueError):
        return None, None
    total, used = 0.0, []
    for k, v in sorted(doc.get("kernels", {}).items()):
        if any(p in k for p in kernel_prefixes) and not any(k.endswith(x) for x in exclude):
            # (template kernels carry a "void " prefix and "<N>")
            total += v["hbm_bytes_per_launch"]
            used.append(k)
    if not used:
        return None, None
    return total, os.path.relpath(PMC_TRAFFIC, ROOT) + ":" + "+".join(used)


def engine_options(args):
    """--opt name=value (repeatable): cvxg_set_option settings for A/B runs (include/cvxg.h; product defaults otherwise)."""
    out = {}
    for kv in getattr(args, "opt", None) or []:
        k, v = kv.split("=", 1)
        out[k] = int(v)
    return out


def workload_spec(args, rank):
    """The per-rank synthetic instance of the selected workload (seed 20261015 + rank): (spec, n, m, SYRK rows, name)."""
    from cvx_amd import problems as Z
    wl = args.workload
    if wl == "C4":
        nout, k = args.m or 2048, (args.n or 513) - 1
        spec = Z.kl_dual_spec(nout, k, instance=rank)
        n, m = k + 1, k
        syrk_rows = nout  # the B diag(y) B' Hessian: a weighted SYRK over the outcomes; the bound rows are sparse
        workload = (f"C4: KL dual barrier (Dist_KL via Duality), {nout} outcomes, dual dimension {n}, {k} bound rows"
                    f", full barrier Newton iterations")
        return spec, n, m, syrk_rows, workload
    if wl == "C4P":  # the direct KL solve: Dist_KL.objectiveFunction over kl_1's rows and sum(x) = 1 (KKT, p = 1)
        n = args.n or 2048
        spec = Z.kl_primal_spec(n, "kl_1")
        m = spec["A"].shape[0]
        workload = (f"C4P: KL primal barrier (Dist_KL.objectiveFunction, kl_1 rows: {n} positivity + 2 expectation "
                    f"rows, sum(x) = 1), n = {n}, full barrier Newton iterations on the KKT path")
        return spec, n, m, 2, workload
    n = args.n or (1024 if wl in ("C2", "C2PD") else 4096)
    m0 = args.m or (2048 if wl in ("C2", "C2PD") else 8192)
    if wl == "C3B":
        spec = Z.random_qp_bounds(n, m0, instance=rank)
    elif wl == "C3EQ":  # KKTSystem.solve with p equality rows (p + 1 > 9: the wide Schur path)
        spec = Z.random_qp_eq(n, m0, args.p, instance=rank)
    else:
        spec = Z.random_qp(n, m0, instance=rank)
    m = spec["A"].shape[0]
    syrk_rows = m0  # dense rows (the sparse rows' Hessian entries are per-entry sums, not SYRK work)
    workload = (f"{wl}: random dense QP n={n} m={m0}" + (f" plus {m - m0} sparse bound/difference rows"
                                                           if wl == "C3B" else "") +
                (f" with {args.p} equality rows (KKT path)" if wl == "C3EQ" else "") +
                (", primal-dual iterations (PrimalDualSolver: KKT-matrix SYRK + 2x Ruiz + Cholesky + solves + "
                 "residual line search)" if wl.endswith("PD") else
                 ", full barrier Newton iterations (assembly + Ruiz + Cholesky + solves + line search)") +
                " on one MI355X per rank")
    return spec, n, m, syrk_rows, workload


def run_rank(args, engine_cls=None, backend: str = "nccl", device=None):
    """The per-rank body of bench.py (config C5 when WORLD_SIZE > 1): process-group init from the torchrun
    environment, device selection (cuda:LOCAL_RANK), this rank's independent instance on its engine, W untimed and K
    timed steps bracketed by a barrier + device synchronize on both sides, the MAX of the elapsed time over ranks and
    one gather of {stats, x} to rank 0 (cvx_amd/dist.py).  engine_cls / backend / device let the world-size-2 gloo
    test run this same body on the CPU with a stand-in engine.  Returns (result dict, gathered records) on rank 0,
    (None, None) elsewhere."""
    import torch

    from cvx_amd import dist as D
    from cvx_amd.api import SolverParams
    if engine_cls is None:
        from cvx_amd.engine import Engine as engine_cls

    rank, local_rank, world = D.env_rank()
    if world > 1:
        D.init(backend)
    if device is None:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    wl = args.workload
    spec, n, m, syrk_rows, workload = workload_spec(args, rank)
    pars = SolverParams.standardParams()

    p_eq = 0 if spec.get("Aeq") is None else spec["Aeq"].shape[0]
    eng = engine_cls(n, m, p_eq, device=local_rank, **engine_options(args))
    eng.load_problem(spec)
    eng.set_x(spec["x0"])
    state = {"t": 1.0}
    eng.centering_begin(1.0)

    def one_step():
        st = eng.newton_step(pars)
        if st.done:
            if m / state["t"] < pars.tolSolver:  # barrier finished: restart the path from x0
                eng.set_x(spec["x0"])
                state["t"] = 1.0
            else:
                state["t"] *= 10.0
            eng.centering_begin(state["t"])
        return st

    syrk_ms, chol_ms, solve_ms, ruiz_ms, ls_ms = [], [], [], [], []

    def record(ph):
        syrk_ms.append(ph[5])
        ruiz_ms.append(ph[1])
        chol_ms.append(ph[2])
        solve_ms.append(ph[3])
        ls_ms.append(ph[4])

    def pd_solve():  # one whole PrimalDualSolver.solve from x0; returns its KKT solves
        eng.set_x(spec["x0"])
        s_ = eng.pd_solve(pars)
        return s_.newton_steps

    steps = args.steps
    if wl.endswith("PD"):
        pd_solve()  # warm-up solve
    else:
        for _ in range(args.warmup):
            one_step()
    # phase timers: HIP events on the stream of each phase, recorded per step into a ring and read once after the
    # timed region (cvxg_get_phase_times), so the timing never makes a step wait.  The timed region records only the
    # assembly and Cholesky phases (the roofline's kernels): each event record is a marker packet that idles the GPU
    # ~3-4 us (microbench/hostcost.hip); the other phases are timed on a few untimed steps after it.
    eng.set_timing(True, all_phases=wl.endswith("PD"))
    reruns0 = eng.ruiz_lookahead()
    D.barrier(device)
    sync()
    t0 = time.perf_counter()
    if wl.endswith("PD"):  # whole solves until at least `steps` KKT solves were timed
        done = 0
        while done < steps:
            done += pd_solve()
        steps = done
    full_steps = 0  # timed steps whose line search accepted t = 1 (their next evaluation rides the search's sweep)
    for _ in range(0 if wl.endswith("PD") else steps):
        full_steps += int(one_step().step == 1.0)
    sync()
    D.barrier(device)
    elapsed = time.perf_counter() - t0
    elapsed = D.max_over_ranks(elapsed, device)
    ph = eng.phase_times()  # per-step means over the timed steps (the last 63 at most)
    # timed steps whose Ruiz lookahead fell short (their Cholesky phase holds the re-run sweeps + factorization)
    ruiz_reruns = eng.ruiz_lookahead() - reruns0
    x_final, t_final = eng.get_x(), state["t"]  # (the timed steps' iterate: the detail steps below move on from it)
    if not wl.endswith("PD"):  # the other phases, on a few steps after the timed region
        eng.set_timing(True, all_phases=True)
        for _ in range(min(steps, 10)):
            one_step()
        ph_all = eng.phase_times()
        ph = [ph[i] if i in (0, 2, 5) else ph_all[i] for i in range(len(ph))]
    record(ph)
    eng.set_timing(False)
    # (the late-path state is the default C3 instance's: instance 0, n = 4096, m = 8192)
    steady = steady_state(eng, pars, sync) if (wl == "C3" and rank == 0 and (n, m) == (4096, 8192)) else None

    stats = np.array([rank, steps, elapsed, t_final], dtype=np.float64)
    gathered = D.gather_results(x_final, stats, device)
    eng.close()
    if rank != 0:
        return None, None

    total_steps = steps * world
    value = total_steps / elapsed
    syrk = float(np.mean(syrk_ms))
    chol = float(np.mean(chol_ms))
    tf = (lambda fl, ms: fl / (ms * 1e-3) / 1e12 if ms > 0 else None)  # noqa: E731
    flops_syrk = float(syrk_rows) * n * (n + 1)  # lower triangle incl. diagonal
    ach = tf(flops_syrk, syrk)
    kkt_ms = float(np.mean(ruiz_ms)) + chol + float(np.mean(solve_ms))
    flops_chol = n ** 3 / 3.0 + n * n / 2.0 + n / 6.0  # dpotrf flops; all but O(n^2) are trailing SYRK/GEMM
    frac = (lambda a: a / FP64_MFMA_PEAK_TFLOPS if a is not None else None)  # noqa: E731
    chol_traffic, chol_src = (pmc_traffic(("cvxg::k_chol_dataflow",), exclude=("/short",)) if wl == "C3"
                              else (None, None))  # ("/short": attempts voided by an open Ruiz lookahead)
    chol_sq = None
    if wl == "C3":  # MFMA utilisation of the Cholesky from the committed SQ counter passes (scripts/pmc_sq.sh)
        try:
            sq_path = latest_profile("pmc_chol_dataflow_sq.json")
            d = json.load(open(sq_path))["derived"]
            chol_sq = {"source": os.path.relpath(sq_path, ROOT),
                       "mfma_work_over_algorithmic": d["mfma_work_over_algorithmic"],
                       "mfma_busy_vs_clock_limited_peak": d[
                           "mfma_busy_vs_clock_limited_peak (x 0.93, the SYRK main wave's measured fraction)"]}
        except (OSError, ValueError, KeyError):
            chol_sq = None
    trailing = {"kernel": "k_chol_dataflow (trailing SYRK/GEMM updates + 64x64 POTRF/TRSM tasks)",
                "flops_per_launch": flops_chol, "avg_launch_ms": chol, "achieved": tf(flops_chol, chol),
                "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": frac(tf(flops_chol, chol)),
                "traffic": chol_traffic, "traffic_unit": "bytes/factorization (algorithmic: 8 n^2 = 134 MB, the "
                "lower triangle read and written once)", "traffic_source": chol_src, "pmc_sq": chol_sq}
    traffic, traffic_src = (pmc_traffic(("cvxg::k_syrk_direct", "cvxg::k_syrk_reduce")) if wl == "C3"
                            else (None, None))
    assembly = {"kernel": "k_syrk_direct + k_syrk_reduce (H = tP + A'diag(w)A)", "achieved": ach,
                "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": frac(ach), "traffic": traffic,
                "traffic_unit": "bytes/assembly (main wave + split-K tail + reduce)", "traffic_source": traffic_src,
                "flops_per_launch": flops_syrk, "avg_launch_ms": syrk}
    comb_ach = tf(flops_syrk + flops_chol, syrk + chol)
    tr, tr_src = trace_roofline() if wl == "C3" else (None, None)
    # the same fractions recomputed from a COMMITTED rocprofv3 kernel trace of this command (not this run): a
    # cross-check of the event timing, labelled with its source so it is never mistaken for a live measurement
    committed = None if tr is None else {
        "source": tr_src, "note": "kernel-trace durations of a committed profile of `bench.py --steps 20 --warmup 5 "
        "--no-cpu-baseline`, not measured by this run", "combined_frac": tr["combined_frac"],
        "assembly_frac": tr["assembly_frac"], "cholesky_frac": tr["cholesky_frac"]}
    both = (traffic + chol_traffic) if (traffic is not None and chol_traffic is not None) else None
    # "% MFMA roofline on trailing SYRK" = (assembly SYRK + POTRF trailing flops) / (their kernel time)
    roofline = {"bound": "mfma", "kernel": "assembly SYRK + Cholesky (SURVEY.md §8d: the SYRK-type flops of the "
                "assembly and of the POTRF trailing updates over the two phases' kernel time)",
                "achieved": comb_ach, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": frac(comb_ach),
                "frac_definition": "combined: (assembly SYRK + Cholesky) flops / (their HIP-event kernel time) / peak "
                                   "(since round 4; round 1-3 lines carried the assembly SYRK alone, now in "
                                   "roofline.assembly)",
                "committed_trace": committed,
                "traffic": both, "traffic_unit": "bytes/step (assembly + factorization, PMC)",
                "flops_per_launch": flops_syrk + flops_chol, "avg_launch_ms": syrk + chol,
                "assembly": assembly, "trailing": trailing}
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "Newton KKT solves/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded generators of cvx_amd/problems.py, SURVEY.md §8d)",
        "config": {"workload": workload, "n": n, "m": m,
                   "parallelism": f"replicas x{world}: one independent QP per GPU (config C5), "
                                  "RCCL gather of results after the timed region"},
        "roofline": roofline,
        "phases_ms": {"syrk": syrk, "ruiz": float(np.mean(ruiz_ms)), "cholesky_fused_fwd": chol,
                      "bwd_solve_residual": float(np.mean(solve_ms)), "line_search": float(np.mean(ls_ms))},
        "kkt_factor_solve_per_s": 1e3 / kkt_ms if kkt_ms > 0 else None,
        "cholesky_tflops": tf(n ** 3 / 3, chol),
        "ruiz_lookahead_reruns": ruiz_reruns,
        "ls_full_steps": full_steps,
        "steady_state": steady,
        "whole_solve_committed": committed_whole_solve() if wl == "C3" else None,
        "gathered_ranks": len(gathered),
    }
    return out, gathered


def _hist(v):
    """{value: count} of a list of ints, keys as strings (JSON)."""
    out = {}
    for x in v:
        out[str(x)] = out.get(str(x), 0) + 1
    return dict(sorted(out.items(), key=lambda kv: int(kv[0])))


LATE_FIXTURE = os.path.join(ROOT, "tests", "golden", "big", "C3late_n4096_m8192.npz")


def steady_state(eng, pars, sync, t_late=1e11, steps=50, detail=10):
    """The late path, where a full C3 solve spends 96 % of its Newton steps (t = 1e10 .. 1e12, three centerings that
    run to maxIter; bench_c3full): `steps` Newton steps of the centering at t = 1e11 from the engine's own iterate
    entering it (the committed state of tests/golden/big/C3late_n4096_m8192.npz, recorded by scripts/c3_late_states.py),
    wall-clocked like the headline window, then `detail` more with every phase timed.  A side figure: `value` stays the
    t = 1 window.  None when the fixture is absent."""
    try:
        fx = np.load(LATE_FIXTURE)
        k = [i for i in range(fx["t"].shape[0]) if float(fx["t"][i]) == t_late and int(fx["it_n"][i]) == 0][0]
        x = np.array(fx["x"][k])
    except (OSError, IndexError, KeyError):
        return None
    eng.set_x(x)
    eng.centering_begin(t_late)
    eng.newton_step(pars)  # (the first step: its assembly is not prefetched)
    sync()
    t0 = time.perf_counter()
    reg = 0
    for _ in range(steps):
        st = eng.newton_step(pars)
        reg += st.regularized
    sync()
    el = time.perf_counter() - t0
    eng.set_timing(True, all_phases=True)
    for _ in range(detail):
        reg += eng.newton_step(pars).regularized
    ms, cnt = eng.phase_stats()
    eng.set_timing(False)
    return {"t": t_late, "steps": steps, "steps_per_s": steps / el, "ms_per_step": el / steps * 1e3,
            "regularized_steps": reg, "x_source": os.path.relpath(LATE_FIXTURE, ROOT) + f" (state {k})",
            "phases_ms": {"syrk": float(ms[5]), "ruiz": float(ms[1]), "cholesky_fused_fwd": float(ms[2]),
                          "bwd_solve_residual": float(ms[3]), "line_search": float(ms[4])},
            "note": "late-path window (t = 1e11 centering, which runs to maxIter in a full solve); value is the t = 1 "
                    "window"}


def run_full_solve(args):
    """--workload C3FULL ("steady state over a full barrier solve"): one complete C3 barrier solve from
    x0 with the reference's standard parameters (SolverParams.scala:35-46: maxIter 1000 per centering), the t-loop of
    BarrierSolver.scala:70-117 (t = 1, t *= 10 per centering until m / t < tolSolver) driven step by step through
    cvxg_newton_step.  Solve 1 (timers off) gives Newton steps/s over the whole path; solve 2 (every phase timed, the
    ring read every 50 steps) gives the per-phase means over the path.  Both report the Ruiz sweep histogram, the
    regularized refactorizations, the fallbacks and the steps per centering.  One GPU, one instance."""
    import torch

    from cvx_amd.api import SolverParams
    from cvx_amd.engine import Engine
    torch.cuda.set_device(0)
    n, m = args.n or 4096, args.m or 8192
    from cvx_amd import problems as Z
    spec = Z.random_qp(n, m, instance=0)
    pars = SolverParams.standardParams()
    eng = Engine(n, m, 0, device=0, **engine_options(args))
    eng.load_problem(spec)

    def solve(timed):
        eng.set_x(spec["x0"])
        t, steps, per_center, hist = 1.0, 0, [], {}
        reg = fb = full = 0
        small_piv = []  # regularized steps: the row block where the first attempt stopped (0: it ran to the end)
        ph_sum, ph_cnt = np.zeros(8), np.zeros(8)  # per phase: summed ms over its occurrences, occurrences
        if timed:
            eng.set_timing(True, all_phases=True)
        c0 = eng.counters()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while True:  # BarrierSolver.scala:70-117: center at t, gap = m / t, stop below tolSolver, else t *= mu
            eng.centering_begin(t)
            k = 0
            while True:  # every call computes one Newton direction (a KKT solve); done ends the centering
                st = eng.newton_step(pars)
                k += 1
                steps += 1
                hist[st.ruiz_sweeps] = hist.get(st.ruiz_sweeps, 0) + 1
                reg += st.regularized
                if st.regularized:
                    small_piv.append(int(st.small_pivot))
                fb += int(st.fallback != 0)
                full += int(st.took_step == 1 and st.step == 1.0)
                if timed and steps % 50 == 0:  # the timer ring holds 63 steps: read and restart it
                    ms, cnt = eng.phase_stats()
                    ph_sum += ms * cnt
                    ph_cnt += cnt
                    eng.set_timing(True, all_phases=True)
                if st.done:
                    break
            per_center.append(k)
            if m / t < pars.tolSolver or len(per_center) >= 100:
                break
            t *= 10.0
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        c1 = eng.counters()
        if timed:
            ms, cnt = eng.phase_stats()
            ph_sum += ms * cnt
            ph_cnt += cnt
            eng.set_timing(False)
        # per step: a phase's total time over the solve / the steps (the inline assembly runs on few steps); per
        # occurrence: its mean duration when it runs
        return dict(elapsed=el, steps=steps, per_center=per_center, hist=hist, reg=reg, fb=fb, full=full,
                    phases=(ph_sum / max(steps, 1)).tolist(),
                    phases_occ=(ph_sum / np.maximum(ph_cnt, 1)).tolist(), occ=ph_cnt.tolist(), x=eng.get_x(),
                    small_piv=small_piv, counters={k: c1[k] - c0[k] for k in c1})

    a = solve(False)
    b = solve(True)
    eng.close()
    same = bool(np.array_equal(a["x"], b["x"]))
    ph, po = b["phases"], b["phases_occ"]
    out = {"metric": METRIC, "value": a["steps"] / a["elapsed"], "unit": "Newton KKT solves/s", "n_gpus": 1,
           "steps": a["steps"], "warmup": 0, "ms_per_step": a["elapsed"] / a["steps"] * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (seeded generators of cvx_amd/problems.py, SURVEY.md §8d)",
           "config": {"workload": f"C3FULL: one complete barrier solve of the C3 random dense QP n={n} m={m} from x0, "
                                  "standard parameters (maxIter 1000 per centering), t-loop to m/t < 1e-8",
                      "n": n, "m": m},
           "solve_s": a["elapsed"], "centerings": len(a["per_center"]), "steps_per_centering": a["per_center"],
           "ruiz_sweep_histogram": {str(k): v for k, v in sorted(a["hist"].items())},
           "regularized_refactorizations": a["reg"], "fallbacks": a["fb"], "line_search_full_steps": a["full"],
           "phases_ms_per_step_timed_solve": {"assembly_prefetched": ph[5], "assembly_inline": ph[0], "ruiz": ph[1],
                                              "cholesky_fused_fwd": ph[2], "bwd_solve_residual": ph[3],
                                              "line_search": ph[4]},
           "phases_ms_per_occurrence_timed_solve": {"assembly_prefetched": po[5], "assembly_inline": po[0],
                                                    "ruiz": po[1], "cholesky_fused_fwd": po[2],
                                                    "bwd_solve_residual": po[3], "line_search": po[4]},
           "phase_occurrences_timed_solve": {"assembly_prefetched": b["occ"][5], "assembly_inline": b["occ"][0],
                                             "cholesky_fused_fwd": b["occ"][2]},
           "first_attempt_stop_rows": _hist(a["small_piv"]),
           "factorization_counters": a["counters"],
           "timed_solve_s": b["elapsed"], "timed_solve_same_x": same}
    return out


def run_shared_gpu(args):
    """--workload C3X2 (side workload, not the headline): `--instances` independent C3 problems (seeds 20261015 + i)
    on ONE GPU, each with its own context and stream, each driven by its own host thread through cvxg_newton_step
    (the t-loop of BarrierSolver.scala:70-117 per instance); aggregate Newton steps/s over K steps per instance
    against one instance alone on the same box.  Shows how much of the Cholesky chain's idle workers and the
    host/launch gaps a second independent instance reclaims (config C5's independence, one GPU).  Also times the
    lockstep form, cvxg_batch_newton_step (one call advances every instance by one step).
    --workload C2X (round 6): the same with C2 instances (n = 1024, m = 2048), the form SURVEY.md §8d prescribes for the
    smaller configuration -- one C2 step leaves most of the chip idle -- with the combined roofline fraction of the
    aggregate rate beside it."""
    import threading

    import torch

    from cvx_amd import problems as Z
    from cvx_amd.api import SolverParams
    from cvx_amd.engine import Engine, batch_newton_step
    torch.cuda.set_device(0)
    c2 = args.workload == "C2X"
    n, m, k = args.n or (1024 if c2 else 4096), args.m or (2048 if c2 else 8192), max(2, args.instances)
    pars = SolverParams.standardParams()
    specs = [Z.random_qp(n, m, instance=i) for i in range(k)]
    engs = []
    for spec in specs:
        e = Engine(n, m, 0, device=0, **engine_options(args))
        e.load_problem(spec)
        engs.append(e)
    ts = [1.0] * k

    def begin(i):
        engs[i].set_x(specs[i]["x0"])
        ts[i] = 1.0
        engs[i].centering_begin(1.0)

    def step(i, st=None):
        st = st if st is not None else engs[i].newton_step(pars)
        if st.done:
            if m / ts[i] < pars.tolSolver:
                begin(i)
            else:
                ts[i] *= 10.0
                engs[i].centering_begin(ts[i])

    def run(i, steps):
        for _ in range(steps):
            step(i)

    for i in range(k):
        begin(i)
        run(i, args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()  # one instance alone
    run(0, args.steps)
    torch.cuda.synchronize()
    one = args.steps / (time.perf_counter() - t0)
    th = [threading.Thread(target=run, args=(i, args.steps)) for i in range(k)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()  # all instances, one host thread each
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    agg = k * args.steps / el
    torch.cuda.synchronize()
    t0 = time.perf_counter()  # lockstep: cvxg_batch_newton_step
    for _ in range(args.steps):
        infos, st = batch_newton_step(engs, pars)
        assert st == [0] * k, st
        for i in range(k):
            step(i, infos[i])
    torch.cuda.synchronize()
    lock = k * args.steps / (time.perf_counter() - t0)
    for e in engs:
        e.close()
    # SURVEY §8d's combined roofline: the assembly SYRK's and the factorization's flops per step at the aggregate rate
    flop = m * n * (n + 1) + n ** 3 / 3 + n ** 2 / 2 + n / 6
    roof = {"bound": "mfma", "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "flop_per_step": flop,
            "achieved_threaded": flop * agg / 1e12, "frac_threaded": flop * agg / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "achieved_lockstep": flop * lock / 1e12, "frac_lockstep": flop * lock / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "achieved_one": flop * one / 1e12, "frac_one": flop * one / 1e12 / FP64_MFMA_PEAK_TFLOPS}
    name = "C2X" if c2 else "C3X2"
    return {"metric": METRIC, "value": agg, "unit": "Newton KKT solves/s", "n_gpus": 1, "steps": args.steps * k,
            "warmup": args.warmup, "ms_per_step": el / (k * args.steps) * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded generators of cvx_amd/problems.py, SURVEY.md §8d)",
            "config": {"workload": f"{name}: {k} independent random dense QPs n={n} m={m} sharing one MI355X, one "
                                   "context + stream + host thread each, full barrier Newton iterations",
                       "n": n, "m": m, "instances": k},
            "one_instance_steps_per_s": one, "aggregate_over_one": agg / one,
            "lockstep_batch_steps_per_s": lock, "roofline": roof}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="C3",
                    choices=["C2", "C3", "C3B", "C3EQ", "C4", "C4P", "C2PD", "C3PD", "C3FULL", "C3X2", "C2X"],
                    help="C3 (default, the metric's config): random dense QP n=4096 m=8192; C2: n=1024 m=2048; "
                         "C3B: C3 plus 9216 sparse bound / difference rows; C4: KL dual, 2048 outcomes, k=512; "
                         "C2PD / C3PD: the primal-dual solver (solverType PD) on C2 / C3, steps = its KKT solves; "
                         "C3EQ: C3 with --p equality rows (KKT path); C4P: the direct KL solve, n = 2048; "
                         "C3FULL: one complete C3 barrier solve with standard parameters (steady state over the path); "
                         "C3X2: --instances independent C3 problems sharing one GPU (aggregate steps/s); "
                         "C2X: the same with C2 problems")
    ap.add_argument("--instances", type=int, default=2, help="instances of C3X2")
    ap.add_argument("--p", type=int, default=64, help="equality rows of C3EQ")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=30.0)
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option name=value (cvxg_set_option, e.g. ruiz_loop=1); A/B runs only")
    args = ap.parse_args()

    from cvx_amd import dist as D
    rank, _, world = D.env_rank()
    if args.workload == "C3FULL":
        print(json.dumps(run_full_solve(args)), flush=True)
        return
    if args.workload in ("C3X2", "C2X"):
        print(json.dumps(run_shared_gpu(args)), flush=True)
        return
    out, _ = run_rank(args)
    if rank == 0:
        if not args.no_cpu_baseline and world == 1 and args.workload == "C3":
            spec = workload_spec(args, 0)[0]
            out["cpu_baseline"] = cpu_baseline(spec, args.cpu_budget)
            out["cpu_baseline_blas"] = cpu_baseline_blas(spec)
        elif not args.no_cpu_baseline:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
