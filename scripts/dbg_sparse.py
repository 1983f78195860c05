import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from cvx_amd import problems as Z
from cvx_amd.api import SolverParams
from cvx_amd.engine import Engine
from oracle import cvx_oracle as O
spec = Z.random_qp_bounds(24, 16, instance=6)
pars = SolverParams.standardParams()
m = spec["A"].shape[0]
eng = Engine(24, m, 0); eng.load_problem(spec); eng.set_x(spec["x0"])
pb = O.Problem(a0=spec["a0"], r0=spec["r0"], P=spec["P"], A=spec["A"], r=spec["r"], ub=spec["ub"])
ref = O.barrier_solve(pb, spec["x0"], pars, record=True)
t = 1.0; k = 0
while m / t >= pars.tolSolver / 10 and k < 400:
    eng.centering_begin(t)
    while True:
        st = eng.newton_step(pars)
        if st.done and not st.took_step: break
        r = ref.records[k] if k < len(ref.records) else None
        if t >= 1e9: print(f"t={t:g} it={st.iter} step={st.step} kc={st.backtracks_c} ka={st.backtracks_armijo} fresh={st.ls_fresh} "
              f"nd={st.newton_decrement:.3e} ng={st.norm_grad:.3e} | ref step={getattr(r,'step',None)} kc={getattr(r,'backtracks_c',None)} ka={getattr(r,'backtracks_armijo',None)} nd={getattr(r,'newton_decrement',0):.3e}")
        k += 1
        if st.done or k > 400 or st.iter > 40: break
    t *= 10
