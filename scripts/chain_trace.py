"""Run one C3 Newton direction with the dataflow-Cholesky task trace on (CVXG_DF_TRACE) and print the
per-type task durations (scripts/df_trace.py) and the critical-chain stamps (scripts/chain_stamps.py).
  python scripts/chain_trace.py [n m] [out]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
m = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", "df_trace.bin")
os.environ["CVXG_DF_TRACE"] = out

from cvx_amd import problems as Z  # noqa: E402
from cvx_amd.api import SolverParams  # noqa: E402
from cvx_amd.engine import Engine  # noqa: E402

spec = Z.random_qp(n, m, instance=0)
eng = Engine(n, m, 0)
eng.load_problem(spec)
pars = SolverParams.standardParams()
for _ in range(3):
    eng.newton_direction(pars, 1.0, spec["x0"])
eng.close()
import chain_stamps  # noqa: E402
import df_trace  # noqa: E402
df_trace.main(out)
chain_stamps.main(out)
