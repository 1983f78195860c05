"""CPU checks of the host-side mirror's control logic (cvx_amd/api.py) that need no device: termination criteria,
the feasibility report and the InfeasibleProblemException branch of withFeasiblePoint."""
import numpy as np
import pytest


def test_termination_criteria():
    """CvxUtils.scala:61-87."""
    from cvx_amd.api import CvxUtils, OptimizationState, SolverParams
    pars = SolverParams.standardParams()
    std = CvxUtils.standardTerminationCriterion(pars)
    ph1 = CvxUtils.phase_I_TerminationCriterion()
    assert std(OptimizationState(None, None, 1e-9, None, 5.0))
    assert not std(OptimizationState(None, None, 1e-9, 1e-7, 5.0))
    assert not std(OptimizationState(None, None, 1e-7, 0.0, 5.0))
    assert ph1(OptimizationState(None, None, 1.0, None, -1e-3))
    assert not ph1(OptimizationState(None, None, 1.0, 1e-5, -1e-3))
    assert not ph1(OptimizationState(None, None, 1.0, 0.0, 0.0))
    with pytest.raises(AssertionError):  # "Nonempty duality gap required"
        std(OptimizationState(None, None, None, None, 0.0))


def test_with_feasible_point_raises_infeasible_problem_exception(monkeypatch):
    """ConstraintSet.withFeasiblePoint (ConstraintSet.scala:556-575): a phase-I report that is not feasible at
    pars.tolSolver (FeasibilityReport.isFeasible: max(s) < tol and the equality error < tol) raises
    InfeasibleProblemException carrying the report; a feasible one adds the point."""
    from cvx_amd import api
    pars = api.SolverParams.standardParams()
    cs = api.ConstraintSet(2, api.Constraints.allCoordinatesPositive(2), np.ones(2))
    monkeypatch.setattr(api.ConstraintSet, "phase_I_Analysis",
                        lambda self, eqs, p: api.FeasibilityReport(np.array([-1.0, 0.5]), [0.25], False, self, 0.0))
    with pytest.raises(api.InfeasibleProblemException) as ei:
        cs.withFeasiblePoint(None, pars)
    assert ei.value.report.s[0] == 0.25
    assert [c.id for c in ei.value.report.violatedConstraints(pars.tolSolver)] == ["x_0>0"]
    monkeypatch.setattr(api.ConstraintSet, "phase_I_Analysis",
                        lambda self, eqs, p: api.FeasibilityReport(np.array([0.5, 0.5]), [-0.1], True, self, 0.0))
    fp = cs.withFeasiblePoint(None, pars).feasiblePoint
    assert np.array_equal(fp, [0.5, 0.5])
