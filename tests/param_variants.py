"""The MPCParameters variants the parity tests run (``src/control/mpc_controller.py:17-30``).

Shared by ``test_gpu_params.py`` (GPU against the exact oracle), ``golden/gen_qp_forms.py`` (the
reference's own QP captured per variant) and ``test_qp_forms.py``.  ``variant`` works on any
dataclass with the reference's fields (the reference's, the product's or the oracle's), so the
same variant is applied to each side of a comparison.
"""
from __future__ import annotations

from dataclasses import replace

import numpy as np

VARIANTS = ["q_nondiag", "r_offdiag", "dt_0.05", "dt_0.2", "wheelbase_14px", "tight_bounds", "slack_x10",
            "slack_div10", "relaxed_du"]


def resolution(name: str) -> float:
    """map_resolution the variant's base parameters are made at (0.2 -> wheelbase 14 px)."""
    return 0.2 if name == "wheelbase_14px" else 0.8


def relaxed(p):
    """The retry parameters of ``control_stage.py:50-56`` (du_bounds widened by (5, 0.05))."""
    return replace(p, du_bounds=((p.du_bounds[0][0] - 5.0, p.du_bounds[0][1] + 5.0),
                                 (p.du_bounds[1][0] - 0.05, p.du_bounds[1][1] + 0.05)))


def variant(p, name: str):
    """Apply variant ``name`` to base parameters ``p`` (made at ``resolution(name)``)."""
    if name == "q_nondiag":  # symmetric: cvxpy's quad_form takes only symmetric matrices
        q = np.array(p.q, float)
        q[0, 1] = q[1, 0] = 1.5
        q[2, 3] = q[3, 2] = 0.1
        q[0, 2] = q[2, 0] = 0.3
        qn = np.array(p.q_terminal, float)
        qn[0, 1] = qn[1, 0] = 3.0
        qn[1, 3] = qn[3, 1] = 0.15
        assert np.linalg.eigvalsh(q).min() > 0 and np.linalg.eigvalsh(qn).min() > 0
        return replace(p, q=q, q_terminal=qn)
    if name == "r_offdiag":
        return replace(p, r=np.array([[0.03, 0.02], [0.02, 0.25]]))
    if name == "dt_0.05":
        return replace(p, dt=0.05)
    if name == "dt_0.2":
        return replace(p, dt=0.2)
    if name == "wheelbase_14px":
        return p
    if name == "tight_bounds":
        return replace(p, u_bounds=((-5.0, 4.0), (-0.3, 0.25)), v_bounds=(2.0, 18.0),
                       du_bounds=((-3.0, 2.5), (-0.05, 0.04)))
    if name == "slack_x10":
        return replace(p, slack_velocity=1e4, slack_input=5e3, slack_rate=5e3)
    if name == "slack_div10":
        return replace(p, slack_velocity=1e2, slack_input=50.0, slack_rate=50.0)
    if name == "relaxed_du":
        return relaxed(p)
    raise KeyError(name)
