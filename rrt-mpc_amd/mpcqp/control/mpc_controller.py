"""Linear time-varying MPC on MI355X: drop-in for ``src/control/mpc_controller.py``.

``MPCParameters`` and ``MPCController.solve`` keep the reference's names,
arguments, return values and failure behaviour (``mpc_controller.py:17-145``);
the QP that the reference assembles in cvxpy and hands to OSQP
(``:53-132``) is built and solved by the HIP kernels of ``libmpcqp.so``
(``csrc/mpcqp.hip``: K1 ``k_build`` = unwrap + linearize, K2 ``k_solve`` =
condense + OSQP-algorithm ADMM + polish).  ``BatchedMPCController`` is the
batched entry point that thousands of candidate trajectories go through at once.
"""
from __future__ import annotations

import ctypes
import logging
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import NamedTuple, Optional, Tuple

import numpy as np

from .. import _lib

LOG = logging.getLogger(__name__)

FloatArray = np.ndarray


@dataclass
class MPCParameters:
    """Same fields and defaults as ``src/control/mpc_controller.py:17-30``."""

    wheelbase_px: float
    dt: float
    horizon: int
    q: FloatArray
    r: FloatArray
    q_terminal: FloatArray
    u_bounds: Tuple[Tuple[float, float], Tuple[float, float]]
    v_bounds: Tuple[float, float]
    du_bounds: Tuple[Tuple[float, float], Tuple[float, float]]
    slack_velocity: float = 1e3
    slack_input: float = 5e2
    slack_rate: float = 5e2


class BatchSolution(NamedTuple):
    """Device tensors of one ``solve_batch`` call (views into controller-owned buffers,
    valid until the next call on the same controller)."""

    u0: "object"  # (B, 2)      float64
    X: "object"  # (B, 4, N+1)  float64
    U: "object"  # (B, 2, N)    float64
    status: "object"  # (B,)    int32   (1 solved, 2 solved_inaccurate, -2 max_iter, -10 numerical)
    iters: "object"  # (B, 4)   int32   {ADMM its, polish its, KKT factorizations, line-search trials}
    active: "object"  # (B, 5N+1) uint8 {0 inactive, 1 lower, 2 upper} per soft row


def _arr_key(a) -> bytes:
    if type(a) is np.ndarray and a.dtype == np.float64 and a.flags.c_contiguous:
        return a.tobytes()
    return np.asarray(a, float).tobytes()


_NUM = (float, int, np.floating, np.integer)


def _tuple_key(a) -> tuple:
    """Value key of a bounds field: a flat tuple of floats whatever the container (a tuple of tuples
    of numbers takes the fast path; lists, arrays and tuples holding them are converted), so equal
    bounds share one workspace and an unhashable leaf never reaches the cache."""
    if type(a) is tuple:
        if all(type(r) is tuple and all(isinstance(v, _NUM) for v in r) for r in a):
            return tuple(float(v) for r in a for v in r)
        if all(isinstance(v, _NUM) for v in a):
            return tuple(float(v) for v in a)
    return tuple(np.asarray(a, float).ravel().tolist())


def _params_key(params, method: int, settings: dict) -> tuple:
    """Value key of a parameter block + solver settings (the B=1 controller cache; computed once per
    drop-in solve, so it avoids array conversions where the fields already are float64 arrays /
    tuples, as MPCConfig.to_parameters and dataclasses.replace produce them)."""
    return (
        params.horizon,
        params.wheelbase_px,
        params.dt,
        _arr_key(params.q),
        _arr_key(params.r),
        _arr_key(params.q_terminal),
        _tuple_key(params.u_bounds),
        _tuple_key(params.v_bounds),
        _tuple_key(params.du_bounds),
        getattr(params, "slack_velocity", 1e3),
        getattr(params, "slack_input", 5e2),
        getattr(params, "slack_rate", 5e2),
        int(method),
        tuple(sorted(settings.items())),
    )


class BatchedMPCController:
    """Solve B independent MPC QPs per call on one GPU.

    ``solve_batch(x0[B,4], ref[B,N+1,4], u_prev[B,2])`` runs K1 + K2 asynchronously on
    the current torch stream (or ``stream``).  Inputs may be numpy arrays (copied to the
    device) or float64 device tensors (used in place).

    ``pairing`` ("auto", "on", "off"): two QPs per wave for horizons N <= 15 (``mpcqp_set_pairing``;
    the same results bit for bit).  "auto" pairs a launch with more QPs than the GPU has wave slots.
    """

    def __init__(self, params, max_batch: int, *, device=None, method: str = "admm", pairing: str = "auto",
                 **settings) -> None:
        import torch

        if method not in ("admm", "newton"):
            raise ValueError("method must be 'admm' or 'newton'")
        if not torch.cuda.is_available():
            raise _lib.LibraryError("BatchedMPCController needs a ROCm GPU; there is no CPU fallback")
        self._torch = torch
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.params = params
        self.method = _lib.METHOD_ADMM if method == "admm" else _lib.METHOD_NEWTON
        self.settings = dict(settings)
        self.horizon = int(params.horizon)
        self.max_batch = int(max_batch)
        L = _lib.lib()
        self._L = L
        self._cparams = _lib.to_c_params(params, self.method, **self.settings)
        ws = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.mpcqp_create(ctypes.byref(self._cparams), self.max_batch, self.device.index, ctypes.byref(ws)),
                       "mpcqp_create")
        self._ws = ws
        self.set_pairing(pairing)
        N, B = self.horizon, self.max_batch
        kw = dict(device=self.device)
        self._u0 = torch.empty((B, 2), dtype=torch.float64, **kw)
        self._X = torch.empty((B, 4, N + 1), dtype=torch.float64, **kw)
        self._U = torch.empty((B, 2, N), dtype=torch.float64, **kw)
        self._status = torch.empty((B,), dtype=torch.int32, **kw)
        self._iters = torch.empty((B, 4), dtype=torch.int32, **kw)
        self._active = torch.empty((B, 5 * N + 1), dtype=torch.uint8, **kw)

    # ------------------------------------------------------------------
    def set_params(self, params) -> None:
        """Swap the parameter block (same horizon); stream-ordered."""
        self._cparams = _lib.to_c_params(params, self.method, **self.settings)
        _lib.check(self._L.mpcqp_set_params(self._ws, ctypes.byref(self._cparams)), "mpcqp_set_params")
        self.params = params

    def set_pairing(self, mode: str) -> None:
        """Two QPs per wave for N <= 15: "auto" (default), "on" or "off" (mpcqp_set_pairing)."""
        if mode not in _lib.PAIRING_MODES:
            raise ValueError(f"pairing must be one of {sorted(_lib.PAIRING_MODES)}")
        _lib.check(self._L.mpcqp_set_pairing(self._ws, _lib.PAIRING_MODES[mode]), "mpcqp_set_pairing")
        self.pairing = mode

    def _device_input(self, a, shape, name):
        torch = self._torch
        if isinstance(a, torch.Tensor):
            t = a
            if t.device != self.device or t.dtype != torch.float64:
                t = t.to(device=self.device, dtype=torch.float64)
        else:
            t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(self.device, non_blocking=False)
        t = t.contiguous()
        if tuple(t.shape) != tuple(shape):
            t = t.reshape(shape)
        return t

    def solve_batch(self, x0, ref, u_prev=None, *, stream=None) -> BatchSolution:
        torch = self._torch
        N = self.horizon
        B = int(x0.shape[0])
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch {self.max_batch}")
        x0_t = self._device_input(x0, (B, 4), "x0")
        if len(ref.shape) == 3 and ref.shape[1] > N + 1:  # rows past N are never read (see solve)
            ref = ref[:, : N + 1]
        ref_t = self._device_input(ref, (B, N + 1, 4), "ref")
        up_t = None if u_prev is None else self._device_input(u_prev, (B, 2), "u_prev")
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        s = ctypes.c_void_p(stream.cuda_stream)
        self._keep = (x0_t, ref_t, up_t)  # keep inputs alive until the kernels have consumed them
        _lib.check(self._L.mpcqp_build(self._ws, B, x0_t.data_ptr(), ref_t.data_ptr(),
                                       None if up_t is None else up_t.data_ptr(), s), "mpcqp_build")
        _lib.check(self._L.mpcqp_solve(self._ws, B, self._u0.data_ptr(), self._X.data_ptr(), self._U.data_ptr(),
                                       self._status.data_ptr(), self._iters.data_ptr(), self._active.data_ptr(), s),
                   "mpcqp_solve")
        return BatchSolution(self._u0[:B], self._X[:B], self._U[:B], self._status[:B], self._iters[:B],
                             self._active[:B])

    def solve_one(self, x0, ref, u_prev=None):
        """One QP for the sequential closed loop of ``TrajectoryTracker.track``, where host overhead
        dominates a B=1 step.  The workspace's own blocks of pinned, device-mapped host memory hold
        the inputs and outputs, which the kernels read and write in place (``mpcqp_stage`` /
        ``mpcqp_solve_served``, include/mpcqp.h): the inputs are written into the block, then ONE
        library call hands the QP to the workspace's resident solver wave (started by the first
        call, gone after 2 ms idle) and waits for its answer -- no kernel launch per step.
        ``x0`` (4,), ``ref`` (>= N+1, 4) -- rows 0..N are used --, ``u_prev`` (2,) host arrays.
        Returns host numpy ``(status, u0, X, U)``; X (4, N+1) and U (2, N) are fresh arrays.
        A fault that surfaces at the synchronisation raises ``_lib.DeviceError``."""
        io = self._one
        if io is None:
            io = self._one = self._stage()
        io["x0"][:] = x0
        io["ref"][:] = ref[: self.horizon + 1]
        if u_prev is None:
            io["up"][:] = 0.0
        else:
            io["up"][:] = u_prev
        rc = self._solve1(self._ws)
        if rc != 0:
            msg = self._L.mpcqp_last_error().decode(errors="replace")
            if rc == _lib.E_DEVICE:
                raise _lib.DeviceError(f"B=1 solve: {msg}")
            raise _lib.LibraryError(f"B=1 solve failed ({rc}): {msg}")
        return int(io["status"][0]), io["u0"].copy(), io["X"].copy(), io["U"].copy()

    _one = None

    def _stage(self) -> dict:
        """numpy views of the workspace's B=1 staging blocks (allocated by the first mpcqp_stage;
        an allocation failure raises DeviceError)."""
        N = self.horizon
        # the resident B=1 server (mpcqp_solve_served: no launch per call) unless MPCQP_B1_SERVER=0
        # asks for a launch per call (mpcqp_solve_staged)
        self._solve1 = (self._L.mpcqp_solve_staged if os.environ.get("MPCQP_B1_SERVER", "1") == "0"
                        else self._L.mpcqp_solve_served)
        hin, hout = ctypes.c_void_p(), ctypes.c_void_p()
        offs = (ctypes.c_int32 * 6)()
        with self._torch.cuda.device(self.device):
            rc = self._L.mpcqp_stage(self._ws, ctypes.byref(hin), ctypes.byref(hout), offs)
        if rc != 0:
            raise _lib.DeviceError(f"mpcqp_stage failed ({rc}): {self._L.mpcqp_last_error().decode(errors='replace')}")
        nin = 4 + 4 * (N + 1) + 2
        nout = offs[5] + 5 * N + 1
        fin = np.frombuffer((ctypes.c_double * nin).from_address(hin.value), np.float64)
        fout = np.frombuffer((ctypes.c_uint8 * nout).from_address(hout.value), np.uint8)
        return dict(
            x0=fin[0:4], ref=fin[4:4 + 4 * (N + 1)].reshape(N + 1, 4), up=fin[4 + 4 * (N + 1):],
            u0=fout[offs[0]:offs[0] + 16].view(np.float64),
            X=fout[offs[1]:offs[1] + 32 * (N + 1)].view(np.float64).reshape(4, N + 1),
            U=fout[offs[2]:offs[2] + 16 * N].view(np.float64).reshape(2, N),
            status=fout[offs[3]:offs[3] + 4].view(np.int32),
            iters=fout[offs[4]:offs[4] + 16].view(np.int32),
            active=fout[offs[5]:offs[5] + 5 * N + 1],
        )

    @property
    def closed(self) -> bool:
        return getattr(self, "_ws", None) is None or not self._ws.value

    def close(self) -> None:
        # the staging blocks belong to the workspace: mpcqp_destroy syncs its stream and frees them
        self._one = None
        if getattr(self, "_ws", None) is not None and self._ws.value:
            self._L.mpcqp_destroy(self._ws)
            self._ws = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


_CACHE: "OrderedDict[tuple, BatchedMPCController]" = OrderedDict()
_CACHE_SIZE = 8


def latency_settings(horizon: int) -> dict:
    """Polish schedule of the latency-bound B=1 drop-in (the reference's sequential loop, one QP
    per call).  The library default (`polish_from` 75 with near-tolerance attempts) is tuned for a
    batch, whose time is its slowest QP; one QP's own cost is lower with an attempt at every
    termination check.  Measured on one vehicle's closed loop with the default single Ruiz pass
    (profiles/r03_s14_schedule_single.json): `polish_from` 25 is the fastest schedule
    at N = 10, 15, 20 and 30.  The horizons past the one-wave kernel keep the default (unmeasured).
    Every schedule ends at the exact optimum; the counters match the C restatement under each
    (tests/test_gpu_parity.py)."""
    return {"polish_from": 25} if horizon <= 32 else {}


# OSQP's default Ruiz pass count (this build's default is 1: DESIGN.md §5)
OSQP_SCALING = 10


def _unpolished_fallback(ctrl: BatchedMPCController) -> bool:
    """The drop-in re-solves a QP its polish did not finish under OSQP's 10 Ruiz passes: with a
    polished exact optimum the scaling only changes the work, never the result; without one the
    returned ADMM iterate depends on it.  Method newton has no ADMM iterate."""
    c = ctrl._cparams
    return c.scaling != OSQP_SCALING and c.method == _lib.METHOD_ADMM


def _single_controller(params, method: str = "admm", **settings) -> BatchedMPCController:
    settings = {**latency_settings(int(params.horizon)), **settings}  # the caller's settings win
    key = _params_key(params, 0 if method == "admm" else 1, settings)
    ctrl = _CACHE.get(key)
    if ctrl is not None and ctrl.closed:
        ctrl = None
    if ctrl is None:
        ctrl = BatchedMPCController(params, 1, method=method, **settings)
        _CACHE[key] = ctrl
        while len(_CACHE) > _CACHE_SIZE:
            _CACHE.popitem(last=False)[1].close()
    else:
        _CACHE.move_to_end(key)
    return ctrl


class MPCController:
    """Quadratic-cost MPC controller with soft bounds and rate limits (``mpc_controller.py:33-145``)."""

    def __init__(self, params: MPCParameters, **settings) -> None:
        # ``settings``: optional solver settings of ``mpcqp_params`` (rho, max_iter, polish, ...);
        # the reference's constructor takes ``params`` alone and so does every caller of it.
        self._params = params
        self._settings = dict(settings)

    def solve(
        self,
        x0: FloatArray,
        ref_traj: FloatArray,
        *,
        u_init: Optional[FloatArray] = None,
        u_prev: Optional[FloatArray] = None,
    ) -> Tuple[Optional[FloatArray], Optional[FloatArray], Optional[FloatArray]]:
        # u_init is accepted and ignored, as in the reference (mpc_controller.py:50-51).
        N = int(self._params.horizon)
        x0 = np.asarray(x0, dtype=float)
        ref = np.asarray(ref_traj, dtype=float)
        # The reference reads rows 0..N of ref_traj (mpc_controller.py:68,111) after unwrapping
        # the whole yaw column (:59-60); np.unwrap is a prefix operation, so the first N+1 rows
        # unwrap identically on their own.  Fewer rows fail there (ref[N]) and here.
        if ref.ndim != 2 or ref.shape[1] != 4 or ref.shape[0] < N + 1:
            raise ValueError(f"ref_traj must have shape (>= {N + 1}, 4), got {ref.shape}")
        if x0.size != 4:
            raise ValueError(f"x0 must have 4 entries, got shape {x0.shape}")
        x0 = x0.reshape(4)
        up = None if u_prev is None else np.asarray(u_prev, dtype=float).reshape(2)
        # A missing library or device, or a failed allocation, fails loudly here (no CPU fallback
        # exists) ...
        settings = self._settings
        if "scaling" not in settings and not settings.get("polish", 1):
            # no polish: the result is the ADMM iterate, which depends on the scaling -> OSQP's own
            settings = {**settings, "scaling": OSQP_SCALING}
        ctrl = _single_controller(self._params, **settings)
        try:
            status, _, X, U = ctrl.solve_one(x0, ref, up)
        except _lib.LibraryError:
            # ... while a refused or failed launch of the solve maps to (None, None, None), as the
            # reference maps cp.SolverError (mpc_controller.py:133-135).  A fault that surfaces at
            # the stream sync is a DeviceError and propagates.
            LOG.exception("GPU failed during MPC solve")
            return None, None, None
        if status != _lib.SOLVED and _unpolished_fallback(ctrl):
            # Not the polished exact optimum (the solution then no longer depends on the scaling):
            # solve again under OSQP's own 10 Ruiz passes, so the returned unpolished iterate and
            # status are those of the reference's OSQP settings (mpc_controller.py:119-132).  (The
            # converse -- one pass polishes a QP that ten passes would leave unpolished -- returns
            # the exact optimum; it needs a max_iter far below the reference's 60000.)
            ctrl = _single_controller(self._params, **{**settings, "scaling": OSQP_SCALING})
            try:
                status, _, X, U = ctrl.solve_one(x0, ref, up)
            except _lib.LibraryError:
                LOG.exception("GPU failed during MPC solve")
                return None, None, None
        if status == _lib.NUMERICAL_ERROR:
            LOG.error("MPC solve failed with a numerical error")
            return None, None, None
        if status not in (_lib.SOLVED, _lib.SOLVED_INACCURATE):
            LOG.warning("MPC solve returned status %s", _lib.STATUS_NAMES.get(status, status))
            return None, None, None
        return U[:, 0].copy(), X, U

    @property
    def params(self) -> MPCParameters:
        return self._params


__all__ = ["MPCParameters", "MPCController", "BatchedMPCController", "BatchSolution", "latency_settings"]
