"""Reversible-jump MH chains on the coal-mining change-point model (config C3).

Mirror of examples/coal/coal.jl: the model (:47-62) with k ~ poisson(3)
change points, min_uniform_continuous positions (:18-33), gamma(1, 1/200)
rates and a piecewise Poisson process over the event times
(poisson_process.jl:9-67); `mcmc_step` (:329-336) applies rate_move,
position_move (when k > 0) and birth_death_move, each an involutive MH step
(src/inference/mh.jl:85-98); `simple_mcmc_step` (:338-345) replaces the
birth/death move by mh(trace, select(:k)), the Dynamic DSL regenerate of k.
One device thread per chain.
"""
from __future__ import annotations

from ctypes import POINTER, byref, c_double, c_int32, c_void_p

import numpy as np

from . import _lib
from .pf import Context, default_context

STATE_W = 68
K_MAX = 32


class CoalChains:
    """`n_chains` chains resident in HBM (gh_coal_create/step/read_state):
    run() continues them without moving their state over PCIe; `state` is
    read back on demand."""

    def __init__(self, events, n_chains: int, seed: int = 0, chain0: int = 0, ctx: Context | None = None,
                 kernel: str = "mcmc_step"):
        """kernel: "mcmc_step" (coal.jl:329-336) or "simple_mcmc_step" (:338-345)."""
        self.ctx = ctx or default_context()
        self.events = np.ascontiguousarray(np.sort(np.asarray(events, dtype=np.float64)))
        self.n_chains, self.seed, self.chain0 = int(n_chains), int(seed), int(chain0)
        self.accepts = np.zeros((self.n_chains, 3), dtype=np.int32)
        self.iterations = 0
        self.kernel_ms = 0.0
        self._state = None
        self.h = c_void_p()
        _lib.check(_lib.load().gh_coal_create(self.ctx.h, self.chain0, self.n_chains, _lib.dptr(self.events),
                                              self.events.size, self.seed, byref(self.h)))
        if kernel not in ("mcmc_step", "simple_mcmc_step"):
            raise _lib.GenHipError(1, f"unknown coal kernel {kernel!r}")
        _lib.check(_lib.load().gh_coal_set_kernel(self.h, 1 if kernel == "simple_mcmc_step" else 0))

    def run(self, n_iters: int, k_history: bool = False, accepts: bool = True):
        """n_iters mcmc_steps (the first call draws the start from the prior
        first).  `accepts=False` skips the per-call acceptance download."""
        kh = np.zeros((self.n_chains, max(n_iters, 1)), dtype=np.int32) if k_history else None
        acc = np.zeros((self.n_chains, 3), dtype=np.int32) if accepts else None
        ms = c_double()
        _lib.check(_lib.load().gh_coal_step(
            self.h, n_iters, None if acc is None else acc.ctypes.data_as(POINTER(c_int32)),
            None if kh is None else kh.ctypes.data_as(POINTER(c_int32)), byref(ms)))
        if acc is not None:
            self.accepts += acc
        self.iterations += n_iters
        self.kernel_ms = ms.value
        self._state = None
        return kh

    @property
    def state(self) -> np.ndarray:
        if self._state is None:
            st = np.zeros((self.n_chains, STATE_W))
            _lib.check(_lib.load().gh_coal_read_state(self.h, _lib.dptr(st)))
            self._state = st
        return self._state

    def load_state(self, state, iterations: int = 0):
        """Resume from [n_chains][68] rows (gh_coal_write_state); the next run
        continues at iteration `iterations` + 1."""
        st = np.ascontiguousarray(np.asarray(state, dtype=np.float64).reshape(self.n_chains, STATE_W))
        _lib.check(_lib.load().gh_coal_write_state(self.h, _lib.dptr(st), int(iterations)))
        self.iterations = int(iterations)
        self._state = None

    def close(self):
        if self.h:
            _lib.load().gh_coal_destroy(self.h)
            self.h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def k(self):
        return self.state[:, 0].astype(int)

    @property
    def score(self):
        return self.state[:, 1]

    def changepoints(self, c: int):
        return self.state[c, 2 : 2 + self.k[c]]

    def rates(self, c: int):
        return self.state[c, 2 + K_MAX : 2 + K_MAX + self.k[c] + 1]
