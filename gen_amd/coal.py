"""Reversible-jump MH chains on the coal-mining change-point model (config C3).

Mirror of examples/coal/coal.jl: the model (:47-62) with k ~ poisson(3)
change points, min_uniform_continuous positions (:18-33), gamma(1, 1/200)
rates and a piecewise Poisson process over the event times
(poisson_process.jl:9-67); `mcmc_step` (:329-336) applies rate_move,
position_move (when k > 0) and birth_death_move, each an involutive MH step
(src/inference/mh.jl:85-98).  One device thread per chain.
"""
from __future__ import annotations

from ctypes import POINTER, byref, c_double, c_int32

import numpy as np

from . import _lib
from .pf import Context, default_context

STATE_W = 68
K_MAX = 32


class CoalChains:
    def __init__(self, events, n_chains: int, seed: int = 0, chain0: int = 0, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.events = np.ascontiguousarray(np.sort(np.asarray(events, dtype=np.float64)))
        self.n_chains, self.seed, self.chain0 = int(n_chains), int(seed), int(chain0)
        self.state = np.zeros((self.n_chains, STATE_W))
        self.accepts = np.zeros((self.n_chains, 3), dtype=np.int32)
        self.iterations = 0
        self.started = False
        self.kernel_ms = 0.0

    def run(self, n_iters: int, k_history: bool = False):
        kh = np.zeros((self.n_chains, max(n_iters, 1)), dtype=np.int32) if k_history else None
        acc = np.zeros((self.n_chains, 3), dtype=np.int32)
        ms = c_double()
        _lib.check(_lib.load().gh_coal_run(
            self.ctx.h, self.chain0, self.n_chains, _lib.dptr(self.events), self.events.size, n_iters,
            self.iterations, self.seed, 0 if self.started else 1, _lib.dptr(self.state),
            acc.ctypes.data_as(POINTER(c_int32)), None if kh is None else kh.ctypes.data_as(POINTER(c_int32)),
            byref(ms)))
        self.accepts += acc
        self.iterations += n_iters
        self.started = True
        self.kernel_ms = ms.value
        return kh

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
