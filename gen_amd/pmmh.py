"""Particle-marginal Metropolis–Hastings (config C5) on the device.

Mirror of examples/pmmh/example.jl:20-79: the model draws log var_x and
log var_y from normal(0, 2) and scores the observations with a
ParticleFilterCombinator (examples/pmmh/pf.jl:14-73), whose weight is an
inner particle filter's log-ML estimate; `do_inference` applies, per
iteration, mh(tr, select(:var_x)), mh(tr, select(:var_y)) and the two
random-walk moves with sd sqrt(0.5) (src/inference/mh.jl:14-62).  Every chain
is one workgroup; its threads are the inner particles.
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, byref, c_double, c_int32

import numpy as np

from . import _lib
from .pf import Context, default_context


class PMMHChains:
    """State of n_chains outer chains (this rank's share when distributed)."""

    def __init__(self, ys, n_chains: int, n_inner: int = 256, seed: int = 0, chain0: int = 0,
                 ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.ys = np.ascontiguousarray(np.asarray(ys, dtype=np.float64))
        self.n_chains, self.n_inner, self.seed, self.chain0 = int(n_chains), int(n_inner), int(seed), int(chain0)
        self.lvx = np.zeros(self.n_chains)
        self.lvy = np.zeros(self.n_chains)
        self.lml = np.zeros(self.n_chains)
        self.accepts = np.zeros((self.n_chains, 4), dtype=np.int32)
        self.iterations = 0
        self.started = False
        self.kernel_ms = 0.0

    def run(self, n_iters: int, history: bool = False):
        """Run n_iters iterations (4 MH moves each); the first call also draws
        the start from the prior (generate(model, (), observations))."""
        hist = np.zeros((self.n_chains, max(n_iters, 1), 2)) if history else None
        acc = np.zeros((self.n_chains, 4), dtype=np.int32)
        ms = c_double()
        # the move counters continue across calls (iter0)
        _lib.check(_lib.load().gh_pmmh_run(
            self.ctx.h, self.chain0, self.n_chains, self.n_inner, _lib.dptr(self.ys), self.ys.size,
            n_iters, self.iterations, self.seed, 0 if self.started else 1, _lib.dptr(self.lvx), _lib.dptr(self.lvy),
            _lib.dptr(self.lml), acc.ctypes.data_as(POINTER(c_int32)), _lib.dptr(hist), byref(ms)))
        self.accepts += acc
        self.started = True
        self.iterations += n_iters
        self.kernel_ms = ms.value
        return hist

    @property
    def var_x(self):
        return np.exp(self.lvx)

    @property
    def var_y(self):
        return np.exp(self.lvy)


def pmmh(ys, n_chains: int, n_iters: int, n_inner: int = 256, seed: int = 0, ctx: Context | None = None,
         history: bool = False):
    """Run PMMH from the prior for n_iters iterations; returns the chains."""
    ch = PMMHChains(ys, n_chains, n_inner, seed, ctx=ctx)
    hist = ch.run(n_iters, history)
    return ch, hist
