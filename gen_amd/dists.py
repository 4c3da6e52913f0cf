"""Gen's distribution library over libgen_hip.so (gh_dist_logpdf / gh_dist_random).

Mirrors src/modeling_library/distributions/: each distribution object has
`logpdf(x, *args)` and `random(*args)` (modeling_library.jl:15-41) and is
callable as `dist(*args)` (a draw).  Both are batched on the GPU: x holds n
values (component-major [dim, n] for the vector distributions) and every
argument is either one value shared by the batch or one value per element
(arrays of length n along the first axis).  `random(*args, n=..., seed=...)`
draws n values; value i depends on (seed, i) only.  Categorical values are
1-based, bernoulli values are 0/1, as in Gen.
"""
from __future__ import annotations

import ctypes
from ctypes import byref

import numpy as np

from . import _lib


class DistDesc(ctypes.Structure):
    _fields_ = [("dist", ctypes.c_int32), ("dim", ctypes.c_int32), ("n_params", ctypes.c_int32),
                ("param_stride", ctypes.c_int32), ("params_on_device", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("params", ctypes.POINTER(ctypes.c_double))]


class Distribution:
    """One distribution of the library; `argn` = Gen's argument names."""

    def __init__(self, name: str, code: int, argn: tuple, vector_args: tuple = (), dim_of=None):
        self.name, self.code, self.argn = name, code, argn
        self.vector_args = vector_args  # arguments that are vectors (probs, bounds, mu/std of the vector dists)
        self.dim_of = dim_of  # value dimension from the arguments (vector distributions)

    def __repr__(self):
        return f"gen_amd.{self.name}"

    # parameter rows ---------------------------------------------------------
    def _rows(self, args, n):
        """(flat rows, n_params, per_value, dim)."""
        if len(args) != len(self.argn):
            raise _lib.GenHipError(1, f"{self.name} takes {len(self.argn)} arguments {self.argn}")
        dim = self.dim_of(args) if self.dim_of else 1
        if self.name == "mvnormal":  # one (mu, cov) for the batch; the engine factors cov once
            mu, cov = (np.asarray(a, dtype=np.float64) for a in args)
            if mu.ndim != 1 or cov.shape != (mu.size, mu.size):
                raise _lib.GenHipError(1, "mvnormal: mu [d] and cov [d, d] shared by the batch")
            return np.concatenate([mu, cov.ravel()]), mu.size + mu.size**2, False, dim
        parts, per_value = [], False
        for a, name in zip(args, self.argn):
            v = np.asarray(a, dtype=np.float64)
            vec = name in self.vector_args
            if (v.ndim == 2 and vec) or (v.ndim == 1 and not vec):
                per_value = True
        for a, name in zip(args, self.argn):
            v = np.asarray(a, dtype=np.float64)
            vec = name in self.vector_args
            if per_value:
                if v.ndim == (2 if vec else 1):
                    if v.shape[0] != n:
                        raise _lib.GenHipError(1, f"{self.name}: argument {name} has {v.shape[0]} rows, n = {n}")
                    parts.append(v.reshape(n, -1))
                else:
                    parts.append(np.broadcast_to(v.reshape(1, -1), (n, max(v.size, 1))))
            else:
                parts.append(v.reshape(1, -1))
        rows = np.ascontiguousarray(np.concatenate(parts, axis=1))
        return rows, rows.shape[1], per_value, dim

    def _desc(self, rows, np_, per_value, dim):
        return DistDesc(self.code, dim, np_, np_ if per_value else 0, 0, 0, _lib.dptr(rows))

    # the GFI of a distribution ------------------------------------------------
    def logpdf(self, x, *args, ctx=None) -> np.ndarray | float:
        """logpdf(dist, x, args...) of every value in x."""
        from .pf import default_context

        ctx = ctx or default_context()
        xv = np.asarray(x, dtype=np.float64)
        scalar = xv.ndim == 0 or (self.dim_of is not None and xv.ndim == 1)
        probe_dim = self.dim_of(args) if self.dim_of else 1
        if probe_dim > 1:
            xv = xv.reshape(probe_dim, -1)
        else:
            xv = xv.reshape(-1)
        n = xv.shape[-1]
        rows, np_, per_value, dim = self._rows(args, n)
        xv = np.ascontiguousarray(xv)
        out = np.empty(n)
        d = self._desc(rows, np_, per_value, dim)
        _lib.check(_lib.load().gh_dist_logpdf(ctx.h, byref(d), n, _lib.dptr(xv), _lib.dptr(out)))
        return float(out[0]) if scalar else out

    def random(self, *args, n: int | None = None, seed: int | None = None, ctx=None):
        """n draws (one draw, as a scalar / vector, when n is None).  Without a
        seed every call draws fresh randomness, as Gen's random(dist, args...)
        does from Julia's global RNG (the seeds come from a host generator,
        reseedable with gen_amd.dists.seed); an explicit seed gives a
        reproducible batch: draw i is a function of (seed, i) alone."""
        from .pf import default_context

        ctx = ctx or default_context()
        if seed is None:
            seed = _fresh_seed()
        nn = 1 if n is None else int(n)
        rows, np_, per_value, dim = self._rows(args, nn)
        out = np.empty((dim, nn)) if dim > 1 else np.empty(nn)
        d = self._desc(rows, np_, per_value, dim)
        _lib.check(_lib.load().gh_dist_random(ctx.h, byref(d), nn, int(seed), _lib.dptr(out)))
        if n is None:
            return out[:, 0].copy() if dim > 1 else float(out[0])
        return out

    def __call__(self, *args, seed: int | None = None):
        return self.random(*args, seed=seed)


_seed_rng = np.random.default_rng()


def seed(s: int | None) -> None:
    """Reseed the host generator behind unseeded draws (Random.seed! for
    random(dist, args...) calls without a seed); None: fresh OS entropy."""
    global _seed_rng
    _seed_rng = np.random.default_rng(s)


def _fresh_seed() -> int:
    return int(_seed_rng.integers(0, 1 << 63))


def _vdim(args):
    return int(np.asarray(args[0]).shape[-1]) if np.asarray(args[0]).ndim else 1


normal = Distribution("normal", 1, ("mu", "std"))
broadcasted_normal = Distribution("broadcasted_normal", 2, ("mu", "std"), ("mu", "std"), _vdim)
mvnormal = Distribution("mvnormal", 3, ("mu", "cov"), ("mu", "cov"), _vdim)
uniform_continuous = Distribution("uniform_continuous", 4, ("low", "high"))
uniform = uniform_continuous
uniform_discrete = Distribution("uniform_discrete", 5, ("low", "high"))
bernoulli = Distribution("bernoulli", 6, ("prob",))
categorical = Distribution("categorical", 7, ("probs",), ("probs",))
gamma = Distribution("gamma", 8, ("shape", "scale"))
inv_gamma = Distribution("inv_gamma", 9, ("shape", "scale"))
beta = Distribution("beta", 10, ("alpha", "beta"))
exponential = Distribution("exponential", 11, ("rate",))
poisson = Distribution("poisson", 12, ("lambda",))
binom = Distribution("binom", 13, ("n", "p"))
neg_binom = Distribution("neg_binom", 14, ("r", "p"))
geometric = Distribution("geometric", 15, ("p",))
laplace = Distribution("laplace", 16, ("loc", "scale"))
cauchy = Distribution("cauchy", 17, ("x0", "gamma"))
piecewise_uniform = Distribution("piecewise_uniform", 18, ("bounds", "probs"), ("bounds", "probs"))
beta_uniform = Distribution("beta_uniform", 19, ("theta", "alpha", "beta"))

ALL = [normal, broadcasted_normal, mvnormal, uniform_continuous, uniform_discrete, bernoulli, categorical, gamma,
       inv_gamma, beta, exponential, poisson, binom, neg_binom, geometric, laplace, cauchy, piecewise_uniform,
       beta_uniform]


def logpdf(dist: Distribution, x, *args, ctx=None):
    """Gen.logpdf(dist, x, args...)"""
    return dist.logpdf(x, *args, ctx=ctx)


def random(dist: Distribution, *args, n: int | None = None, seed: int | None = None, ctx=None):
    """Gen.random(dist, args...)"""
    return dist.random(*args, n=n, seed=seed, ctx=ctx)
