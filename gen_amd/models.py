"""Model families: hand-lowered Static-DSL models the engine runs on the GPU.

Each class stands for one Gen generative function (a Static-DSL model whose
time steps are an `Unfold` of a static kernel) and knows
  * its packed parameter layout for gh_model_create (include/gen_hip.h), and
  * its address scheme: which choice-map address holds the observation and
    the latent of time step t, so Gen-style choice maps map onto gh_obs.

Address schemes follow the reference programs they mirror:
  LinearGaussianSSM  :chain => t => :x / :y   (SURVEY.md §8(d) C2 Static-DSL spec)
  DiscreteHMM        :z_init, :x_init, :chain => t-1 => :z / :x
                     (test/inference/particle_filter.jl:66-78)
  KitagawaSSM        :chain => t => :x / :y   (examples/pmmh/model.jl:40-50)
"""
from __future__ import annotations

import numpy as np

from . import _lib


class Model:
    family: int
    d: int = 1
    dy: int = 1
    k: int = 0
    v: int = 0
    latent_name = "x"
    obs_name = "y"

    def params(self) -> np.ndarray:
        raise NotImplementedError

    def obs_address(self, t: int):
        return ("chain", t, self.obs_name)

    def latent_address(self, t: int):
        return ("chain", t, self.latent_name)

    def obs_values(self, value) -> np.ndarray:
        return np.ascontiguousarray(np.atleast_1d(np.asarray(value, dtype=np.float64)).ravel())

    def desc(self) -> tuple[_lib.ModelDesc, np.ndarray]:
        p = np.ascontiguousarray(self.params(), dtype=np.float64)
        d = _lib.ModelDesc(self.family, self.d, self.dy, self.k, self.v, _lib.dptr(p), p.size)
        return d, p


class LinearGaussianSSM(Model):
    """x_1 ~ mvnormal(mu0, P0); x_t ~ mvnormal(A x_{t-1} + b, Q); y_t ~ mvnormal(H x_t + c, R).

    The Static-DSL kernel it lowers (mvnormal: src/modeling_library/distributions/mvnormal.jl:12-33):
        @gen (static) function lg_kernel(t::Int, x_prev, p)
            x = @trace(mvnormal(p.A * x_prev + p.b, p.Q), :x)
            @trace(mvnormal(p.H * x + p.c, p.R), :y)
            return x
        end
    """

    family = _lib.FAMILY_LGSSM

    def __init__(self, A, Q, H, R, mu0, P0, b=None, c=None):
        self.A = np.atleast_2d(np.asarray(A, dtype=np.float64))
        self.d = self.A.shape[0]
        self.H = np.atleast_2d(np.asarray(H, dtype=np.float64))
        self.dy = self.H.shape[0]
        self.Q = np.atleast_2d(np.asarray(Q, dtype=np.float64))
        self.R = np.atleast_2d(np.asarray(R, dtype=np.float64))
        self.mu0 = np.atleast_1d(np.asarray(mu0, dtype=np.float64))
        self.P0 = np.atleast_2d(np.asarray(P0, dtype=np.float64))
        self.b = np.zeros(self.d) if b is None else np.atleast_1d(np.asarray(b, dtype=np.float64))
        self.c = np.zeros(self.dy) if c is None else np.atleast_1d(np.asarray(c, dtype=np.float64))
        shapes = {
            "A": (self.A, (self.d, self.d)),
            "Q": (self.Q, (self.d, self.d)),
            "H": (self.H, (self.dy, self.d)),
            "R": (self.R, (self.dy, self.dy)),
            "P0": (self.P0, (self.d, self.d)),
        }
        for name, (m, s) in shapes.items():
            if m.shape != s:
                raise ValueError(f"{name} has shape {m.shape}, expected {s}")

    def params(self):
        return np.concatenate(
            [self.A.ravel(), self.b, self.Q.ravel(), self.H.ravel(), self.c, self.R.ravel(), self.mu0, self.P0.ravel()]
        )

    def simulate(self, T: int, rng: np.random.Generator):
        """Draw (xs, ys) from the model (numpy RNG; synthetic data only)."""
        xs = np.zeros((T, self.d))
        ys = np.zeros((T, self.dy))
        x = rng.multivariate_normal(self.mu0, self.P0)
        for t in range(T):
            if t > 0:
                x = rng.multivariate_normal(self.A @ x + self.b, self.Q)
            xs[t] = x
            ys[t] = rng.multivariate_normal(self.H @ x + self.c, self.R)
        return xs, ys

    @staticmethod
    def benchmark(d: int = 10, seed: int = 1) -> "LinearGaussianSSM":
        """The C2 synthetic model of SURVEY.md §8(d): A = 0.9 I + 0.01 G rescaled to
        spectral radius 0.95, Q = 0.1 I, H = I, R = 0.5 I, x_1 ~ N(0, I)."""
        rng = np.random.default_rng(seed)
        A = 0.9 * np.eye(d) + 0.01 * rng.standard_normal((d, d))
        A *= 0.95 / max(abs(np.linalg.eigvals(A)))
        return LinearGaussianSSM(A, 0.1 * np.eye(d), np.eye(d), 0.5 * np.eye(d), np.zeros(d), np.eye(d))


class DiscreteHMM(Model):
    """Categorical HMM of test/inference/particle_filter.jl:50-78.

    `transition[:, prev]` is p(z_t | z_{t-1} = prev) and `emission[:, z]` is
    p(x | z), exactly the reference's `transition_dists` / `emission_dists`
    (0-based states and symbols here, 1-based in Julia).
    """

    family = _lib.FAMILY_HMM
    latent_name = "z"
    obs_name = "x"

    def __init__(self, prior, transition, emission):
        self.prior = np.asarray(prior, dtype=np.float64)
        self.T = np.asarray(transition, dtype=np.float64)
        self.E = np.asarray(emission, dtype=np.float64)
        self.k = self.prior.size
        self.v = self.E.shape[0]
        if self.T.shape != (self.k, self.k) or self.E.shape[1] != self.k:
            raise ValueError("transition must be k x k and emission v x k")

    def params(self):
        return np.concatenate([self.prior, self.T.ravel(), self.E.ravel()])

    def obs_address(self, t: int):
        return ("x_init",) if t == 1 else ("chain", t - 1, "x")

    def latent_address(self, t: int):
        return ("z_init",) if t == 1 else ("chain", t - 1, "z")


class KitagawaSSM(Model):
    """Nonlinear SSM of examples/pmmh/model.jl:9-13,40-46:
    x_1 ~ normal(mu1, s1); x_t ~ normal(x/2 + 25 x/(1+x^2) + 8 cos(1.2 t), sqrt(var_x));
    y_t ~ normal(x_t^2 / 20, sqrt(var_y))."""

    family = _lib.FAMILY_KITAGAWA

    def __init__(self, var_x: float = 10.0, var_y: float = 1.0, mu1: float = 0.0, s1: float = 5.0):
        self.var_x, self.var_y, self.mu1, self.s1 = float(var_x), float(var_y), float(mu1), float(s1)

    def params(self):
        return np.array([self.mu1, self.s1, self.var_x, self.var_y])

    def simulate(self, T: int, rng: np.random.Generator):
        xs = np.zeros(T)
        ys = np.zeros(T)
        x = rng.normal(self.mu1, self.s1)
        for t in range(1, T + 1):
            if t > 1:
                x = rng.normal(x / 2 + 25 * x / (1 + x * x) + 8 * np.cos(1.2 * t), np.sqrt(self.var_x))
            xs[t - 1] = x
            ys[t - 1] = rng.normal(x * x / 20.0, np.sqrt(self.var_y))
        return xs, ys
