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
  BayesianLinearRegression  :slope, :intercept, "y-$i"   (examples/regression/quickstart.jl:3-9)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def _mvn_logpdf(x, mean, cov) -> float:
    L = np.linalg.cholesky(cov)
    z = np.linalg.solve(L, np.asarray(x, dtype=np.float64) - mean)
    return float(-0.5 * (x.size * np.log(2 * np.pi) + 2.0 * np.log(np.diag(L)).sum() + z @ z))


def _normal_logpdf(x, mu, std) -> float:
    """normal.jl:56-60"""
    var = std * std
    return float(-((x - mu) ** 2) / (2.0 * var) - 0.5 * np.log(2.0 * np.pi * var))


class Model:
    family: int
    d: int = 1
    dy: int = 1
    k: int = 0
    v: int = 0
    latent_name = "x"
    obs_name = "y"
    static = False  # True: no Unfold (generate only, model_args are the data)

    def params(self) -> np.ndarray:
        raise NotImplementedError

    def obs_address(self, t: int):
        return ("chain", t, self.obs_name)

    def latent_address(self, t: int):
        return ("chain", t, self.latent_name)

    def obs_from_choicemap(self, cm, t: int):
        """The observation of step t in a choice map (None if absent).  Any
        other constrained address would update or delete an existing choice,
        which the PF step forbids (particle_filter.jl:168-170)."""
        addr = self.obs_address(t)
        for a, _ in cm:
            if a != addr:
                raise _lib.GenHipError(
                    2, f"constraint at {a}: only {addr} may be constrained in step {t} (discard must be empty)"
                )
        return cm.get(addr)

    def latent_value(self, x):
        """A latent state row as its choice value (get_choices)."""
        return float(x[0]) if x.size == 1 else x.copy()

    def latent_column(self, col):
        """Latent rows [n, d] as the choice values of n traces (trace[addr])."""
        return col[:, 0] if col.shape[1] == 1 else col

    # a step's latent addresses (one here; a switching slot model has two) and
    # each one's value from the state row / rows
    def latent_addresses(self, t: int) -> list:
        return [self.latent_address(t)]

    def latent_part(self, k: int, x):
        return self.latent_value(x)

    def latent_part_column(self, k: int, col):
        return self.latent_column(col)

    def obs_values(self, value) -> np.ndarray:
        return np.ascontiguousarray(np.atleast_1d(np.asarray(value, dtype=np.float64)).ravel())

    def gh_obs(self, value):
        """(gh_obs of one step's observation, what must stay alive while it is used)."""
        arr = self.obs_values(value)
        return _lib.Obs(_lib.dptr(arr), arr.size, 1, 0, 0, None), arr

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

    def kalman_log_marginal(self, ys) -> float:
        """Exact log p(y_1..T) by the Kalman filter (host, numpy): the value
        Gen's CPU particle filter estimates for this model (the analytic
        reference of the C2 log-ML error)."""
        mu, P = self.mu0.copy(), self.P0.copy()
        ll = 0.0
        for t, y in enumerate(np.atleast_2d(ys)):
            if t > 0:
                mu = self.A @ mu + self.b
                P = self.A @ P @ self.A.T + self.Q
            S = self.H @ P @ self.H.T + self.R
            r = y - (self.H @ mu + self.c)
            ll += -0.5 * (len(y) * np.log(2 * np.pi) + np.linalg.slogdet(S)[1] + r @ np.linalg.solve(S, r))
            K = P @ self.H.T @ np.linalg.inv(S)
            mu = mu + K @ r
            P = P - K @ self.H @ P
        return float(ll)

    def log_joint(self, xs, ys) -> float:
        """Score of a trace (Gen's `get_score`): log p(x_1..T, y_1..T) of one
        latent trajectory xs [T, d] and its observations (None = absent), the
        sum of the mvnormal logpdfs (mvnormal.jl:12-16) of every choice."""
        xs = np.atleast_2d(np.asarray(xs, dtype=np.float64))
        total = 0.0
        for t, x in enumerate(xs):
            mean, cov = (self.mu0, self.P0) if t == 0 else (self.A @ xs[t - 1] + self.b, self.Q)
            total += _mvn_logpdf(x, mean, cov)
            if ys is not None and ys[t] is not None:
                total += _mvn_logpdf(np.atleast_1d(ys[t]), self.H @ x + self.c, self.R)
        return float(total)

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

    def log_joint(self, zs, xs) -> float:
        """Score of a trace: log p(z_1..T, x_1..T) (categorical.jl:10-12)."""
        total = 0.0
        for t, z in enumerate(np.asarray(zs).ravel().astype(int)):
            total += np.log(self.prior[z] if t == 0 else self.T[z, prev])
            if xs is not None and xs[t] is not None:
                total += np.log(self.E[int(np.asarray(xs[t]).ravel()[0]), z])
            prev = z
        return float(total)

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

    def log_joint(self, xs, ys) -> float:
        """Score of a trace: log p(x_1..T, y_1..T) (normal.jl:56-60 per choice)."""
        xs = np.asarray(xs, dtype=np.float64).ravel()
        total = 0.0
        for t in range(1, xs.size + 1):
            x = xs[t - 1]
            if t == 1:
                total += _normal_logpdf(x, self.mu1, self.s1)
            else:
                v = xs[t - 2]
                total += _normal_logpdf(x, v / 2 + 25 * v / (1 + v * v) + 8 * np.cos(1.2 * t), np.sqrt(self.var_x))
            if ys is not None and ys[t - 1] is not None:
                total += _normal_logpdf(float(np.asarray(ys[t - 1]).ravel()[0]), x * x / 20.0, np.sqrt(self.var_y))
        return float(total)

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


class BayesianLinearRegression(Model):
    """examples/regression/quickstart.jl:3-9 (config C1), a static model:
        slope = @trace(normal(mu_s, sd_s), :slope)
        intercept = @trace(normal(mu_i, sd_i), :intercept)
        @trace(normal(slope * x_i + intercept, sigma), "y-$i")   for i = 1..n
    State (d = 2) = (slope, intercept); at most 32 data points per model."""

    family = _lib.FAMILY_REGRESSION
    d = 2
    static = True

    def __init__(self, xs, prior_slope=(0.0, 2.0), prior_intercept=(0.0, 10.0), sigma: float = 1.0):
        self.xs = np.ascontiguousarray(np.asarray(xs, dtype=np.float64).ravel())
        self.dy = self.xs.size
        if not 1 <= self.dy <= 32:
            raise ValueError("1..32 data points")
        self.mu_s, self.sd_s = map(float, prior_slope)
        self.mu_i, self.sd_i = map(float, prior_intercept)
        self.sigma = float(sigma)

    def params(self):
        return np.concatenate([[self.mu_s, self.sd_s, self.mu_i, self.sd_i, self.sigma], self.xs])

    def obs_address(self, t: int = 1):
        return None  # several addresses: "y-1" .. "y-n"

    def y_address(self, i: int):
        return (f"y-{i}",)

    def obs_from_choicemap(self, cm, t: int):
        ys = np.full(self.dy, np.nan)
        seen = 0
        for a, v in cm:
            name = a[0] if len(a) == 1 and isinstance(a[0], str) else None
            i = int(name[2:]) if name and name.startswith("y-") and name[2:].isdigit() else 0
            if not 1 <= i <= self.dy:
                raise _lib.GenHipError(2, f"constraint at {a}: the model observes \"y-1\" .. \"y-{self.dy}\" only")
            ys[i - 1] = float(v)
            seen += 1
        if seen == 0:
            return None
        if seen != self.dy:
            raise _lib.GenHipError(1, "constrain every y-i (partial observations are not lowered)")
        return ys

    def log_joint(self, x, ys) -> float:
        """Score of a trace: log p(slope, intercept, y_1..n)."""
        slope, intercept = np.asarray(x, dtype=np.float64).ravel()[:2]
        total = _normal_logpdf(slope, self.mu_s, self.sd_s) + _normal_logpdf(intercept, self.mu_i, self.sd_i)
        if ys is not None:
            for xi, yi in zip(self.xs, np.asarray(ys, dtype=np.float64).ravel()):
                total += _normal_logpdf(yi, slope * xi + intercept, self.sigma)
        return float(total)

    def constraints(self, ys):
        return {self.y_address(i + 1): float(y) for i, y in enumerate(ys)}

    def log_marginal(self, ys) -> float:
        """Exact log p(ys): y ~ N(X m0, X S0 X' + sigma^2 I), X = [x 1]."""
        X = np.stack([self.xs, np.ones_like(self.xs)], axis=1)
        m0 = np.array([self.mu_s, self.mu_i])
        S0 = np.diag([self.sd_s**2, self.sd_i**2])
        C = X @ S0 @ X.T + self.sigma**2 * np.eye(self.dy)
        r = np.asarray(ys, dtype=np.float64) - X @ m0
        _, logdet = np.linalg.slogdet(C)
        return float(-0.5 * (r @ np.linalg.solve(C, r) + logdet + self.dy * np.log(2 * np.pi)))

    def posterior(self, ys):
        """Exact posterior mean and covariance of (slope, intercept)."""
        X = np.stack([self.xs, np.ones_like(self.xs)], axis=1)
        P0 = np.diag([1 / self.sd_s**2, 1 / self.sd_i**2])
        P = P0 + X.T @ X / self.sigma**2
        S = np.linalg.inv(P)
        mean = S @ (P0 @ np.array([self.mu_s, self.mu_i]) + X.T @ np.asarray(ys) / self.sigma**2)
        return mean, S

    @staticmethod
    def quickstart() -> tuple["BayesianLinearRegression", np.ndarray]:
        """The model and literal data of quickstart.jl:26-27."""
        xs = np.arange(1.0, 11.0)
        ys = np.array([8.23, 5.87, 3.99, 2.59, 0.23, -0.66, -3.53, -6.91, -7.24, -9.90])
        return BayesianLinearRegression(xs), ys


# slot distributions / mean forms of GH_FAMILY_SLOTS (include/gen_hip.h)
_SLOT_DIST = {"mvnormal": 1, "normal": 2, "poisson": 3, "bernoulli": 4, "categorical": 5}
_LINK = {"affine": 0, "x^2/20": 1, "exp": 2, "logistic": 3, "softmax": 4, "logscale": 5}
# library slots (slot distribution 6): any scalar distribution of Gen's library by
# its gh_dists.h id, each argument link(h.x + c)
_LIB = {"normal": (1, 2), "uniform": (4, 2), "uniform_discrete": (5, 2), "bernoulli": (6, 1), "gamma": (8, 2),
        "inv_gamma": (9, 2), "beta": (10, 2), "exponential": (11, 1), "poisson": (12, 1), "binom": (13, 2),
        "neg_binom": (14, 2), "geometric": (15, 1), "laplace": (16, 2), "cauchy": (17, 2), "beta_uniform": (19, 3)}
_ARG_LINK = {"identity": 0, "exp": 2, "logistic": 3}


class SlotSSM(Model):
    """A Static-DSL Unfold kernel given by its address slots (GH_FAMILY_SLOTS,
    gen_amd/csrc/gh_slots.h): the kernels the four hand-lowered families do not
    cover drop in without new device code.  One latent address and 1..4 observed
    addresses per step, any subset of which a step constrains
    (static_ir/generate.jl:24-43; choice_map.jl:163-225):

        @gen (static) function kernel(t::Int, x_prev, p)
            x = @trace(mvnormal(p.A * x_prev + p.b, p.Q), :x)       # latent "affine"
            # or: x = @trace(normal(x_prev/2 + 25x_prev/(1+x_prev^2) + 8cos(1.2t), p.sd_x), :x)
            @trace(mvnormal(p.H * x + p.c, p.R), :y)                # slot "mvnormal"
            @trace(normal(p.h' * x + p.c0, p.sd), :z)                # slot "normal" (or mean x^2/20)
            @trace(normal(p.h' * x + p.c0, exp(p.g' * x + p.s)), :r)  # slot "normal", log-linear sd
            @trace(poisson(exp(p.h' * x + p.c0)), :count)            # slot "poisson"
            @trace(bernoulli(1 / (1 + exp(-(p.h' * x + p.c0)))), :on)  # slot "bernoulli"
            @trace(categorical(softmax(p.W * x + p.c)), :kind)       # slot "categorical" (0-based here)
            @trace(gamma(exp(p.h' * x + p.c0), 2.0), :g)               # a library slot (any scalar
                                                                     # distribution, arguments link(h.x + c))
            return x
        end

    latent: {"form": "affine", "A", "b", "Q", "mu0", "P0"[, "inputs": True]} or
            {"form": "switching", "prior" [nz], "T" [nz, nz], "A" [nz, dx, dx], "b" [nz, dx],
             "Q" [nz, dx, dx], "mu0" [dx], "P0" [dx, dx][, "regime_name": "z"]}: two
            latent addresses, z_t ~ categorical(T[:, z_{t-1}]) and
            x_t ~ mvnormal(A[z_t] x_{t-1} + b[z_t], Q[z_t]); the state is x then z
            one-hot (d = dx + nz), so a slot's h.x + c loads x and adds a
            per-regime offset h[dx + z]; or
            {"form": "kitagawa", "mu1", "s1", "sd_x"} (d = 1) or
            {"form": "categorical", "prior" [K], "T" [K, K] (T[new, prev])}: z_t ~
            categorical(T[:, z_{t-1}]); the engine keeps z one-hot (d = K), so a
            slot's affine mean h.x + c is h[z] + c — per-class parameters
            "inputs": the kernel takes a per-step argument u_t (d values, zero when a
            step gives none): x_t ~ mvnormal(A x_{t-1} + (b + u_t), Q) — the Unfold's
            arguments extended by one value per step, new_args = (t, u_t)
    slots:  [{"name", "dist", ...}] with per distribution
            mvnormal: H [m, d], c [m], R [m, m]; normal: h [d], c, sd (or mean "x^2/20", sd;
            or h [d], c, "log_sd": {"g": [d], "s"} for sd = exp(g.x + s) — stochastic volatility);
            poisson / bernoulli: h [d], c; categorical: W [m, d], c [m];
            library: "args": [a_1, ...], one per argument of the named distribution
            (normal, uniform, uniform_discrete, bernoulli, gamma, inv_gamma, beta,
            exponential, poisson, binom, neg_binom, geometric, laplace, cauchy,
            beta_uniform — Gen's argument order), each a constant or
            {"link": "identity" | "exp" | "logistic", "h": [d], "c"}
    Observations of step t: {("chain", t, name): value} (any subset of the slots).
    A slot may depend on earlier scalar slots of its step: "parents": {name: g}
    adds sum g * y_name to its linear predictor (a normal slot's mean, a Poisson
    or Bernoulli slot's h.x + c, a library slot's first argument); a step that
    constrains such a slot constrains its parents too.
    """

    family = _lib.FAMILY_SLOTS

    def __init__(self, latent: dict, slots: list, latent_name: str = "x"):
        self.latent = dict(latent)
        self.latent_name = latent_name
        form = self.latent.get("form", "affine")
        if form == "affine":
            self.A = np.atleast_2d(np.asarray(latent["A"], dtype=np.float64))
            self.d = self.A.shape[0]
            f = lambda k, shape: np.asarray(latent[k], dtype=np.float64).reshape(shape)  # noqa: E731
            self.b = f("b", (self.d,)) if "b" in latent else np.zeros(self.d)
            self.Q, self.mu0, self.P0 = f("Q", (self.d, self.d)), f("mu0", (self.d,)), f("P0", (self.d, self.d))
            self.inputs = bool(latent.get("inputs", False))
        elif form == "switching":
            self.inputs = False
            self.prior = np.asarray(latent["prior"], dtype=np.float64).ravel()
            self.nz = self.prior.size
            self.T = np.asarray(latent["T"], dtype=np.float64).reshape(self.nz, self.nz)
            self.A = np.asarray(latent["A"], dtype=np.float64)
            self.dx = self.A.shape[-1]
            self.A = self.A.reshape(self.nz, self.dx, self.dx)
            self.b = np.asarray(latent.get("b", np.zeros((self.nz, self.dx))), dtype=np.float64).reshape(self.nz, self.dx)
            self.Q = np.asarray(latent["Q"], dtype=np.float64).reshape(self.nz, self.dx, self.dx)
            self.mu0 = np.asarray(latent["mu0"], dtype=np.float64).reshape(self.dx)
            self.P0 = np.asarray(latent["P0"], dtype=np.float64).reshape(self.dx, self.dx)
            self.regime_name = latent.get("regime_name", "z")
            self.d = self.dx + self.nz
        elif form == "categorical":
            self.inputs = False
            self.prior = np.asarray(latent["prior"], dtype=np.float64).ravel()
            self.d = self.prior.size
            self.T = np.asarray(latent["T"], dtype=np.float64).reshape(self.d, self.d)
        elif form == "kitagawa":
            self.inputs = False
            self.d = 1
            self.mu1, self.s1, self.sd_x = float(latent["mu1"]), float(latent["s1"]), float(latent["sd_x"])
        else:
            raise ValueError(f"latent form {form!r}: 'affine', 'kitagawa', 'categorical' or 'switching'")
        self.form = form
        if not 1 <= len(slots) <= 4:
            raise ValueError("1..4 observed slots")
        self.slots = []
        for s in slots:
            s = dict(s)
            dist = s["dist"]
            if "args" in s:  # a library slot
                if dist not in _LIB:
                    raise ValueError(f"library slot distribution {dist!r}: one of {sorted(_LIB)}")
                lid, na = _LIB[dist]
                if len(s["args"]) != na:
                    raise ValueError(f"{dist} takes {na} arguments")
                args = []
                for a in s["args"]:
                    if isinstance(a, dict):
                        link = a.get("link", "identity")
                        if link not in _ARG_LINK:
                            raise ValueError(f"argument link {link!r}")
                        h = np.asarray(a.get("h", np.zeros(self.d)), dtype=np.float64).reshape(self.d)
                        args.append((link, h, float(a.get("c", 0.0))))
                    else:
                        args.append(("identity", np.zeros(self.d), float(a)))
                s.update(args=args, lib=lid, m=lid, link="library")
                self.slots.append(s)
                continue
            if dist not in _SLOT_DIST:
                raise ValueError(f"slot distribution {dist!r}")
            if dist == "mvnormal":
                s["H"] = np.atleast_2d(np.asarray(s["H"], dtype=np.float64))
                s["m"] = s["H"].shape[0]
                s["c"] = np.asarray(s.get("c", np.zeros(s["m"])), dtype=np.float64).reshape(s["m"])
                s["R"] = np.asarray(s["R"], dtype=np.float64).reshape(s["m"], s["m"])
                s["link"] = "affine"
            elif dist == "categorical":
                s["W"] = np.atleast_2d(np.asarray(s["W"], dtype=np.float64))
                s["m"] = s["W"].shape[0]
                s["c"] = np.asarray(s.get("c", np.zeros(s["m"])), dtype=np.float64).reshape(s["m"])
                s["link"] = "softmax"
            else:
                s["m"] = 1
                s["link"] = {"normal": s.get("mean", "affine"), "poisson": "exp", "bernoulli": "logistic"}[dist]
                if dist == "normal" and "log_sd" in s:
                    if s["link"] != "affine":
                        raise ValueError("a log-linear sd takes the affine mean")
                    s["link"] = "logscale"
                    s["g"] = np.asarray(s["log_sd"]["g"], dtype=np.float64).reshape(self.d)
                    s["s"] = float(s["log_sd"].get("s", 0.0))
                if s["link"] in ("affine", "logscale"):
                    s["h"] = np.asarray(s.get("h", np.zeros(self.d)), dtype=np.float64).reshape(self.d)
                    s["c"] = float(s.get("c", 0.0))
            self.slots.append(s)
        self.names = [s["name"] for s in self.slots]
        self.deps = []  # (child k, parent j, g)
        for k, s in enumerate(self.slots):
            for name, g in dict(s.get("parents", {})).items():
                if name not in self.names[:k]:
                    raise ValueError(f"slot {s['name']!r}: parent {name!r} must be an earlier slot")
                j = self.names.index(name)
                if self.slots[j]["dist"] == "mvnormal" and "lib" not in self.slots[j]:
                    raise ValueError("a parent slot is scalar")
                if not ("lib" in s or s["dist"] in ("poisson", "bernoulli") or
                        (s["dist"] == "normal" and s["link"] != "x^2/20")):
                    raise ValueError(f"slot {s['name']!r}: a dependent slot is a normal (affine mean), poisson, "
                                     "bernoulli or library slot")
                self.deps.append((k, j, float(g)))
        self.dy = sum(s["m"] if s["dist"] == "mvnormal" and "lib" not in s else 1 for s in self.slots)

    def params(self):
        code = {"affine": 2.0 if self.inputs else 0.0, "kitagawa": 1.0, "categorical": 3.0, "switching": 4.0}[self.form]
        p = [code, float(len(self.slots))]
        for s in self.slots:
            if "lib" in s:
                p += [6.0, float(s["lib"]), 0.0]
                continue
            p += [float(_SLOT_DIST[s["dist"]]), float(s["m"]), float(_LINK[s["link"]])]
        if self.form == "affine":
            p += list(self.A.ravel()) + list(self.b) + list(self.Q.ravel()) + list(self.mu0) + list(self.P0.ravel())
        elif self.form == "categorical":
            p += list(self.prior) + list(self.T.ravel())
        elif self.form == "switching":
            p += [float(self.nz)] + list(self.prior) + list(self.T.ravel())
            for z in range(self.nz):
                p += list(self.A[z].ravel()) + list(self.b[z]) + list(self.Q[z].ravel())
            p += list(self.mu0) + list(self.P0.ravel())
        else:
            p += [self.mu1, self.s1, self.sd_x]
        for s in self.slots:
            if "lib" in s:
                for link, h, c in s["args"]:
                    p += [float(_ARG_LINK[link]), *h, c]
            elif s["dist"] == "mvnormal":
                p += list(s["H"].ravel()) + list(s["c"]) + list(s["R"].ravel())
            elif s["dist"] == "normal" and s["link"] == "logscale":
                p += [*s["h"], s["c"], *s["g"], s["s"]]
            elif s["dist"] == "normal":
                p += ([*s["h"], s["c"]] if s["link"] == "affine" else []) + [float(s["sd"])]
            elif s["dist"] == "categorical":
                p += list(s["W"].ravel()) + list(s["c"])
            else:
                p += [*s["h"], s["c"]]
        if self.deps:
            p += [float(len(self.deps))]
            for k, j, g in self.deps:
                p += [float(k), float(j), g]
        return np.asarray(p, dtype=np.float64)

    def obs_address(self, t: int, name: str | None = None):
        return ("chain", t, self.names[0] if name is None else name)

    def obs_from_choicemap(self, cm, t: int):
        """The constrained slots of step t ({name: value}, None if none); any
        other address would update or delete an existing choice
        (particle_filter.jl:168-170)."""
        out = {}
        for a, v in cm:
            if len(a) == 3 and a[0] == "chain" and a[1] == t and a[2] in self.names:
                out[a[2]] = v
            else:
                raise _lib.GenHipError(2, f"constraint at {a}: only the slots {self.names} of step {t} may be "
                                          "constrained (discard must be empty)")
        return out or None

    def _slot_dict(self, value) -> dict:
        if isinstance(value, dict):
            return value
        if len(self.slots) == 1:
            return {self.names[0]: value}
        raise ValueError("a slot model's observation is a {slot name: value} dict")

    def gh_obs(self, value, u=None):
        """The gh_obs chain of one step's observation (slot ids in model order),
        and the step's input u_t (an entry with slot GH_SLOT_INPUT) if given."""
        vals = {} if value is None else self._slot_dict(value)
        present = [(k, np.ascontiguousarray(np.atleast_1d(np.asarray(vals[n], dtype=np.float64)).ravel()))
                   for k, n in enumerate(self.names) if n in vals and vals[n] is not None]
        unknown = set(vals) - set(self.names)
        if unknown:
            raise _lib.GenHipError(1, f"no slot named {sorted(unknown)}")
        if u is not None:
            if not self.inputs:
                raise _lib.GenHipError(1, "this slot model takes no per-step input (latent 'inputs': True)")
            present.append((_lib.SLOT_INPUT, np.ascontiguousarray(np.asarray(u, dtype=np.float64).reshape(self.d))))
        chain = (_lib.Obs * max(1, len(present)))()
        for i, (k, arr) in enumerate(present):
            chain[i] = _lib.Obs(_lib.dptr(arr), arr.size, 1, k, 0, None)
        for i in range(len(present) - 1):
            chain[i].next = ctypes.pointer(chain[i + 1])
        if not present:
            chain[0] = _lib.Obs(None, 0, 0, 0, 0, None)
        keep = {self.names[k]: arr for k, arr in present if k >= 0}
        return chain[0], (chain, keep, [arr for k, arr in present if k < 0])

    def latent_value(self, x):
        if self.form == "categorical":  # (the class: Gen's categorical returns an Int; 0-based here)
            return int(np.argmax(x))
        return super().latent_value(x)

    def latent_addresses(self, t: int) -> list:
        if self.form == "switching":
            return [("chain", t, self.regime_name), ("chain", t, self.latent_name)]
        return [self.latent_address(t)]

    def latent_part(self, k: int, x):
        if self.form == "switching":  # (z: 0-based regime; x: the continuous state)
            x = np.asarray(x)
            return int(np.argmax(x[self.dx:])) if k == 0 else (float(x[0]) if self.dx == 1 else x[:self.dx].copy())
        return self.latent_value(x)

    def latent_part_column(self, k: int, col):
        if self.form == "switching":
            return np.argmax(col[:, self.dx:], axis=1) if k == 0 else (col[:, 0] if self.dx == 1 else col[:, :self.dx])
        return self.latent_column(col)

    def latent_part_logpdf(self, k: int, t: int, xp, x) -> float:
        """A switching model's z (k = 0) or x (k = 1) score at step t."""
        z = int(np.argmax(x[self.dx:]))
        if k == 0:
            return float(np.log(self.prior[z] if t == 1 else self.T[z, int(np.argmax(xp[self.dx:]))]))
        from scipy import stats

        mean, cov = (self.mu0, self.P0) if t == 1 else (self.A[z] @ xp[:self.dx] + self.b[z], self.Q[z])
        return float(stats.multivariate_normal.logpdf(x[:self.dx], mean, cov))

    def latent_column(self, col):
        if self.form == "categorical":
            return np.argmax(col, axis=1)
        return super().latent_column(col)

    # ---- host-side reference densities (numpy / closed forms; the tests' pins)
    def _mean_param(self, s, x, dk: float = 0.0):
        x = np.atleast_1d(x)
        if s["dist"] == "mvnormal":
            return s["H"] @ x + s["c"]
        if s["dist"] == "categorical":
            eta = s["W"] @ x + s["c"]
            e = np.exp(eta - eta.max())
            return e / e.sum()
        if s["link"] == "x^2/20":
            return x[0] * x[0] / 20.0
        eta = float(s["h"] @ x + s["c"]) + dk
        return {"normal": eta, "poisson": np.exp(eta), "bernoulli": 1.0 / (1.0 + np.exp(-eta))}[s["dist"]]

    @staticmethod
    def lib_args(s, x, dk: float = 0.0) -> list:
        """A library slot's arguments at latent x (dk: the parent term, joining the first)."""
        x = np.atleast_1d(x)
        out = []
        for i, (link, h, c) in enumerate(s["args"]):
            eta = float(h @ x + c) + (dk if i == 0 else 0.0)
            out.append({"identity": eta, "exp": float(np.exp(eta)), "logistic": 1.0 / (1.0 + np.exp(-eta))}[link])
        return out

    @staticmethod
    def lib_logpdf(dist: str, y: float, a: list) -> float:
        """The reference's logpdf of a library distribution (scipy's densities;
        Gen's argument conventions: exponential(rate), gamma / inv_gamma(shape,
        scale), neg_binom / geometric count failures, uniform_discrete(lo, hi)
        inclusive, beta_uniform(theta, a, b))."""
        from scipy import stats

        if dist == "normal":
            return float(stats.norm.logpdf(y, a[0], a[1]))
        if dist == "uniform":
            return float(stats.uniform.logpdf(y, a[0], a[1] - a[0]))
        if dist == "uniform_discrete":
            return float(stats.randint.logpmf(y, a[0], a[1] + 1))
        if dist == "bernoulli":
            return float(np.log(a[0]) if y else np.log(1.0 - a[0]))
        if dist == "gamma":
            return float(stats.gamma.logpdf(y, a[0], scale=a[1]))
        if dist == "inv_gamma":
            return float(stats.invgamma.logpdf(y, a[0], scale=a[1]))
        if dist == "beta":
            return float(stats.beta.logpdf(y, a[0], a[1]))
        if dist == "exponential":
            return float(stats.expon.logpdf(y, scale=1.0 / a[0]))
        if dist == "poisson":
            return float(stats.poisson.logpmf(y, a[0]))
        if dist == "binom":
            return float(stats.binom.logpmf(y, a[0], a[1]))
        if dist == "neg_binom":
            return float(stats.nbinom.logpmf(y, a[0], a[1]))
        if dist == "geometric":
            return float(stats.geom.logpmf(y + 1, a[0]))
        if dist == "laplace":
            return float(stats.laplace.logpdf(y, a[0], a[1]))
        if dist == "cauchy":
            return float(stats.cauchy.logpdf(y, a[0], a[1]))
        th = a[0]  # beta_uniform
        return float(np.logaddexp(np.log(th) + stats.beta.logpdf(y, a[1], a[2]), np.log(1.0 - th)))

    @staticmethod
    def lib_sample(dist: str, a: list, rng: np.random.Generator) -> float:
        if dist == "normal":
            return float(rng.normal(a[0], a[1]))
        if dist == "uniform":
            return float(rng.uniform(a[0], a[1]))
        if dist == "uniform_discrete":
            return float(rng.integers(int(a[0]), int(a[1]) + 1))
        if dist == "bernoulli":
            return float(rng.random() < a[0])
        if dist == "gamma":
            return float(rng.gamma(a[0], a[1]))
        if dist == "inv_gamma":
            return float(a[1] / rng.gamma(a[0], 1.0))
        if dist == "beta":
            return float(rng.beta(a[0], a[1]))
        if dist == "exponential":
            return float(rng.exponential(1.0 / a[0]))
        if dist == "poisson":
            return float(rng.poisson(a[0]))
        if dist == "binom":
            return float(rng.binomial(int(a[0]), a[1]))
        if dist == "neg_binom":
            return float(rng.negative_binomial(a[0], a[1]))
        if dist == "geometric":
            return float(rng.geometric(a[0]) - 1)
        if dist == "laplace":
            return float(rng.laplace(a[0], a[1]))
        if dist == "cauchy":
            return float(a[0] + a[1] * rng.standard_cauchy())
        return float(rng.beta(a[1], a[2]) if rng.random() < a[0] else rng.random())

    def slot_sd(self, s, x) -> float:
        """A normal slot's standard deviation at latent x."""
        if s["link"] == "logscale":
            return float(np.exp(s["g"] @ np.atleast_1d(x) + s["s"]))
        return s["sd"]

    def parent_term(self, k: int, yvals: dict | None) -> float:
        """Slot k's parent term, sum of g * y_parent in slot order (the engine
        takes an fma chain; host-side references agree to rounding)."""
        dk = 0.0
        for kk, j, g in sorted(self.deps, key=lambda e: e[1]):
            if kk == k and g != 0.0:
                dk = g * float(np.asarray(yvals[self.names[j]]).ravel()[0]) + dk
        return dk

    def slot_logpdf(self, k: int, y, x, yvals: dict | None = None) -> float:
        """logpdf of slot k's value y at latent x (scipy-free closed forms of
        the reference's distributions); yvals: the step's other slot values
        (a dependent slot's parents)."""
        from math import lgamma

        s = self.slots[k]
        dk = self.parent_term(k, yvals) if any(kk == k for kk, _, _ in self.deps) else 0.0
        if "lib" in s:
            a = self.lib_args(s, x, dk)
            return self.lib_logpdf(s["dist"], float(y), a)
        mp = self._mean_param(s, x, dk)
        if s["dist"] == "mvnormal":
            return _mvn_logpdf(np.atleast_1d(y), mp, s["R"])
        if s["dist"] == "normal":
            return _normal_logpdf(float(y), mp, self.slot_sd(s, x))
        if s["dist"] == "poisson":
            return float(y * np.log(mp) - mp - lgamma(y + 1.0))
        if s["dist"] == "bernoulli":
            return float(np.log(mp) if y else np.log(1.0 - mp))
        return float(np.log(mp[int(y)]))

    def simulate(self, T: int, rng: np.random.Generator, inputs=None):
        """Draw (xs [T, d], ys [T] of {slot name: value}) from the model (numpy
        RNG; synthetic data only); inputs [T, d]: the per-step inputs u_t of a
        model with inputs (row t - 1 for step t; row 0 unused)."""
        xs = np.zeros((T, self.d))
        ys = []
        for t in range(1, T + 1):
            if self.form == "affine":
                u = np.zeros(self.d) if inputs is None or t == 1 else np.asarray(inputs[t - 1], dtype=np.float64)
                x = (rng.multivariate_normal(self.mu0, self.P0) if t == 1 else
                     rng.multivariate_normal(self.A @ xs[t - 2] + (self.b + u), self.Q))
            elif self.form == "switching":  # (x then z one-hot, as the engine stores it)
                zp = None if t == 1 else int(np.argmax(xs[t - 2, self.dx:]))
                pz = self.prior if t == 1 else self.T[:, zp]
                z = rng.choice(self.nz, p=pz / pz.sum())
                xc = (rng.multivariate_normal(self.mu0, self.P0) if t == 1 else
                      rng.multivariate_normal(self.A[z] @ xs[t - 2, :self.dx] + self.b[z], self.Q[z]))
                x = np.concatenate([xc, np.eye(self.nz)[z]])
            elif self.form == "categorical":  # (one-hot, as the engine stores it)
                pz = self.prior if t == 1 else self.T[:, int(np.argmax(xs[t - 2]))]
                x = np.eye(self.d)[rng.choice(self.d, p=pz / pz.sum())]
            else:
                v = xs[t - 2, 0]
                x = np.array([rng.normal(self.mu1, self.s1) if t == 1 else
                              rng.normal(v / 2 + 25 * v / (1 + v * v) + 8 * np.cos(1.2 * t), self.sd_x)])
            xs[t - 1] = x
            y = {}
            for k, s in enumerate(self.slots):
                dk = self.parent_term(k, y) if any(kk == k for kk, _, _ in self.deps) else 0.0
                if "lib" in s:
                    y[s["name"]] = self.lib_sample(s["dist"], self.lib_args(s, x, dk), rng)
                    continue
                mp = self._mean_param(s, x, dk)
                if s["dist"] == "mvnormal":
                    y[s["name"]] = rng.multivariate_normal(mp, s["R"])
                elif s["dist"] == "normal":
                    y[s["name"]] = float(rng.normal(mp, self.slot_sd(s, x)))
                elif s["dist"] == "poisson":
                    y[s["name"]] = float(rng.poisson(mp))
                elif s["dist"] == "bernoulli":
                    y[s["name"]] = float(rng.random() < mp)
                else:
                    y[s["name"]] = float(rng.choice(s["m"], p=mp))
            ys.append(y)
        return xs, ys
