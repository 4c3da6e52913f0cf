"""The slot-described Unfold family (GH_FAMILY_SLOTS, gen_amd/csrc/gh_slots.h).

A Static-DSL kernel outside the four hand-lowered families is described by
its address slots — one latent, up to four observed addresses with their
distributions and mean forms (static_ir/generate.jl:24-43) — and a step may
constrain any subset of them (choice_map.jl:163-225).  Pins:

* CPU: the oracle's slot restatement reduces to the LGSSM and Kitagawa
  families' restatements bit for bit when the slots describe those models,
  and every slot's score equals the reference distribution's closed form
  (mvnormal.jl:12-16, normal.jl:56-60, poisson.jl:10-12, bernoulli.jl:10-12,
  categorical.jl:10-12) to 1e-12 — scipy's densities where scipy has them;
* GPU: the device family equals those families bit for bit (states, weights,
  ancestors), and equals the oracle bit for bit on a Poisson-count SSM with
  several observed addresses per step (some steps constraining a subset,
  one step none), call by call and batched, with simulate, the score columns
  and rejuvenation.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import gen_amd as gen  # noqa: E402
from oracle import oracle as O  # noqa: E402


def lg_as_slots(lg):
    return gen.SlotSSM({"form": "affine", "A": lg.A, "b": lg.b, "Q": lg.Q, "mu0": lg.mu0, "P0": lg.P0},
                       [{"name": "y", "dist": "mvnormal", "H": lg.H, "c": lg.c, "R": lg.R}])


def kit_as_slots(kit):
    # (sd_x = sqrt(var_x) exactly: var_x = 4; the family takes variances, the slot a standard deviation)
    return gen.SlotSSM({"form": "kitagawa", "mu1": kit.mu1, "s1": kit.s1, "sd_x": float(np.sqrt(kit.var_x))},
                       [{"name": "y", "dist": "normal", "mean": "x^2/20", "sd": float(np.sqrt(kit.var_y))}])


def count_model():
    """A Poisson-count SSM with three more observed addresses per step."""
    return gen.SlotSSM(
        {"form": "affine", "A": [[0.9, 0.05], [0.0, 0.8]], "b": [0.0, 0.1], "Q": [[0.05, 0.01], [0.01, 0.04]],
         "mu0": [0.5, 0.0], "P0": [[0.3, 0.0], [0.0, 0.3]]},
        [{"name": "count", "dist": "poisson", "h": [1.0, 0.5], "c": 0.2},
         {"name": "z", "dist": "normal", "h": [0.3, -0.2], "c": 0.1, "sd": 0.7},
         {"name": "on", "dist": "bernoulli", "h": [1.5, 0.0], "c": -0.3},
         {"name": "kind", "dist": "categorical", "W": [[1.0, 0.0], [0.0, 1.0], [-1.0, 1.0]], "c": [0.0, 0.2, -0.1]}])


def changed_count_model():
    """count_model() with other numbers in every block (the same slot layout):
    a parameter change, new_args = (t, model')."""
    return gen.SlotSSM(
        {"form": "affine", "A": [[0.8, 0.1], [-0.05, 0.85]], "b": [0.05, 0.0], "Q": [[0.07, 0.0], [0.0, 0.05]],
         "mu0": [0.5, 0.0], "P0": [[0.3, 0.0], [0.0, 0.3]]},
        [{"name": "count", "dist": "poisson", "h": [0.9, 0.6], "c": 0.1},
         {"name": "z", "dist": "normal", "h": [0.25, -0.1], "c": 0.0, "sd": 0.9},
         {"name": "on", "dist": "bernoulli", "h": [1.2, 0.3], "c": -0.1},
         {"name": "kind", "dist": "categorical", "W": [[0.8, 0.0], [0.1, 1.1], [-1.0, 0.7]], "c": [0.1, 0.0, -0.2]}])


def count_model_inputs():
    """count_model() whose kernel takes a per-step input u_t:
    x_t ~ mvnormal(A x_{t-1} + (b + u_t), Q)."""
    m = count_model()
    lat = dict(m.latent)
    lat["inputs"] = True
    return gen.SlotSSM(lat, [dict(sl) for sl in count_model().slots])


def count_inputs(T=10, seed=11):
    """Per-step inputs (row t - 1 for step t), some steps without one (None)."""
    rng = np.random.default_rng(seed)
    u = [0.4 * rng.standard_normal(2) for _ in range(T)]
    u[0] = None  # (step 1 has no transition)
    u[3] = None
    return u


def switching_model():
    """A 3-state switching model: a categorical latent z_t (one-hot) with
    per-class normal, Poisson, Bernoulli and categorical emissions (a slot's
    affine mean h.x + c is h[z] + c)."""
    return gen.SlotSSM(
        {"form": "categorical", "prior": [0.5, 0.3, 0.2],
         "T": [[0.8, 0.1, 0.2], [0.15, 0.85, 0.1], [0.05, 0.05, 0.7]]},
        [{"name": "level", "dist": "normal", "h": [-1.0, 0.5, 2.0], "c": 0.1, "sd": 0.6},
         {"name": "count", "dist": "poisson", "h": [0.0, 1.0, 2.0], "c": -0.2},
         {"name": "alarm", "dist": "bernoulli", "h": [-2.0, 0.0, 1.5], "c": 0.0},
         {"name": "kind", "dist": "categorical", "W": [[1.0, 0.0, -1.0], [0.0, 1.0, 0.0], [-1.0, 0.0, 1.0]],
          "c": [0.0, 0.0, 0.1]}])


def sv_model():
    """A stochastic-volatility model: an AR(1) log-volatility
    h_t ~ normal(mu + phi (h_{t-1} - mu), sigma) and returns
    r_t ~ normal(0, exp(h_t / 2)), plus a second return with a mean and its own
    log-linear scale (normal slots with a log-linear standard deviation)."""
    mu, phi, sig = -0.5, 0.95, 0.25
    return gen.SlotSSM(
        {"form": "affine", "A": [[phi]], "b": [mu * (1 - phi)], "Q": [[sig * sig]], "mu0": [mu],
         "P0": [[sig * sig / (1 - phi * phi)]]},
        [{"name": "r", "dist": "normal", "log_sd": {"g": [0.5], "s": 0.0}},
         {"name": "r2", "dist": "normal", "h": [0.3], "c": 0.1, "log_sd": {"g": [0.25], "s": -0.5}}])


def sv_obs(T=12, seed=8):
    m = sv_model()
    _, ys = m.simulate(T, np.random.default_rng(seed))
    obs = [dict(y) for y in ys]
    del obs[3]["r2"]
    obs[5] = {}
    return m, obs


_LAT2 = {"form": "affine", "A": [[0.9, 0.05], [0.0, 0.8]], "b": [0.0, 0.1], "Q": [[0.05, 0.01], [0.01, 0.04]],
         "mu0": [0.5, 0.0], "P0": [[0.3, 0.0], [0.0, 0.3]]}


def _arg(link, h, c):
    return {"link": link, "h": h, "c": c}


def library_models():
    """Slot models whose observed addresses are library distributions with
    latent-dependent arguments: between them every scalar distribution a
    library slot may name."""
    return {
        "m1": gen.SlotSSM(_LAT2, [
            {"name": "g", "dist": "gamma", "args": [_arg("exp", [0.5, 0.2], 0.3), 2.0]},
            {"name": "nb", "dist": "neg_binom", "args": [3.0, _arg("logistic", [1.0, -0.5], 0.2)]},
            {"name": "lp", "dist": "laplace", "args": [_arg("identity", [1.0, 0.5], 0.1), 0.5]},
            {"name": "b", "dist": "beta", "args": [_arg("exp", [0.4, 0.0], 0.5), _arg("exp", [0.0, -0.4], 0.7)]}]),
        "m2": gen.SlotSSM(_LAT2, [
            {"name": "e", "dist": "exponential", "args": [_arg("exp", [0.3, 0.3], 0.0)]},
            {"name": "bn", "dist": "binom", "args": [10.0, _arg("logistic", [1.2, 0.0], -0.3)]},
            {"name": "ge", "dist": "geometric", "args": [_arg("logistic", [0.0, 1.0], -0.5)]},
            {"name": "ca", "dist": "cauchy", "args": [_arg("identity", [0.8, 0.0], 0.0), 0.7]}]),
        "m3": gen.SlotSSM(_LAT2, [
            {"name": "n", "dist": "normal", "args": [_arg("identity", [1.0, 0.0], 0.0), _arg("exp", [0.0, 0.5], -0.7)]},
            {"name": "u", "dist": "uniform", "args": [-4.0, 4.0]},
            {"name": "ig", "dist": "inv_gamma", "args": [_arg("exp", [0.2, 0.2], 1.0), 1.5]},
            {"name": "ud", "dist": "uniform_discrete", "args": [0.0, 5.0]}]),
        "m4": gen.SlotSSM(_LAT2, [
            {"name": "p", "dist": "poisson", "args": [_arg("exp", [1.0, 0.5], 0.2)]},
            {"name": "be", "dist": "bernoulli", "args": [_arg("logistic", [1.5, 0.0], -0.3)]},
            {"name": "bu", "dist": "beta_uniform", "args": [_arg("logistic", [0.5, 0.5], 0.0), 2.0,
                                                            _arg("exp", [0.3, 0.0], 0.4)]}]),
    }


def library_obs(name, T=10, seed=6):
    m = library_models()[name]
    _, ys = m.simulate(T, np.random.default_rng(seed))
    obs = [dict(y) for y in ys]
    del obs[2][m.names[0]]
    obs[4] = {}
    return m, obs


def slds_model(same=False):
    """A switching linear dynamical system: two latent addresses per step,
    z_t ~ categorical(T[:, z_{t-1}]) and x_t ~ mvnormal(A[z] x + b[z], Q[z]),
    with a normal observation of x (plus a per-regime offset) and a Poisson
    count whose rate depends on the regime.  same=True: both regimes share the
    dynamics and the emission ignores z (the LG-SSM with a decoupled chain)."""
    A = np.array([[[0.95, 0.1], [0.0, 0.9]], [[0.5, -0.3], [0.2, 0.6]]])
    b = np.array([[0.0, 0.1], [0.5, -0.2]])
    Q = np.array([[[0.05, 0.01], [0.01, 0.04]], [[0.2, 0.0], [0.0, 0.15]]])
    if same:
        A, b, Q = np.stack([A[0], A[0]]), np.stack([b[0], b[0]]), np.stack([Q[0], Q[0]])
    lat = {"form": "switching", "prior": [0.7, 0.3], "T": [[0.9, 0.2], [0.1, 0.8]], "A": A, "b": b, "Q": Q,
           "mu0": [0.0, 0.0], "P0": [[0.5, 0.0], [0.0, 0.5]]}
    if same:
        return gen.SlotSSM(lat, [{"name": "y", "dist": "mvnormal", "H": [[1.0, 0.0, 0.0, 0.0], [0.0, 1.0, 0.0, 0.0]],
                                  "c": [0.0, 0.0], "R": [[0.3, 0.0], [0.0, 0.3]]}])
    return gen.SlotSSM(lat, [{"name": "y", "dist": "normal", "h": [1.0, 0.5, 0.0, 1.5], "c": 0.0, "sd": 0.4},
                             {"name": "n", "dist": "poisson", "h": [0.2, 0.0, 0.0, 1.0], "c": 0.3}])


def slds_obs(T=12, seed=4):
    m = slds_model()
    _, ys = m.simulate(T, np.random.default_rng(seed))
    obs = [dict(y) for y in ys]
    del obs[3]["n"]
    obs[6] = {}
    return m, obs


def dep_model(g=(0.3, -0.5, 0.1, 0.05)):
    """Observed addresses that depend on each other within a step: a normal
    reading, a count whose log-rate adds 0.3 x the reading, an alarm whose
    logit adds -0.5 x the reading + 0.1 x the count, and a gamma whose log-shape
    adds 0.05 x the count."""
    return gen.SlotSSM(_LAT2, [
        {"name": "a", "dist": "normal", "h": [1.0, 0.0], "c": 0.0, "sd": 0.5},
        {"name": "n", "dist": "poisson", "h": [0.5, 0.2], "c": 0.1, "parents": {"a": g[0]}},
        {"name": "b", "dist": "bernoulli", "h": [0.0, 1.0], "c": 0.0, "parents": {"a": g[1], "n": g[2]}},
        {"name": "g", "dist": "gamma", "args": [_arg("exp", [0.2, 0.0], 0.1), 1.5], "parents": {"n": g[3]}}])


def dep_obs(T=10, seed=12):
    m = dep_model()
    _, ys = m.simulate(T, np.random.default_rng(seed))
    obs = [dict(y) for y in ys]
    del obs[2]["b"]           # a child left out: fine
    del obs[4]["g"], obs[4]["b"]
    obs[6] = {"a": obs[6]["a"]}
    return m, obs


def count_obs(T=10, seed=5):
    """Observations with some slots missing at some steps (and one empty step)."""
    m = count_model()
    _, ys = m.simulate(T, np.random.default_rng(seed))
    obs = [dict(y) for y in ys]
    del obs[2]["z"]
    obs[4] = {}
    del obs[5]["count"]
    del obs[6]["kind"], obs[6]["on"]
    return m, obs


def _obs_at(model, y, t):
    if isinstance(y, dict):
        return {("chain", t, k): v for k, v in y.items()}
    return {model.obs_address(t): y}


# ------------------------------------------------------------------ CPU
def test_oracle_slots_reduce_to_lgssm_family_bitexact():
    lg = gen.LinearGaussianSSM.benchmark(4)
    sl = lg_as_slots(lg)
    _, ys = lg.simulate(10, np.random.default_rng(2))
    a = O.run_pf(lg, ys, 3000, 7)
    b = O.run_pf(sl, [{"y": y} for y in ys], 3000, 7)
    assert np.array_equal(a.state(), b.state())
    assert np.array_equal(a.parents(), b.parents())
    assert np.array_equal(a.log_weights(), b.log_weights())
    assert a.log_ml_estimate() == b.log_ml_estimate()
    for x, y in zip(a.scores(per_step=True), b.scores(per_step=True)):
        assert np.array_equal(x, y)


def test_oracle_slots_reduce_to_kitagawa_family_bitexact():
    kit = gen.KitagawaSSM(4.0, 1.0)
    _, ys = kit.simulate(12, np.random.default_rng(3))
    a = O.run_pf(kit, ys, 3000, 7)
    b = O.run_pf(kit_as_slots(kit), [{"y": y} for y in ys], 3000, 7)
    assert np.array_equal(a.state(), b.state())
    assert np.array_equal(a.parents(), b.parents())
    assert np.array_equal(a.log_weights(), b.log_weights())
    for x, y in zip(a.scores(per_step=True), b.scores(per_step=True)):
        assert np.array_equal(x, y)


def test_oracle_slot_scores_equal_reference_densities():
    """simulate's per-step scores: the observation column = the sum of the
    slots' logpdfs by the reference's formulas (scipy where it has the
    distribution), the latent column = mvnormal's logpdf."""
    from scipy import stats

    m = count_model()
    T, n = 5, 64
    X, Y, PS, _ = O.simulate(m, T, n, 3)
    s = m.slots
    for t in range(T):
        for j in range(n):
            x, y = X[t, :, j], Y[t, :, j]
            eta = [float(np.dot(s[k]["h"], x) + s[k]["c"]) for k in range(3)]
            logits = s[3]["W"] @ x + s[3]["c"]
            probs = np.exp(logits - logits.max())
            probs /= probs.sum()
            ref = (stats.poisson.logpmf(y[0], np.exp(eta[0])) + stats.norm.logpdf(y[1], eta[1], 0.7)
                   + stats.bernoulli.logpmf(y[2], 1.0 / (1.0 + np.exp(-eta[2]))) + np.log(probs[int(y[3])]))
            assert abs(ref - PS[t, 1, j]) < 1e-12 * max(1.0, abs(ref)), (t, j, ref, PS[t, 1, j])
            xp = X[t - 1, :, j] if t > 0 else None
            mean, cov = (m.mu0, m.P0) if t == 0 else (m.A @ xp + m.b, m.Q)
            assert abs(stats.multivariate_normal.logpdf(x, mean, cov) - PS[t, 0, j]) < 1e-12 * 10
    # the samplers: counts, switches and classes with the model's means
    T, n = 2, 20000
    X, Y, _, _ = O.simulate(m, T, n, 4)
    x = X[1]
    lam = np.exp(s[0]["h"] @ x + s[0]["c"])
    assert abs(Y[1, 0].mean() - lam.mean()) < 4 * np.sqrt(lam.mean() / n) + 1e-3
    p_on = 1.0 / (1.0 + np.exp(-(s[2]["h"] @ x + s[2]["c"])))
    assert abs(Y[1, 2].mean() - p_on.mean()) < 4 * np.sqrt(0.25 / n)


def test_oracle_sv_slot_scores_equal_reference_density():
    """The log-linear-scale normal slot: simulate's observation column is
    normal.jl:56-60's logpdf with std = exp(g.x + s) (scipy), the returns
    divided by their standard deviation are standard normal, and with g = 0
    the slot scores as the fixed-sd normal slot (to rounding: the fixed slot
    folds 1/(2 var) and the log-normaliser into constants)."""
    from scipy import stats

    m = sv_model()
    T, n = 6, 128
    X, Y, PS, _ = O.simulate(m, T, n, 3)
    for t in range(T):
        h = X[t, 0]
        ref = (stats.norm.logpdf(Y[t, 0], 0.0, np.exp(0.5 * h))
               + stats.norm.logpdf(Y[t, 1], 0.3 * h + 0.1, np.exp(0.25 * h - 0.5)))
        np.testing.assert_allclose(PS[t, 1], ref, rtol=1e-12, atol=1e-12)
    X, Y, _, _ = O.simulate(m, 2, 40000, 4)
    z = Y[1, 0] / np.exp(0.5 * X[1, 0])
    assert abs(z.mean()) < 4 / np.sqrt(40000) and abs(z.var() - 1.0) < 6 * np.sqrt(2 / 40000)
    lat = {"form": "affine", "A": [[0.9]], "b": [0.0], "Q": [[0.1]], "mu0": [0.0], "P0": [[1.0]]}
    fixed = gen.SlotSSM(lat, [{"name": "y", "dist": "normal", "h": [1.0], "c": 0.2, "sd": 0.7}])
    logs = gen.SlotSSM(lat, [{"name": "y", "dist": "normal", "h": [1.0], "c": 0.2,
                              "log_sd": {"g": [0.0], "s": float(np.log(0.7))}}])
    _, ys = fixed.simulate(8, np.random.default_rng(1))
    a = O.run_pf(fixed, ys, 500, 5, thr=0.0)
    b = O.run_pf(logs, ys, 500, 5, thr=0.0)
    assert np.array_equal(a.state(), b.state())
    np.testing.assert_allclose(b.log_weights(), a.log_weights(), rtol=1e-13, atol=1e-12)
    # the particle filter on it: the log-ML of two seeds agree at this size
    m, obs = sv_obs()
    l1 = O.run_pf(m, obs, 20000, 1).log_ml_estimate()
    l2 = O.run_pf(m, obs, 20000, 2).log_ml_estimate()
    assert np.isfinite(l1) and abs(l1 - l2) < 0.2


def test_oracle_library_slot_scores_equal_reference_densities():
    """Library slots (any scalar distribution of Gen's library, arguments
    link(h.x + c)): simulate's observation column is the sum of the slots'
    reference logpdfs (scipy's densities under Gen's argument conventions) for
    all fifteen distributions, and the samplers' means match the model's."""
    for name, m in library_models().items():
        T, n = 4, 48
        X, Y, PS, _ = O.simulate(m, T, n, 5)
        for t in range(T):
            for j in range(n):
                x = X[t, :, j]
                ref = sum(m.slot_logpdf(k, Y[t, k, j], x) for k in range(len(m.slots)))
                assert np.isfinite(ref), (name, t, j)
                assert abs(ref - PS[t, 1, j]) < 1e-10 * max(1.0, abs(ref)), (name, t, j, ref, PS[t, 1, j])
    m = library_models()["m1"]
    X, Y, _, _ = O.simulate(m, 2, 40000, 6)
    x = X[1]
    shape = np.exp(0.5 * x[0] + 0.2 * x[1] + 0.3)
    assert abs(Y[1, 0].mean() - (2.0 * shape).mean()) < 6 * np.sqrt((4.0 * shape).mean() / 40000)
    p = 1.0 / (1.0 + np.exp(-(x[0] - 0.5 * x[1] + 0.2)))
    nb_mean = 3.0 * (1 - p) / p
    assert abs(Y[1, 1].mean() - nb_mean.mean()) < 6 * np.sqrt((nb_mean / p).mean() / 40000)


def test_oracle_library_slots_reduce_to_the_fixed_slots():
    """A library poisson(exp(h.x + c)) or bernoulli(logistic(h.x + c)) slot is
    the fixed Poisson / Bernoulli slot bit for bit; a library normal with
    constant sd is the fixed normal slot to rounding (which folds its
    constants)."""
    fixed = gen.SlotSSM(_LAT2, [{"name": "count", "dist": "poisson", "h": [1.0, 0.5], "c": 0.2},
                                {"name": "on", "dist": "bernoulli", "h": [1.5, 0.0], "c": -0.3},
                                {"name": "z", "dist": "normal", "h": [0.3, -0.2], "c": 0.1, "sd": 0.7}])
    lib = gen.SlotSSM(_LAT2, [{"name": "count", "dist": "poisson", "args": [_arg("exp", [1.0, 0.5], 0.2)]},
                              {"name": "on", "dist": "bernoulli", "args": [_arg("logistic", [1.5, 0.0], -0.3)]},
                              {"name": "z", "dist": "normal", "args": [_arg("identity", [0.3, -0.2], 0.1), 0.7]}])
    _, ys = fixed.simulate(8, np.random.default_rng(2))
    two = [{k: y[k] for k in ("count", "on")} for y in ys]
    a = O.run_pf(fixed, two, 600, 5)
    b = O.run_pf(lib, two, 600, 5)
    assert np.array_equal(a.state(), b.state()) and np.array_equal(a.log_weights(), b.log_weights())
    a = O.run_pf(fixed, ys, 600, 5, thr=0.0)
    b = O.run_pf(lib, ys, 600, 5, thr=0.0)
    assert np.array_equal(a.state(), b.state())
    np.testing.assert_allclose(b.log_weights(), a.log_weights(), rtol=1e-13, atol=1e-12)


def test_oracle_switching_latent_scores_equal_reference_densities():
    """The switching latent (two latent addresses): simulate's latent column is
    log p(z_t | z_{t-1}) + mvnormal's logpdf of x_t under regime z_t (scipy),
    the observation column the slots' densities; with both regimes sharing
    the dynamics and an emission that ignores z, the filter's log-ML is the
    Kalman filter's of the LG-SSM to Monte Carlo error."""
    from scipy import stats

    m = slds_model()
    T, n = 5, 64
    X, Y, PS, _ = O.simulate(m, T, n, 3)
    for t in range(T):
        for j in range(n):
            x = X[t, :, j]
            xp = X[t - 1, :, j] if t > 0 else None
            ref = m.latent_part_logpdf(0, t + 1, xp, x) + m.latent_part_logpdf(1, t + 1, xp, x)
            assert abs(ref - PS[t, 0, j]) < 1e-11 * max(1.0, abs(ref)), (t, j, ref, PS[t, 0, j])
            z = int(np.argmax(x[2:]))
            assert x[2 + z] == 1.0 and x[2:].sum() == 1.0
            ob = stats.norm.logpdf(Y[t, 0, j], x[0] + 0.5 * x[1] + 1.5 * z, 0.4) + \
                stats.poisson.logpmf(Y[t, 1, j], np.exp(0.2 * x[0] + 0.3 + z))
            assert abs(ob - PS[t, 1, j]) < 1e-11 * max(1.0, abs(ob))
    same = slds_model(same=True)
    lg = gen.LinearGaussianSSM(same.A[0], same.Q[0], np.eye(2), 0.3 * np.eye(2), same.mu0, same.P0, b=same.b[0])
    _, ys = same.simulate(15, np.random.default_rng(7))
    exact = lg.kalman_log_marginal([v["y"] for v in ys])
    est = [O.run_pf(same, ys, 20000, s).log_ml_estimate() for s in (1, 2)]
    assert all(abs(e - exact) < 0.25 for e in est), (est, exact)


def test_oracle_dependent_slots_scores_equal_reference_densities():
    """Observed addresses depending on earlier ones in the step: simulate's
    observation column is the sum of the reference densities with each
    child's linear predictor shifted by g x its parents' values; with every
    coefficient 0 the model filters as the one without dependencies, bit for
    bit; a step constraining a child without its parent is refused on the
    host side (the oracle's weights turn NaN)."""
    m = dep_model()
    T, n = 5, 64
    X, Y, PS, _ = O.simulate(m, T, n, 3)
    for t in range(T):
        for j in range(n):
            x = X[t, :, j]
            yv = {name: Y[t, k, j] for k, name in enumerate(m.names)}
            ref = sum(m.slot_logpdf(k, Y[t, k, j], x, yv) for k in range(4))
            assert abs(ref - PS[t, 1, j]) < 1e-10 * max(1.0, abs(ref)), (t, j, ref, PS[t, 1, j])
    flat = dep_model(g=(0.0, 0.0, 0.0, 0.0))
    plain = gen.SlotSSM(_LAT2, [{k: v for k, v in sl.items() if k != "parents"} for sl in
                                [{"name": "a", "dist": "normal", "h": [1.0, 0.0], "c": 0.0, "sd": 0.5},
                                 {"name": "n", "dist": "poisson", "h": [0.5, 0.2], "c": 0.1},
                                 {"name": "b", "dist": "bernoulli", "h": [0.0, 1.0], "c": 0.0},
                                 {"name": "g", "dist": "gamma", "args": [_arg("exp", [0.2, 0.0], 0.1), 1.5]}]])
    _, obs = dep_obs()
    a = O.run_pf(flat, obs, 500, 4)
    b = O.run_pf(plain, obs, 500, 4)
    assert np.array_equal(a.state(), b.state()) and np.array_equal(a.log_weights(), b.log_weights())
    pf = O.OraclePF(m, 50, 1)
    pf.init({"n": 2.0})  # the count without the reading it depends on
    assert np.all(np.isnan(pf.log_weights()))
    with pytest.raises(ValueError):
        gen.SlotSSM(_LAT2, [{"name": "n", "dist": "poisson", "h": [0.0, 0.0], "c": 0.0, "parents": {"a": 1.0}},
                            {"name": "a", "dist": "normal", "h": [1.0, 0.0], "c": 0.0, "sd": 0.5}])


def test_slot_model_rejects_bad_descriptions():
    with pytest.raises(ValueError):
        gen.SlotSSM({"form": "affine", "A": np.eye(2), "Q": np.eye(2), "mu0": np.zeros(2), "P0": np.eye(2)},
                    [{"name": "y", "dist": "gamma"}])
    with pytest.raises(ValueError):  # (gamma takes two arguments)
        gen.SlotSSM(_LAT2, [{"name": "y", "dist": "gamma", "args": [1.0]}])
    with pytest.raises(ValueError):
        gen.SlotSSM(_LAT2, [{"name": "y", "dist": "dirichlet", "args": [1.0]}])
    m = count_model()
    with pytest.raises(gen.GenHipError):
        m.gh_obs({"nope": 1.0})
    # an address that is not a slot of the step is a discard (particle_filter.jl:168-170)
    with pytest.raises(gen.GenHipError):
        m.obs_from_choicemap(gen.ChoiceMap({("chain", 2, "count"): 1.0, ("chain", 3, "count"): 2.0}), 2)


# ------------------------------------------- the linear custom proposal (CPU)
def _flat(*a):
    return np.concatenate([np.asarray(x, dtype=np.float64).ravel() for x in a])


def _count_obs_lpdf(m, x, y):
    """The count model's observed-slot logpdfs at latent x for the present
    slots of y (the reference's closed forms; scipy where it has them)."""
    from scipy import stats

    s, tot = m.slots, 0.0
    for k, sl in enumerate(s):
        if sl["name"] not in y:
            continue
        v = y[sl["name"]]
        if sl["dist"] == "categorical":
            logits = np.asarray(sl["W"]) @ x + np.asarray(sl["c"])
            tot += logits[int(v)] - logits.max() - np.log(np.exp(logits - logits.max()).sum())
            continue
        eta = float(np.dot(sl["h"], x) + sl["c"])
        if sl["dist"] == "poisson":
            tot += stats.poisson.logpmf(v, np.exp(eta))
        elif sl["dist"] == "normal":
            tot += stats.norm.logpdf(v, eta, sl["sd"])
        else:
            tot += stats.bernoulli.logpmf(v, 1.0 / (1.0 + np.exp(-eta)))
    return tot


def test_oracle_slot_linear_proposal_weights():
    """GH_PROPOSAL_LINEAR on a slot model: q = mvnormal(P x_{t-1} + u_t,
    Sigma_q); weight = log p(x_t | x_{t-1}) + sum of the present slots'
    logpdfs - log q(x_t) (particle_filter.jl:79-91,139-154 via
    trace_translators.jl:775-802) against scipy."""
    from scipy import stats

    m, obs = count_obs()
    n = 200
    P, S, u1, u2 = 0.6 * m.A, np.array([[0.08, 0.01], [0.01, 0.06]]), np.array([0.4, 0.1]), np.array([-0.2, 0.3])
    pf = O.OraclePF(m, n, 3)
    pf.set_proposal_args(_flat(P, S, u1))
    pf.init(obs[0], O.LINEAR)
    x1 = pf.state().copy()
    w1 = np.array([stats.multivariate_normal.logpdf(x1[:, i], m.mu0, m.P0) + _count_obs_lpdf(m, x1[:, i], obs[0])
                   - stats.multivariate_normal.logpdf(x1[:, i], u1, S) for i in range(n)])
    np.testing.assert_allclose(pf.log_weights(), w1, rtol=1e-11, atol=1e-10)
    pf.set_proposal_args(u2)  # u alone: P and Sigma_q kept
    pf.maybe_resample(0.0)
    pf.step(obs[1], O.LINEAR)
    x2 = pf.state()
    w2 = w1 + np.array([stats.multivariate_normal.logpdf(x2[:, i], m.A @ x1[:, i] + m.b, m.Q)
                        + _count_obs_lpdf(m, x2[:, i], obs[1])
                        - stats.multivariate_normal.logpdf(x2[:, i], P @ x1[:, i] + u2, S) for i in range(n)])
    np.testing.assert_allclose(pf.log_weights(), w2, rtol=1e-11, atol=1e-9)


def test_oracle_slot_prior_as_linear_proposal_is_the_bootstrap_filter():
    """q = the prior (P = A, u = b, Sigma_q = Q; t = 1: mu0, P0) draws the
    bootstrap filter's latents and weighs them to rounding."""
    m, obs = count_obs()
    n = 400
    boot = O.run_pf(m, obs, n, 9, thr=0.0)
    pf = O.OraclePF(m, n, 9)
    pf.set_proposal_args(_flat(m.A, m.P0, m.mu0))
    pf.init(obs[0], O.LINEAR)
    pf.set_proposal_args(_flat(m.A, m.Q, m.b))
    for y in obs[1:]:
        pf.maybe_resample(0.0)
        pf.step(y, O.LINEAR)
    np.testing.assert_allclose(pf.state(), boot.state(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(pf.log_weights(), boot.log_weights(), rtol=1e-10, atol=1e-9)


def test_oracle_slot_step_params():
    """A parameter change on a slot model (orc_pf_step_params): to the same
    numbers it is the plain step bit for bit; a model with another slot
    layout is refused."""
    m, obs = count_obs()
    runs = []
    for change in (False, True):
        pf = O.OraclePF(m, 500, 4)
        pf.init(obs[0])
        for t in range(2, 7):
            pf.maybe_resample(None)
            if change and t == 5:
                pf.step_params(count_model(), obs[t - 1])
            else:
                pf.step(obs[t - 1])
        runs.append(pf)
    assert np.array_equal(runs[0].log_weights(), runs[1].log_weights())
    assert np.array_equal(runs[0].state(), runs[1].state())
    other = gen.SlotSSM({"form": "affine", "A": m.A, "b": m.b, "Q": m.Q, "mu0": m.mu0, "P0": m.P0},
                        [{"name": "count", "dist": "poisson", "h": [1.0, 0.5], "c": 0.2}])
    with pytest.raises(ValueError):
        runs[0].step_params(other, {"count": 1.0})


def _with_input(y, u):
    y = dict(y)
    if u is not None:
        y["__input__"] = u
    return y


def test_oracle_slot_zero_inputs_are_the_plain_model():
    """A model with per-step inputs given none (or zeros) filters as the model
    without inputs, bit for bit; with inputs, each state moves by its step's
    input (the same normals) and the latent score is mvnormal(A x + b + u, Q)."""
    from scipy import stats

    m, obs = count_obs()
    mi = count_model_inputs()
    a = O.run_pf(m, obs, 400, 7, thr=0.0)
    b = O.run_pf(mi, obs, 400, 7, thr=0.0)
    c = O.run_pf(mi, [_with_input(y, np.zeros(2)) for y in obs], 400, 7, thr=0.0)
    for r in (b, c):
        assert np.array_equal(a.state(), r.state()) and np.array_equal(a.log_weights(), r.log_weights())
        for x, y in zip(a.scores(per_step=True), r.scores(per_step=True)):
            assert np.array_equal(x, y)
    u = count_inputs()
    # step 2: x2 = A x1 + (b + u2) + L z with the plain model's normals z
    pc, pd = O.OraclePF(m, 300, 4), O.OraclePF(mi, 300, 4)
    pc.init(obs[0])
    pd.init(obs[0])
    x1 = pd.state().copy()
    pc.maybe_resample(0.0)
    pd.maybe_resample(0.0)
    pc.step(obs[1])
    pd.step(_with_input(obs[1], u[1]))
    np.testing.assert_allclose(pd.state() - pc.state(), np.repeat(u[1][:, None], 300, axis=1), atol=1e-12)
    _, ps = pd.scores(per_step=True)
    x2 = pd.state()
    ref = [stats.multivariate_normal.logpdf(x2[:, i], m.A @ x1[:, i] + m.b + u[1], m.Q) for i in range(300)]
    np.testing.assert_allclose(ps[1, 0], ref, rtol=1e-12, atol=1e-10)


def test_oracle_hmm_as_slots_matches_reference_forward_algorithm():
    """The categorical latent pinned to the reference's HMM test
    (test/inference/particle_filter.jl:96-168): the HMM written as a slot model
    (categorical latent, one categorical emission slot with W = log E, so
    softmax(W[:, z]) = E[:, z]) draws the HMM family's latents (no
    resampling: the same states) and its log-ML at the reference's N is within
    the reference's atol of the exact forward algorithm."""
    import json

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "hmm.json")))["pf_test"]
    E = np.array(g["emission"])
    hmm = gen.DiscreteHMM(g["prior"], np.array(g["transition"]), E)
    sl = gen.SlotSSM({"form": "categorical", "prior": g["prior"], "T": g["transition"]},
                     [{"name": "x", "dist": "categorical", "W": np.log(E), "c": np.zeros(E.shape[0])}])
    obs = g["obs"]
    a = O.run_pf(hmm, [[o] for o in obs], 2000, 3, thr=0.0)
    b = O.run_pf(sl, [{"x": float(o)} for o in obs], 2000, 3, thr=0.0)
    assert np.array_equal(np.argmax(b.state(), axis=0), a.state()[0].astype(int))
    np.testing.assert_allclose(b.log_weights(), a.log_weights(), rtol=1e-12, atol=1e-12)
    pf = O.run_pf(sl, [{"x": float(o)} for o in obs], g["num_particles"], 0, thr=g["ess_threshold"])
    assert abs(pf.log_ml_estimate() - g["log_ml"]) < g["atol"]
    _, ps = b.scores(per_step=True)
    _, ps_h = a.scores(per_step=True)
    np.testing.assert_allclose(ps[:, 0], ps_h[:, 0], rtol=0, atol=0)  # log prior / log T: identical


def test_oracle_simulate_with_inputs_moves_the_latents():
    """simulate(model, (T, U)) of a model with per-step inputs: zero inputs
    reproduce the plain model's traces bit for bit; each step's latent moves
    by its input (the same normals) and scores as mvnormal(A x + b + u, Q)."""
    from scipy import stats

    m, mi = count_model(), count_model_inputs()
    T, n = 5, 200
    X0, Y0, P0, _ = O.simulate(m, T, n, 9)
    Xz, Yz, Pz, _ = O.simulate(mi, T, n, 9, inputs=np.zeros((T, 2)))
    assert np.array_equal(X0, Xz) and np.array_equal(Y0, Yz) and np.array_equal(P0, Pz)
    U = np.zeros((T, 2))
    U[1] = [0.5, -0.3]
    X1, _, P1, _ = O.simulate(mi, T, n, 9, inputs=U)
    np.testing.assert_allclose(X1[1] - X0[1], np.repeat(U[1][:, None], n, axis=1), atol=1e-12)
    ref = [stats.multivariate_normal.logpdf(X1[1, :, j], m.A @ X1[0, :, j] + m.b + U[1], m.Q) for j in range(n)]
    np.testing.assert_allclose(P1[1, 0], ref, rtol=1e-12, atol=1e-10)
    with pytest.raises(ValueError):  # (the inputs are required arguments)
        O.simulate(mi, T, n, 9)


# ------------------------------------------------------------------ GPU
def _gpu_run(model, obs, n, seed, batched, thr=None, rejuv=0):
    st = gen.initialize_particle_filter(model, (1,), _obs_at(model, obs[0], 1), n, seed=seed)
    if rejuv:
        gen.rejuvenate(st, rejuv)
    if batched:
        gen.run_particle_filter(st, list(obs[1:]), thr)
    else:
        for t in range(2, len(obs) + 1):
            gen.maybe_resample(st, thr)
            gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), _obs_at(model, obs[t - 1], t))
            if rejuv:
                gen.rejuvenate(st, rejuv)
    return st


def _orc_run(model, obs, n, seed, thr=None, rejuv=0):
    pf = O.OraclePF(model, n, seed)
    pf.init(obs[0])
    if rejuv:
        pf.rejuvenate(rejuv)
    for y in obs[1:]:
        pf.maybe_resample(thr)
        pf.step(y)
        if rejuv:
            pf.rejuvenate(rejuv)
    return pf


def _same(st, ref_st=None, orc=None):
    if ref_st is not None:
        assert np.array_equal(st.states(), ref_st.states())
        assert np.array_equal(st.parents, ref_st.parents)
        assert np.array_equal(gen.get_log_weights(st), gen.get_log_weights(ref_st))
        assert gen.log_ml_estimate(st) == gen.log_ml_estimate(ref_st)
    if orc is not None:
        assert np.array_equal(st.states().T, orc.state())
        assert np.array_equal(st.parents, orc.parents())
        assert np.array_equal(gen.get_log_weights(st), orc.log_weights())
        a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
        assert abs(a - b) <= 1e-9 * abs(b), (a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("d", [4, 10])
def test_gpu_lgssm_as_slots_equals_family_bitexact(gh_ctx, d, batched):
    """The C2 model (and d = 4) written as slots filters as the LGSSM family
    (LGModel<D, 3>, the benchmark's structured kernel) does: bit for bit."""
    lg = gen.LinearGaussianSSM.benchmark(d)
    _, ys = lg.simulate(12, np.random.default_rng(2))
    n = 20011
    a = _gpu_run(lg, list(ys), n, 9, batched)
    b = _gpu_run(lg_as_slots(lg), [{"y": y} for y in ys], n, 9, batched)
    _same(b, ref_st=a)
    for x, y in zip(gen.get_traces(a).scores(per_step=True), gen.get_traces(b).scores(per_step=True)):
        assert np.array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [False, True])
def test_gpu_kitagawa_as_slots_equals_family_bitexact(gh_ctx, batched):
    """The nonlinear SSM written as slots (Kitagawa latent, normal slot with
    the x^2/20 mean) equals the Kitagawa family (whose default step is the pair
    kernel) bit for bit."""
    kit = gen.KitagawaSSM(4.0, 1.0)
    _, ys = kit.simulate(15, np.random.default_rng(3))
    n = 1 << 15
    a = _gpu_run(kit, list(ys), n, 9, batched)
    b = _gpu_run(kit_as_slots(kit), [{"y": y} for y in ys], n, 9, batched)
    _same(b, ref_st=a)


@pytest.mark.gpu
@pytest.mark.parametrize("batched,thr,rejuv", [(False, None, 0), (True, None, 0), (False, 1e9, 2), (True, 0.0, 0)])
def test_gpu_count_ssm_slots_equal_oracle_bitexact(gh_ctx, batched, thr, rejuv):
    """A Poisson-count SSM with normal, bernoulli and categorical addresses,
    steps constraining every subset used (one step none): GPU == oracle bit
    for bit (states, weights, parents; log-ML 1e-9), with rejuvenation moves
    (mh(trace, select(:x)) per particle) in one case."""
    m, obs = count_obs()
    n = 4099
    st = _gpu_run(m, obs, n, 13, batched, thr, rejuv)
    orc = _orc_run(m, obs, n, 13, thr, rejuv)
    _same(st, orc=orc)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    # a trace's choices: every latent and every constrained slot
    cm = gen.get_traces(st)[0].get_choices()
    assert cm[("chain", 1, "count")] == obs[0]["count"] and ("chain", 3, "z") not in dict(cm)


@pytest.mark.gpu
def test_gpu_slots_simulate_equals_oracle_bitexact(gh_ctx):
    for m in (count_model(), lg_as_slots(gen.LinearGaussianSSM.benchmark(3)),
              kit_as_slots(gen.KitagawaSSM(4.0, 1.0))):
        tr = gen.simulate(m, (6,), num_traces=777, seed=21)
        X, Y, PS, TOT = O.simulate(m, 6, 777, 21)
        assert np.array_equal(tr.xs, X) and np.array_equal(tr.ys, Y)
        assert np.array_equal(tr.per_step, PS) and np.array_equal(tr.total, TOT)


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [False, True])
def test_gpu_stochastic_volatility_slots_equal_oracle_bitexact(gh_ctx, batched):
    """Normal slots with a log-linear standard deviation (the stochastic-
    volatility emission): GPU == oracle bit for bit (states, weights, parents,
    score columns; log-ML 1e-9), some steps constraining one slot or none;
    simulate bit-exact too."""
    m, obs = sv_obs()
    n = 6151
    st = _gpu_run(m, obs, n, 17, batched)
    orc = _orc_run(m, obs, n, 17)
    _same(st, orc=orc)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    tr = gen.simulate(m, (7,), num_traces=999, seed=23)
    X, Y, PS, TOT = O.simulate(m, 7, 999, 23)
    assert np.array_equal(tr.xs, X) and np.array_equal(tr.ys, Y)
    assert np.array_equal(tr.per_step, PS) and np.array_equal(tr.total, TOT)


@pytest.mark.gpu
@pytest.mark.parametrize("name,batched", [("m1", False), ("m1", True), ("m2", True), ("m3", True), ("m4", False)])
def test_gpu_library_slots_equal_oracle_bitexact(gh_ctx, name, batched):
    """Library slots (gamma, neg_binom, laplace, beta / exponential, binom,
    geometric, cauchy / normal, uniform, inv_gamma, uniform_discrete / poisson,
    bernoulli, beta_uniform, arguments linked to the latent): GPU == oracle bit
    for bit (states, weights, parents, score columns; log-ML 1e-9), and
    simulate (the device samplers) bit-exact."""
    m, obs = library_obs(name)
    n = 3001
    st = _gpu_run(m, obs, n, 19, batched)
    orc = _orc_run(m, obs, n, 19)
    _same(st, orc=orc)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    tr = gen.simulate(m, (5,), num_traces=513, seed=29)
    X, Y, PS, TOT = O.simulate(m, 5, 513, 29)
    assert np.array_equal(tr.xs, X) and np.array_equal(tr.ys, Y)
    assert np.array_equal(tr.per_step, PS) and np.array_equal(tr.total, TOT)


@pytest.mark.gpu
@pytest.mark.parametrize("batched,rejuv", [(False, 0), (True, 0), (False, 2)])
def test_gpu_switching_latent_bitexact(gh_ctx, batched, rejuv):
    """A switching linear dynamical system (two latent addresses per step):
    GPU == oracle bit for bit (states, weights, parents, score columns;
    log-ML 1e-9), with rejuvenation moves of the whole latent in one case;
    the traces name both addresses; simulate bit-exact."""
    m, obs = slds_obs()
    n = 4097
    st = _gpu_run(m, obs, n, 23, batched, None, rejuv)
    orc = _orc_run(m, obs, n, 23, None, rejuv)
    _same(st, orc=orc)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    tr = gen.get_traces(st)
    cm = dict(tr[5].get_choices())
    z, x = cm[("chain", 3, "z")], cm[("chain", 3, "x")]
    assert z in (0, 1) and np.asarray(x).shape == (2,)
    assert np.array_equal(tr.column(("chain", 3, "z")), np.argmax(st.states(3)[:, 2:], axis=1))
    sim = gen.simulate(m, (6,), num_traces=321, seed=31)
    X, Y, PS, TOT = O.simulate(m, 6, 321, 31)
    assert np.array_equal(sim.xs, X) and np.array_equal(sim.ys, Y)
    assert np.array_equal(sim.per_step, PS) and np.array_equal(sim.total, TOT)


@pytest.mark.gpu
@pytest.mark.parametrize("batched,rejuv", [(False, 0), (True, 0), (False, 2)])
def test_gpu_dependent_slots_bitexact(gh_ctx, batched, rejuv):
    """Dependent observed addresses (normal -> Poisson -> Bernoulli, Poisson
    -> gamma library slot), steps leaving children out: GPU == oracle bit for
    bit (states, weights, parents, score columns; log-ML 1e-9), with
    rejuvenation moves in one case (the likelihood evaluated repeatedly in one
    launch), simulate bit-exact (a fixed-sd normal slot after a library slot,
    over several steps); a step constraining a child without its parent is
    refused."""
    m, obs = dep_obs()
    n = 4093
    st = _gpu_run(m, obs, n, 27, batched, None, rejuv)
    orc = _orc_run(m, obs, n, 27, None, rejuv)
    _same(st, orc=orc)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    sim = gen.simulate(m, (6,), num_traces=257, seed=37)
    X, Y, PS, TOT = O.simulate(m, 6, 257, 37)
    assert np.array_equal(sim.xs, X) and np.array_equal(sim.ys, Y)
    assert np.array_equal(sim.per_step, PS) and np.array_equal(sim.total, TOT)
    with pytest.raises(gen.GenHipError):
        gen.initialize_particle_filter(m, (1,), _obs_at(m, {"n": 2.0}, 1), 64, seed=1)


@pytest.mark.gpu
def test_gpu_slots_constrained_twice_is_discard(gh_ctx):
    """A step's chain naming one slot twice is rejected (GH_E_DISCARD)."""
    import ctypes

    from gen_amd import _lib

    m = count_model()
    ctx = gen.get_default_context() if hasattr(gen, "get_default_context") else None
    h = ctypes.c_void_p()
    desc, keep = m.desc()
    lib = _lib.load()
    _lib.check(lib.gh_model_create(gh_ctx.h, ctypes.byref(desc), ctypes.byref(h)))
    v = np.array([1.0])
    chain = (_lib.Obs * 2)()
    chain[0] = _lib.Obs(_lib.dptr(v), 1, 1, 0, 0, None)
    chain[1] = _lib.Obs(_lib.dptr(v), 1, 1, 0, 0, None)
    chain[0].next = ctypes.pointer(chain[1])
    opts = _lib.PFOpts()
    lib.gh_pf_opts_default(ctypes.byref(opts))
    pf = ctypes.c_void_p()
    rc = lib.gh_pf_init(h, ctypes.byref(chain[0]), 0, 1024, 1, ctypes.byref(opts), ctypes.byref(pf))
    assert rc == 2, rc  # GH_E_DISCARD
    lib.gh_model_destroy(h)
    del ctx, keep


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["count", "kit"])
def test_gpu_slot_linear_proposal_bitexact(gh_ctx, name):
    """The linear custom proposal on slot models (an affine latent with four
    observed addresses; the Kitagawa latent with its x^2/20 slot), arguments
    changing between steps (full and u-only), resampling on some steps:
    states, weights, parents and score columns bit-exact against the oracle."""
    if name == "count":
        m, obs = count_obs()
        d = 2
    else:
        kit = gen.KitagawaSSM(4.0, 1.0)
        m = kit_as_slots(kit)
        _, ys = kit.simulate(9, np.random.default_rng(3))
        obs = [{"y": y} for y in ys]
        obs[3] = {}
        d = 1
    rng = np.random.default_rng(8)

    def full(t):
        G = rng.standard_normal((d, d))
        return _flat(0.5 * np.eye(d) + 0.05 * rng.standard_normal((d, d)), 0.1 * np.eye(d) + 0.02 * G @ G.T,
                     0.3 * rng.standard_normal(d))

    n, seed = 6007, 19
    a0 = full(1)
    st = gen.initialize_particle_filter(m, (1,), _obs_at(m, obs[0], 1), gen.LinearGaussianProposal, (a0,), n,
                                        seed=seed)
    orc = O.OraclePF(m, n, seed)
    orc.set_proposal_args(a0)
    orc.init(obs[0], O.LINEAR)
    for t in range(2, len(obs) + 1):
        thr = n if t % 3 else None
        assert gen.maybe_resample(st, thr) == orc.maybe_resample(thr)[0]
        args = full(t) if t % 2 == 0 else full(t)[-d:]
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), _obs_at(m, obs[t - 1], t),
                                 gen.LinearGaussianProposal, (args,))
        orc.set_proposal_args(args)
        orc.step(obs[t - 1], O.LINEAR)
        assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64)), t
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(st.parents, orc.parents()), t
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * abs(b)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    st.close()


@pytest.mark.gpu
def test_gpu_slot_step_params_bitexact(gh_ctx):
    """particle_filter_step with new_args = (t, model') on a slot model
    (gh_pf_step_params: every particle re-scored along its genealogy under the
    new numbers, then the step under them) and later steps: states, weights,
    parents, log-ML and score columns bit-exact against the oracle; a model
    with another slot layout is refused."""
    m, obs = count_obs()
    m2 = changed_count_model()
    n, seed, K = 5003, 21, 5
    st = gen.initialize_particle_filter(m, (1,), _obs_at(m, obs[0], 1), n, seed=seed)
    orc = O.OraclePF(m, n, seed)
    orc.init(obs[0])
    for t in range(2, len(obs) + 1):
        assert gen.maybe_resample(st, None) == orc.maybe_resample(None)[0]
        if t == K:
            gen.particle_filter_step(st, (t, m2), (gen.UnknownChange(), gen.UnknownChange()), _obs_at(m2, obs[t - 1], t))
            orc.step_params(m2, obs[t - 1])
        else:
            mt = m2 if t > K else m
            gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), _obs_at(mt, obs[t - 1], t))
            orc.step(obs[t - 1])
        assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64)), t
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(st.parents, orc.parents()), t
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * abs(b)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    other = gen.SlotSSM({"form": "affine", "A": m.A, "b": m.b, "Q": m.Q, "mu0": m.mu0, "P0": m.P0},
                        [{"name": "count", "dist": "poisson", "h": [1.0, 0.5], "c": 0.2}])
    t = len(obs) + 1
    with pytest.raises(gen.GenHipError):
        gen.particle_filter_step(st, (t, other), (gen.UnknownChange(), gen.UnknownChange()),
                                 {("chain", t, "count"): 1.0})
    st.close()


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [None, 1e9])
def test_gpu_slot_conditional_smc_bitexact(gh_ctx, thr):
    """Conditional SMC (examples/pmmh/smc.jl:100-151) on the count SSM:
    particle 0 pinned to a reference trajectory, the others resampled
    multinomially — states, weights, parents and trajectories bit-exact
    against the oracle's conditional run."""
    m, obs = count_obs()
    xs, _ = m.simulate(len(obs), np.random.default_rng(5))
    ref = np.asarray(xs, dtype=np.float64).reshape(len(obs), -1) * 0.9
    n, seed = 3001, 17
    st = gen.initialize_conditional_particle_filter(m, (1,), _obs_at(m, obs[0], 1), n, ref[0], seed=seed)
    orc = O.OraclePF(m, n, seed, O.MULTINOMIAL)
    orc.init_conditional(obs[0], ref[0])
    for t in range(2, len(obs) + 1):
        assert gen.maybe_resample(st, thr) == orc.maybe_resample(thr)[0]
        gen.conditional_particle_filter_step(st, (t,), (gen.UnknownChange(),), _obs_at(m, obs[t - 1], t), ref[t - 1])
        orc.step_conditional(obs[t - 1], ref[t - 1])
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64)), t
        assert np.array_equal(st.parents, orc.parents()), t
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * abs(b)
    T = len(obs)
    for t in (1, T // 2, T):
        assert np.array_equal(st.states(t).T, orc.trajectory(t)), t
    assert np.array_equal(np.stack([st.states(t)[0] for t in range(1, T + 1)]), ref)
    st.close()


@pytest.mark.gpu
@pytest.mark.parametrize("batched,linear", [(False, False), (True, False), (False, True)])
def test_gpu_slot_inputs_bitexact(gh_ctx, batched, linear):
    """Per-step inputs of a slot model (new_args = (t, u_t); run_particle_filter's
    inputs_per_step), some steps without one, with the default and the linear
    custom proposal (whose mean offset follows the input): states, weights,
    parents and score columns bit-exact against the oracle; an input to a
    model without inputs and simulate of an input model are refused."""
    mi = count_model_inputs()
    _, obs = count_obs()
    u = count_inputs()
    n, seed = 4099, 23
    q = (np.concatenate([(0.6 * mi.A).ravel(), (0.5 * mi.Q).ravel(), [0.1, -0.2]]),) if linear else ()
    prop = gen.LinearGaussianProposal if linear else None
    st = gen.initialize_particle_filter(mi, (1,), _obs_at(mi, obs[0], 1), *((prop, q) if linear else ()), n,
                                        seed=seed)
    orc = O.OraclePF(mi, n, seed)
    if linear:
        orc.set_proposal_args(q[0])
    orc.init(obs[0], O.LINEAR if linear else O.DEFAULT)
    if batched:
        gen.run_particle_filter(st, list(obs[1:]), None, inputs_per_step=u[1:])
        for t in range(2, len(obs) + 1):
            orc.maybe_resample(None)
            orc.step(_with_input(obs[t - 1], u[t - 1]))
    else:
        for t in range(2, len(obs) + 1):
            assert gen.maybe_resample(st, None) == orc.maybe_resample(None)[0]
            na = (t,) if u[t - 1] is None else (t, u[t - 1])
            gen.particle_filter_step(st, na, (gen.UnknownChange(),) * len(na), _obs_at(mi, obs[t - 1], t),
                                     *((prop, ()) if linear else ()))
            orc.step(_with_input(obs[t - 1], u[t - 1]), O.LINEAR if linear else O.DEFAULT)
            assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
    assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64))
    assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    assert np.array_equal(st.parents, orc.parents())
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * abs(b)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    st.close()
    m = count_model()
    st2 = gen.initialize_particle_filter(m, (1,), _obs_at(m, obs[0], 1), 1000, seed=1)
    with pytest.raises(gen.GenHipError):  # (the plain model takes no input: new_args[1] must be a model)
        gen.particle_filter_step(st2, (2, np.zeros(2)), (gen.UnknownChange(),) * 2, _obs_at(m, obs[1], 2))
    st2.close()
    with pytest.raises(gen.GenHipError):  # (its inputs are arguments: simulate(model, (T, U)))
        gen.simulate(mi, (4,), num_traces=10, seed=1)
    U = np.stack([np.zeros(2) if v is None else v for v in u])
    tr = gen.simulate(mi, (len(u), U), num_traces=777, seed=5)
    X, Y, PS, TOT = O.simulate(mi, len(u), 777, 5, inputs=U)
    assert np.array_equal(tr.xs, X) and np.array_equal(tr.ys, Y)
    assert np.array_equal(tr.per_step, PS) and np.array_equal(tr.total, TOT)


@pytest.mark.gpu
@pytest.mark.parametrize("batched,rejuv", [(False, 0), (True, 0), (False, 2)])
def test_gpu_categorical_latent_bitexact(gh_ctx, batched, rejuv):
    """A switching model (categorical latent, four per-class emission slots,
    some steps constraining a subset): states (one-hot), weights, parents,
    score columns and simulate bit-exact against the oracle; the trace's latent
    choice is the class index; a Gaussian drift and the linear proposal are
    refused for it."""
    m = switching_model()
    xs, ys = m.simulate(9, np.random.default_rng(4))
    obs = [dict(y) for y in ys]
    del obs[2]["count"]
    obs[5] = {}
    n, seed = 5003, 29
    st = _gpu_run(m, obs, n, seed, batched, None, rejuv)
    orc = _orc_run(m, obs, n, seed, None, rejuv)
    _same(st, orc=orc)
    tot, ps = gen.get_traces(st).scores(per_step=True)
    otot, ops = orc.scores(per_step=True)
    assert np.array_equal(tot, otot) and np.array_equal(ps, ops)
    z = gen.get_traces(st)[0].get_choices()[("chain", 3, "x")]
    assert isinstance(z, int) and 0 <= z < 3
    assert np.array_equal(gen.get_traces(st).column(("chain", 3, "x")), np.argmax(st.states(3), axis=1))
    with pytest.raises(gen.GenHipError):
        gen.mh(st, gen.gaussian_drift, (gen.select(m.latent_address(len(obs))), [0.1, 0.1, 0.1]))
    st.close()
    with pytest.raises(gen.GenHipError):
        gen.initialize_particle_filter(m, (1,), _obs_at(m, obs[0], 1), gen.LinearGaussianProposal,
                                       (np.zeros(3 * 3 * 2 + 3),), 100, seed=1)
    tr = gen.simulate(m, (6,), num_traces=555, seed=8)
    X, Y, PS, TOT = O.simulate(m, 6, 555, 8)
    assert np.array_equal(tr.xs, X) and np.array_equal(tr.ys, Y)
    assert np.array_equal(tr.per_step, PS) and np.array_equal(tr.total, TOT)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["count", "switch"])
def test_gpu_slot_models_full_size_bitexact(gh_ctx, name):
    """Slot models at the C2 size (2^20 particles, the batched loop with the
    one-launch resample at ESS < N/2): final states, weights and parents
    bit-exact against the oracle's OpenMP build."""
    if name == "count":
        m, obs = count_obs(T=8)
    else:
        m = switching_model()
        _, ys = m.simulate(8, np.random.default_rng(6))
        obs = [dict(y) for y in ys]
    n = 1 << 20
    st = gen.initialize_particle_filter(m, (1,), _obs_at(m, obs[0], 1), n, seed=42)
    gen.run_particle_filter(st, list(obs[1:]))
    O.set_openmp(True)
    try:
        orc = O.run_pf(m, obs, n, 42, record_history=False)
    finally:
        O.set_openmp(False)
    _, did = st.ess_history()
    assert did.sum() >= 1
    assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64))
    assert np.array_equal(st.parents, orc.parents())
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * abs(b)
    st.close()
