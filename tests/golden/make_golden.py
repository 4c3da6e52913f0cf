"""Generate the golden vectors under tests/golden/ (numpy only, no reference code).

Each fixture restates an assertion of the reference's own test-suite, or an
analytic oracle of the same kind, as data:

  philox_kat.json   Philox4x32-10 known-answer vectors (Salmon et al. SC'11,
                    Random123 kat_vectors): the RNG every sampling path uses.
  hmm.json          test/inference/particle_filter.jl: the hand-enumerated
                    forward-algorithm KAT (:29-48) and the PF test model
                    (:52-81) with its exact log marginal likelihood.
  unfold_kats.json  test/modeling_library/unfold.jl:116-481: the closed-form
                    update/regenerate weights and scores of the linear-Gaussian
                    Unfold kernel x ~ normal(x_prev*alpha + beta, 1) (:5-8),
                    evaluated with normal.jl:56-60's formula.
  kalman.json       exact Kalman-filter log-ML of seeded LG-SSMs (the PF's
                    analytic oracle for the C2 workload).

Run: python tests/golden/make_golden.py
"""
import json
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def normal_logpdf(x, mu, std):
    # src/modeling_library/distributions/normal.jl:56-60
    var = std * std
    diff = x - mu
    return -(diff * diff) / (2.0 * var) - 0.5 * math.log(2.0 * math.pi * var)


def hmm_forward(prior, E, T, obs):
    # test/inference/particle_filter.jl:1-27 (0-based symbols here)
    ml = 1.0
    alpha = np.asarray(prior, dtype=float)
    for i in range(1, len(obs)):
        pp = alpha * E[obs[i - 1], :]
        den = pp.sum()
        pp = pp / den
        alpha = T @ pp
        ml *= den
    pp = alpha * E[obs[-1], :]
    ml *= pp.sum()
    return ml


def philox_kat():
    return {
        "vectors": [
            {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
            {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2, "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
            {
                "ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                "key": [0xA4093822, 0x299F31D0],
                "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1],
            },
        ]
    }


def hmm():
    # hand enumeration KAT, particle_filter.jl:32-46 (Julia obs [2,1] -> 0-based [1,0])
    prior = [0.4, 0.6]
    E = np.array([[0.1, 0.9], [0.7, 0.3]]).T
    T = np.array([[0.5, 0.5], [0.2, 0.8]]).T
    obs = [1, 0]
    exp = 0.0
    for z1 in range(2):
        for z2 in range(2):
            exp += prior[z1] * T[z2, z1] * E[obs[0], z1] * E[obs[1], z2]
    kat = {"prior": prior, "emission": E.tolist(), "transition": T.tolist(), "obs": obs, "marg_lik": exp}
    # the PF test model, particle_filter.jl:52-81 (obs_x [1,1,2,3] -> [0,0,1,2])
    prior = [0.2, 0.3, 0.5]
    E = np.array([[0.1, 0.2, 0.7], [0.2, 0.7, 0.1], [0.7, 0.2, 0.1]]).T
    T = np.array([[0.4, 0.4, 0.2], [0.2, 0.3, 0.5], [0.9, 0.05, 0.05]]).T
    obs = [0, 0, 1, 2]
    pf = {
        "prior": prior,
        "emission": E.tolist(),
        "transition": T.tolist(),
        "obs": obs,
        "log_ml": math.log(hmm_forward(prior, E, T, obs)),
        "num_particles": 10000,
        "ess_threshold": 10000,
        "atol": 0.01,
    }
    return {"forward_kat": kat, "pf_test": pf}


def unfold_kats():
    s = 1.0
    x_init, alpha, beta, x1, x2 = 0.1, 0.2, 0.3, 1.1, 1.2
    lp = normal_logpdf
    cases = {}
    # generate with constraints on 1 and 3 (unfold.jl:44-72): x2 free -> weight depends on x2
    # update case 1 (unfold.jl:131-166)
    x2n, x3n, an = 1.3, 1.4, 0.5
    cases["update_extend_change"] = {
        "score": lp(x1, x_init * an + beta, s) + lp(x2n, x1 * an + beta, s) + lp(x3n, x2n * an + beta, s),
        "weight": lp(x3n, x2n * an + beta, s) + lp(x2n, x1 * an + beta, s) - lp(x2, x1 * alpha + beta, s)
        + lp(x1, x_init * an + beta, s) - lp(x1, x_init * alpha + beta, s),
    }
    # update case 2 (unfold.jl:168-195)
    x1n = 1.3
    cases["update_shrink_change"] = {
        "score": lp(x1n, x_init * an + beta, s),
        "weight": lp(x1n, x_init * an + beta, s) - lp(x1, x_init * alpha + beta, s) - lp(x2, x1 * alpha + beta, s),
    }
    # update, no change (unfold.jl:233-249)
    cases["update_nochange"] = {"score": lp(x1, x_init * alpha + beta, s) + lp(x2, x1 * alpha + beta, s), "weight": 0.0}
    # update, change x2 (unfold.jl:251-275)
    x2n = 3.3
    cases["update_change_x2"] = {
        "score": lp(x1, x_init * alpha + beta, s) + lp(x2n, x1 * alpha + beta, s),
        "weight": lp(x2n, x1 * alpha + beta, s) - lp(x2, x1 * alpha + beta, s),
    }
    # update, params changed (unfold.jl:299-324)
    cases["update_params"] = {
        "score": lp(x1, x_init * an + beta, s) + lp(x2, x1 * an + beta, s),
        "weight": lp(x1, x_init * an + beta, s) - lp(x1, x_init * alpha + beta, s)
        + lp(x2, x1 * an + beta, s) - lp(x2, x1 * alpha + beta, s),
    }
    # regenerate, init changed (unfold.jl:437-458)
    xin = -0.1
    cases["regenerate_init"] = {
        "score": lp(x1, xin * alpha + beta, s) + lp(x2, x1 * alpha + beta, s),
        "weight": lp(x1, xin * alpha + beta, s) - lp(x1, x_init * alpha + beta, s),
    }
    return {
        "kernel": "x ~ normal(x_prev * alpha + beta, 1)",
        "args": {"x_init": x_init, "alpha": alpha, "beta": beta, "x1": x1, "x2": x2},
        "normal_logpdf": [
            {"x": x, "mu": mu, "std": sd, "logpdf": lp(x, mu, sd)}
            for (x, mu, sd) in [(1.1, 0.32, 1.0), (1.3, 0.85, 1.0), (3.3, 0.52, 1.0), (0.0, 0.0, 2.0), (-4.0, 1.5, 0.3)]
        ],
        "cases": cases,
    }


def kalman_loglik(A, b, Q, H, c, R, mu0, P0, ys):
    mu, P = mu0.copy(), P0.copy()
    ll = 0.0
    for t, y in enumerate(ys):
        if t > 0:
            mu = A @ mu + b
            P = A @ P @ A.T + Q
        S = H @ P @ H.T + R
        r = y - (H @ mu + c)
        ll += -0.5 * (len(y) * math.log(2 * math.pi) + np.linalg.slogdet(S)[1] + r @ np.linalg.solve(S, r))
        K = P @ H.T @ np.linalg.inv(S)
        mu = mu + K @ r
        P = P - K @ H @ P
    return ll


def lg_benchmark(d, seed=1):
    rng = np.random.default_rng(seed)
    A = 0.9 * np.eye(d) + 0.01 * rng.standard_normal((d, d))
    A *= 0.95 / max(abs(np.linalg.eigvals(A)))
    return A, np.zeros(d), 0.1 * np.eye(d), np.eye(d), np.zeros(d), 0.5 * np.eye(d), np.zeros(d), np.eye(d)


def simulate(A, b, Q, H, c, R, mu0, P0, T, seed):
    rng = np.random.default_rng(seed)
    x = rng.multivariate_normal(mu0, P0)
    ys = []
    for t in range(T):
        if t > 0:
            x = rng.multivariate_normal(A @ x + b, Q)
        ys.append(rng.multivariate_normal(H @ x + c, R))
    return np.array(ys)


def kalman():
    out = {}
    for name, d, T in [("lg2", 2, 20), ("lg10", 10, 100)]:
        P = lg_benchmark(d)
        ys = simulate(*P, T=T, seed=2)
        A, b, Q, H, c, R, mu0, P0 = P
        out[name] = {
            "d": d,
            "A": A.tolist(),
            "ys": ys.tolist(),
            "log_ml": kalman_loglik(A, b, Q, H, c, R, mu0, P0, ys),
            "note": "Q=0.1I, H=I, R=0.5I, mu0=0, P0=I, b=c=0; A seed 1, data seed 2",
        }
    return out


def main():
    for name, fn in [("philox_kat", philox_kat), ("hmm", hmm), ("unfold_kats", unfold_kats), ("kalman", kalman)]:
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(fn(), f, indent=1)
        print("wrote", name)


if __name__ == "__main__":
    main()
