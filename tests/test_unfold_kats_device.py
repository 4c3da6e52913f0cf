"""The reference's own Unfold known-answer tests driven through the device path.

test/modeling_library/unfold.jl:116-481 scores and re-weights traces of the
Unfold of kernel x ~ normal(x_prev * alpha + beta, 1) (unfold.jl:5-8) at
literal states (x_init 0.1, alpha 0.2, beta 0.3, x1 1.1, x2 1.2, ...); the
fixture tests/golden/unfold_kats.json holds its numbers.  Here the same states
go through the engine's device code: the kernel is the LG-SSM family at d = 1
(A = alpha, b = beta, Q = 1, x_1 ~ normal(alpha x_init + beta, 1)), the
literal trajectory is the distinguished particle of a conditional filter
(gh_pf_init_conditional / gh_pf_step_conditional pin particle 0 to it), and
the trace's score columns come from k_scores (gh_pf_get_scores: the latent's
log p(x_t | x_{t-1}) per step).  Each case's score is the sum of its latent
columns and each weight the reference's own difference of them; the normal
logpdf rows go through gh_dist_logpdf on the device.
"""
import json
import os

import numpy as np
import pytest

import gen_amd as gen
from gen_amd import dists as D

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "unfold_kats.json")


def latent_scores(alpha, beta, x_init, traj):
    """Device latent score columns of particle 0 pinned to `traj`."""
    m = gen.LinearGaussianSSM([[alpha]], [[1.0]], [[1.0]], [[1.0]], [alpha * x_init + beta], [[1.0]], b=[beta])
    T = len(traj)
    st = gen.conditional_smc(m, [np.zeros(1)] * T, 64, np.asarray(traj, dtype=np.float64).reshape(T, 1), seed=3)
    tr = gen.get_traces(st)
    assert np.array_equal(np.array([tr.step_states(t)[0, 0] for t in range(1, T + 1)]), np.asarray(traj))
    _, ps = tr.scores(per_step=True)
    out = ps[:, 0, 0].copy()
    st.close()
    return out


def test_device_scores_match_unfold_kats(gh_ctx):
    g = json.load(open(GOLD))
    a, want = g["args"], g["cases"]
    xi, al, be, x1, x2 = a["x_init"], a["alpha"], a["beta"], a["x1"], a["x2"]
    an = 0.5  # the new alpha of the argdiff cases (unfold.jl:196-481)
    noch = latent_scores(al, be, xi, [x1, x2])
    cx2 = latent_scores(al, be, xi, [x1, 3.3])
    par = latent_scores(an, be, xi, [x1, x2])
    ext = latent_scores(an, be, xi, [x1, 1.3, 1.4])
    shr = latent_scores(an, be, xi, [1.3])
    reg = latent_scores(al, be, -0.1, [x1, x2])
    got = {
        "update_nochange": (noch.sum(), 0.0),
        "update_change_x2": (cx2.sum(), cx2[1] - noch[1]),
        "update_params": (par.sum(), par[0] - noch[0] + par[1] - noch[1]),
        "update_extend_change": (ext.sum(), ext[2] + ext[1] - noch[1] + ext[0] - noch[0]),
        "update_shrink_change": (shr.sum(), shr[0] - noch[0] - noch[1]),
        "regenerate_init": (reg.sum(), reg[0] - noch[0]),
    }
    assert set(got) == set(want)
    for k, (score, weight) in got.items():
        assert abs(score - want[k]["score"]) <= 1e-13 * max(1.0, abs(want[k]["score"])), (k, score, want[k])
        assert abs(weight - want[k]["weight"]) <= 1e-12 * max(1.0, abs(want[k]["weight"])), (k, weight, want[k])


def test_device_normal_logpdf_matches_fixture(gh_ctx):
    for row in json.load(open(GOLD))["normal_logpdf"]:
        got = D.normal.logpdf(row["x"], row["mu"], row["std"])
        assert abs(got - row["logpdf"]) <= 1e-13 * max(1.0, abs(row["logpdf"])), row
