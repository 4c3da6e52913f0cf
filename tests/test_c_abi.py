"""The C ABI driven from C alone (tests/c/pf_driver.c), as a Julia `ccall`
shim would drive it: the reference's HMM particle-filter test
(test/inference/particle_filter.jl:145-168) through gh_pf_init /
gh_pf_maybe_resample / gh_pf_step / gh_pf_log_ml_estimate, and the same
filter through gh_pf_run.

CPU: the driver is built (by __graft_entry__.build) against include/gen_hip.h
and resolves libgen_hip.so.  GPU: its log-ML is within the reference test's
atol of the exact forward-algorithm value, the batched run gives the same
filter (parents identical, log-ML to 1e-12) and the error path reports
GH_E_INVAL with a message.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "c", "pf_driver")


def _args(g, n, seed, thr):
    import numpy as np

    k, v = len(g["prior"]), len(g["emission"])
    T = np.asarray(g["transition"], dtype=float).ravel()  # T[new, prev] -> T[new*k + prev]
    E = np.asarray(g["emission"], dtype=float).ravel()    # E[x, z] -> E[x*k + z]
    nums = list(g["prior"]) + list(T) + list(E) + [float(x) for x in g["obs"]]
    return [DRIVER, str(k), str(v), str(n), str(seed), repr(float(thr)), str(len(g["obs"]))] + [repr(float(x)) for x in nums]


def test_driver_built_and_linked():
    if not os.path.exists(DRIVER):
        pytest.skip("tests/c/pf_driver not built (run __graft_entry__.build())")
    out = subprocess.run(["ldd", DRIVER], capture_output=True, text=True).stdout
    line = [l for l in out.splitlines() if "libgen_hip.so" in l]
    assert line and "not found" not in line[0], out
    assert os.path.realpath(line[0].split("=>")[1].split("(")[0].strip()) == \
        os.path.realpath(os.path.join(ROOT, "gen_amd", "libgen_hip.so"))


@pytest.mark.gpu
def test_reference_hmm_pf_test_from_c():
    with open(os.path.join(ROOT, "tests", "golden", "hmm.json")) as f:
        g = json.load(f)["pf_test"]
    r = subprocess.run(_args(g, g["num_particles"], 0, g["ess_threshold"]), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    got = dict(l.split() for l in r.stdout.strip().splitlines())
    lml, lml_run = float(got["log_ml_calls"]), float(got["log_ml_run"])
    assert abs(lml - g["log_ml"]) < g["atol"], (lml, g["log_ml"])
    assert abs(lml_run - lml) <= 1e-12 * abs(lml), (lml_run, lml)
    assert got["parents_equal"] == "1"
    assert int(got["resamples"]) == len(g["obs"]) - 1  # threshold N: every step resamples
    assert int(got["n"]) == g["num_particles"]
    assert got["error_path_ok"] == "1"
