"""The C-ABI boundary (CPU only: no compute calls without a GPU).

libgen_hip.so must load and export every entry point include/gen_hip.h
declares, with the argument structs laid out as the header says.
"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gen_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gh_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_pf_api():
    syms = declared_symbols()
    for s in ["gh_pf_init", "gh_pf_step", "gh_pf_maybe_resample", "gh_pf_log_ml_estimate",
              "gh_pf_get_log_weights", "gh_pf_sample_unweighted", "gh_is_run", "gh_ctx_create_dist"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from gen_amd import _lib

    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # every declared symbol has a ctypes signature in the binding
    assert set(declared_symbols()) <= set(_lib.SIGNATURES)


def test_host_only_entry_points():
    from gen_amd import _lib

    lib = _lib.load()
    assert lib.gh_version().decode().startswith("gen_hip")
    o = _lib.PFOpts()
    lib.gh_pf_opts_default(ctypes.byref(o))
    assert o.resampler == _lib.RESAMPLE_SYSTEMATIC and o.record_history == 1
    # argument validation happens before any device work
    rc = lib.gh_ctx_create(0, None, None)
    assert rc == 1 and b"NULL" in lib.gh_last_error()


def test_struct_layouts_match_header():
    from gen_amd import _lib

    assert ctypes.sizeof(_lib.ModelDesc) == 5 * 4 + 4 + 8 + 8  # 5 int32, pad, ptr, int64
    assert ctypes.sizeof(_lib.Obs) == 32  # ptr, n_values, present, slot, reserved, next
    assert _lib.Obs.next.offset == 24 and _lib.Obs.slot.offset == 16
    assert ctypes.sizeof(_lib.PFOpts) == 32


def test_oracle_is_not_reachable_from_the_product():
    """The product package never imports the oracle (it is test infrastructure)."""
    pkg = os.path.join(ROOT, "gen_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", src).replace("CPU oracle", ""), f


def test_python_api_validates_before_the_device():
    import gen_amd as gen
    from gen_amd.pf import _step_obs

    m = gen.DiscreteHMM([0.5, 0.5], [[0.9, 0.1], [0.1, 0.9]], [[0.8, 0.3], [0.2, 0.7]])
    obs, _ = _step_obs(m, 3, gen.choicemap((("chain", 2, "x"), 1)))
    assert obs.present == 1 and obs.n_values == 1
    with pytest.raises(gen.GenHipError) as e:
        _step_obs(m, 3, gen.choicemap((("chain", 1, "x"), 1)))  # constrains an old choice
    assert e.value.code == 2  # GH_E_DISCARD, particle_filter.jl:168-170
    obs, _ = _step_obs(m, 1, gen.choicemap((("x_init",), 0)))
    assert obs.present == 1
    obs, _ = _step_obs(m, 4, None)
    assert obs.present == 0
