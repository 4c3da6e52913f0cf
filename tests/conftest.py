import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgen_hip.so on cuda:0)")


@pytest.fixture(scope="session")
def gh_ctx():
    """One HIP context for the whole GPU session (tests run in one process)."""
    import gen_amd

    ctx = gen_amd.Context(device=0)
    gen_amd.set_default_context(ctx)
    yield ctx
