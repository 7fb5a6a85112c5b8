import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


@pytest.fixture
def gpu():
    """GPU tests FAIL (never skip) without a device: the HIP path has no fallback."""
    import torch
    assert torch.cuda.is_available(), "gpu test selected but no GPU is visible"
    from posfeat_amd import _lib
    _lib.require_device()
    return torch.device("cuda", torch.cuda.current_device())


GOLDEN = os.path.join(ROOT, "tests", "golden")

# The A/B build (posfeat_amd/csrc: make ab): the shipped library ignores the
# POSFEAT_* switches that select the non-default paths; tests that compare the
# default path with one of them run against this library -- in a child
# process (ab_env) or, for in-process tests, when the session itself loaded it
# (POSFEAT_HIP_LIB=posfeat_amd/libposfeat_hip_ab.so; the `ab` fixture).
AB_LIB = os.path.join(ROOT, "posfeat_amd", "libposfeat_hip_ab.so")


def ab_loaded():
    from posfeat_amd import _lib
    return _lib.lib().posfeat_ab_build() == 1


def ab_env():
    """Environment entries that make a child process load the A/B build."""
    if not os.path.exists(AB_LIB):
        pytest.skip("A/B build missing (make -C posfeat_amd/csrc ab)")
    return {"POSFEAT_HIP_LIB": AB_LIB}


def run_ab_child(code, out, timeout=300):
    """Run ``code`` (a Python program that writes the npz ``out``) in a child
    process on the A/B build, with the repository and tests/ importable;
    returns the npz contents.  The default GPU suite thus runs every A/B
    comparison, whatever library the session itself loaded."""
    import subprocess
    import numpy as np
    env = dict(os.environ, **ab_env())
    env["PYTHONPATH"] = os.pathsep.join([ROOT, os.path.join(ROOT, "tests"),
                                         env.get("PYTHONPATH", "")])
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=timeout)
    d = np.load(out)
    return {k: d[k] for k in d.files}


@pytest.fixture
def ab(gpu):
    """In-process A/B tests: the session must have loaded the A/B build."""
    if not ab_loaded():
        pytest.skip("A/B path switch: run with POSFEAT_HIP_LIB=posfeat_amd/libposfeat_hip_ab.so "
                    "(the shipped library ignores the switch)")
    return gpu
