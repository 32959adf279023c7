"""Host-side (no GPU) checks of the product library: it loads, exports every symbol the
headers declare, and its native gym seeding reproduces the reference fixture's resets."""
import os
import re

import numpy as np
import pytest

from tests.conftest import ROOT


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rd[dmlp]?_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from reacherdistilation_amd import _native, build
    build.build(verbose=False)
    return _native.load()


@pytest.mark.parametrize("header", sorted(os.listdir(os.path.join(ROOT, "include"))))
def test_library_exports_header(lib, header):
    names = _declared(header)
    assert names, header
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{header}: not exported: {missing}"


def test_version_string(lib):
    assert b"gfx950" in lib.rd_version()


def test_gym_seeding_matches_fixture(lib, golden):
    from reacherdistilation_amd.env import gym_reset_draws
    d = gym_reset_draws(0, 25)
    q0, q1, v0, v1, tx, ty = d.T
    exp = np.stack([np.cos(q0), np.cos(q1), np.sin(q0), np.sin(q1), tx, ty, v0, v1], axis=1)
    assert np.array_equal(exp, golden["ob"][:, 0, :8])


@pytest.mark.parametrize("seed", [0, 1, 41, 10000, 2 ** 40 + 3])
def test_gym_seeding_matches_numpy_rng(lib, seed):
    from oracle import reacher_np as rn
    from reacherdistilation_amd.env import gym_reset_draws
    rng = rn.gym_rng(seed)
    exp = np.array([rn.reset_draw(rng) for _ in range(40)])
    assert np.array_equal(gym_reset_draws(seed, 40), exp)


def test_bad_arguments_report_errors(lib):
    import ctypes
    from reacherdistilation_amd import _native as nat
    h = ctypes.c_void_p()
    rc = lib.rd_create(ctypes.byref(h), 0, 0, 0, 0, None)
    assert rc == -100000
    assert b"bad argument" in lib.rd_last_error()
    with pytest.raises(nat.NativeError):
        nat.check(rc, "rd_create")


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: pointing the loader at a missing build raises."""
    import subprocess
    import sys
    code = ("import os; os.environ['RD_LIB']='libreacher_missing.so'\n"
            "from reacherdistilation_amd import _native\n"
            "try:\n    _native.load()\nexcept _native.NativeError as e:\n    print('raised', e)\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert "raised" in out.stdout, out.stdout + out.stderr
