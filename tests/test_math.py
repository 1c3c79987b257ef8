"""Device math (hybrid9_amd/csrc/h9_math.h) vs this machine's glibc 2.35.

The reference calls glibc expf/powf (flang lowers EXP and real powers to
them).  CPU tests check the header's host build -- the same source the
gfx950 kernels compile -- bit-for-bit: expf over ALL 2^32 inputs, powf on
random, hot-path-shaped and special pairs.  The GPU test checks the
device build through h9g_math_selftest."""
import subprocess

import numpy as np
import pytest

from tests.conftest import same_bits
from tests.helpers import check_math_bin, glibc_expf, glibc_powf, math_inputs


def _run(*args, timeout=600):
    r = subprocess.run([str(check_math_bin()), *args], capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
    return r.stdout


def test_expf_exhaustive():
    _run("expf_all")


def test_powf_random():
    _run("powf_rand", "50000000", "11")


def test_powf_special():
    _run("powf_special")


def test_shipped_library_host_math():
    import hybrid9_amd as h
    lb = h.lib()
    x, y = math_inputs(1 << 12, seed=3)
    e = np.array([lb.h9g_host_expf(float(v)) for v in x[:20000]], np.float32)
    p = np.array([lb.h9g_host_powf(float(a), float(b)) for a, b in zip(x[:20000], y[:20000])],
                 np.float32)
    assert same_bits(e, glibc_expf(x[:20000]))
    assert same_bits(p, glibc_powf(x[:20000], y[:20000]))


@pytest.mark.gpu
def test_device_math_matches_glibc():
    import hybrid9_amd as h
    lb = h.lib()
    x, y = math_inputs()
    out = np.empty_like(x)
    assert lb.h9g_math_selftest(0, x.size, h._fp(x), None, h._fp(out)) == 0
    assert same_bits(out, glibc_expf(x))
    assert lb.h9g_math_selftest(0, x.size, h._fp(x), h._fp(y), h._fp(out)) == 0
    assert same_bits(out, glibc_powf(x, y))
