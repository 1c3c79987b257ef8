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


@pytest.mark.gpu
def test_device_fast_math_matches_glibc():
    """The year kernels' math (MathFast): glibc's main path branch-free, and
    every input glibc sends down another path (|x| >= 88 for expf; x not a
    positive normal or |y log2 x| >= 126 for powf) redone in place -- equal
    to glibc everywhere, including the under/overflowing powers of very dry
    layers, which round 1 re-ran the whole substep for."""
    import ctypes as C
    import hybrid9_amd as h
    lb = h.lib()
    x, y = math_inputs()
    # hot-path shaped underflowing powers: s1^(2b+2) with tiny s1, large b
    rng = np.random.default_rng(9)
    k = 1 << 18
    xs = rng.uniform(1e-6, 0.05, k).astype(np.float32)
    ys = rng.uniform(2.0, 25.0, k).astype(np.float32)
    xe = rng.uniform(-110.0, -85.0, k).astype(np.float32)       # expf of deep water tables
    px, py = np.concatenate([x, xs]), np.concatenate([y, ys])
    ex = np.concatenate([x, xe])
    out = np.empty_like(ex)
    flag = np.empty(ex.size, np.int32)
    fp = flag.ctypes.data_as(C.POINTER(C.c_int))
    assert lb.h9g_math_fast_selftest(0, ex.size, h._fp(ex), None, h._fp(out), fp) == 0
    assert same_bits(out, glibc_expf(ex))
    assert flag[x.size:].sum() > 0.5 * k                            # took the redo branch
    out = np.empty_like(px)
    flag = np.empty(px.size, np.int32)
    fp = flag.ctypes.data_as(C.POINTER(C.c_int))
    assert lb.h9g_math_fast_selftest(0, px.size, h._fp(px), h._fp(py), h._fp(out), fp) == 0
    assert same_bits(out, glibc_powf(px, py))
    assert flag[x.size:].sum() > 0.1 * k


def div_inputs(n=1 << 22, seed=5):
    """Dividends/divisors over the whole float range plus the cases that
    stress a reciprocal-based division: divisors near powers of two,
    quotients near 1, in the subnormal range and near overflow."""
    rng = np.random.default_rng(seed)
    bits = lambda k: rng.integers(0, 1 << 32, k, dtype=np.uint64).astype(np.uint32).view(np.float32)
    x, d = bits(n), bits(n)
    k = n // 8
    x[:k] = rng.uniform(-1e4, 1e4, k).astype(np.float32)            # physical magnitudes
    d[:k] = rng.uniform(-1e5, 1e5, k).astype(np.float32)
    d[k:2 * k] = np.ldexp(1.0 + rng.integers(-4, 5, k) * 2.0 ** -23,
                          rng.integers(-20, 20, k)).astype(np.float32)
    with np.errstate(invalid="ignore"):     # NaN divisors here are filtered out below
        x[2 * k:3 * k] = np.clip(d[2 * k:3 * k].astype(np.float64) * (1.0 + rng.uniform(-1e-6, 1e-6, k)),
                                 -3e38, 3e38).astype(np.float32)
    x[3 * k:4 * k] = np.ldexp(rng.uniform(1, 2, k), rng.integers(-149, -100, k)).astype(np.float32)
    ok = np.isfinite(x) & np.isfinite(d) & (d != 0)
    return x[ok], d[ok]


@pytest.mark.gpu
def test_device_fast_division_is_correctly_rounded():
    """MathFast::div with the device reciprocal equals IEEE x/d bit for bit
    wherever it does not defer, and defers exactly on subnormal quotients."""
    import ctypes as C
    import hybrid9_amd as h
    x, d = div_inputs()
    out = np.empty_like(x)
    flag = np.empty(x.size, np.int32)
    rc = h.lib().h9g_div_selftest(0, x.size, h._fp(x), h._fp(d), h._fp(out),
                                  flag.ctypes.data_as(C.POINTER(C.c_int)))
    assert rc == 0
    with np.errstate(all="ignore"):
        ref = x / d
    # exact everywhere; the subnormal quotients are the ones redone as x / d
    assert same_bits(out, ref)
    sub = (ref != 0) & (np.abs(ref) < np.float32(2.0 ** -126))
    assert np.array_equal(flag.astype(bool), sub | ((out != 0) & (np.abs(out) < np.float32(2.0 ** -126))))


@pytest.mark.gpu
def test_device_fast_division_defers_on_zero_inf_nan_divisors():
    """recip64 of 0, inf or NaN is NaN, so MathFast::div redoes the quotient
    as x / d (IEEE: inf, 0 or NaN there)."""
    import ctypes as C
    import hybrid9_amd as h
    d = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 0.0, np.inf], np.float32)
    x = np.array([1.5, -2.0, 3.0, 0.0, 1.0, 0.0, np.inf], np.float32)
    out = np.empty_like(x)
    flag = np.empty(x.size, np.int32)
    rc = h.lib().h9g_div_selftest(0, x.size, h._fp(x), h._fp(d), h._fp(out),
                                  flag.ctypes.data_as(C.POINTER(C.c_int)))
    assert rc == 0
    assert flag.all()
    with np.errstate(all="ignore"):
        assert same_bits(out, x / d)


def test_markstein_quotient_of_conductivity_phase(tmp_path):
    """hk_fast (h9g_pair.h) computes s1 = 0.5a / 0.5b (HYDROLOGY.f90:605-608)
    from the stored RN(1/b) with one Markstein correction; it must equal the
    IEEE quotient over the operand range it accepts (tools/markstein_check.c:
    every b significand, midpoint-adjacent a, random a and b in [2^-60, 2^60),
    and a control with a one-ulp-off reciprocal that must fail)."""
    from pathlib import Path
    src = Path(__file__).resolve().parents[1] / "tools" / "markstein_check.c"
    exe = tmp_path / "markstein_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"], check=True)
    r = subprocess.run([str(exe), "8"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": 0 mismatches") == 2, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_markstein_quotient_exhaustive_slice_on_gpu(mode):
    """The exhaustive proof of hk_fast's s1 quotient (tools/markstein_exhaustive.hip:
    every pair of float significands, 7.04e13 pairs, 0 mismatches on the
    MI355X, profiles/markstein_r04.txt) re-run on the slice ADVICE r03 named:
    the 65,536 divisors whose significand is nearest all-ones, against every
    dividend significand (5.5e11 pairs), plus the one-ulp-off control that
    must fail.  Mode 1 is the refined v_rcp_f32 reciprocal of mk_div
    (h9g_step.h: the energy balance's and the conductivity phase's runtime
    divisors, round 5; full sweep in profiles/markstein_rcp_r04.txt), with
    its check of v_rcp_f32's scale invariance over [2^-60, 2^60)."""
    from tests.helpers import BUILD, ROOT, _build
    src = ROOT / "tools" / "markstein_exhaustive.hip"
    exe = ROOT / "tools" / "_build" / "markstein_exhaustive"
    if not exe.exists() or exe.stat().st_mtime < src.stat().st_mtime:
        exe.parent.mkdir(exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off",
                        "-fhip-fp32-correctly-rounded-divide-sqrt", "-o", str(exe), str(src)], check=True)
    r = subprocess.run([str(exe), str((1 << 23) - (1 << 16)), str(1 << 23), str(mode)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches against the IEEE quotient: 0" in r.stdout, r.stdout
