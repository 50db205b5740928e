"""The shared transcendentals (isaklm-raytracer_amd/csrc/rt_libm.h) — CPU.

Both the oracle and the gfx950 kernels evaluate sinf/cosf/tanf/powf through
rt_libm.h (stand-ins for CUDA libdevice), so parity between them
is by construction; this test checks the functions themselves against glibc's
double-precision results rounded to float (i.e. correct rounding in practice).
"""
import ctypes

import numpy as np
import pytest

import oracle


def _eval(kind, x):
    L = oracle.lib()
    L.or_libm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.or_libm.restype = None
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    L.or_libm(kind, x.ctypes.data, out.ctypes.data, len(x))
    return out


@pytest.mark.parametrize("kind,fn", [(0, np.sin), (1, np.cos), (2, np.tan)])
def test_trig_correctly_rounded(kind, fn):
    rng = np.random.default_rng(kind)
    tau = np.float32(3.1415926536) * np.float32(2)
    # the device domain (phi = xi * TAU, xi in [0, 1]) densely, plus the camera/mesh angles
    x = np.concatenate([rng.uniform(0, tau, 400_000), np.linspace(0, tau, 100_000),
                        rng.uniform(-8, 8, 100_000), [0.0, tau, np.float32(1.5707963705062866) / 2]]).astype(np.float32)
    got = _eval(kind, x)
    ref = fn(x.astype(np.float64)).astype(np.float32)
    assert np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32)) == 0


def test_trig_exact_values():
    assert _eval(0, [0.0])[0] == 0.0 and _eval(1, [0.0])[0] == 1.0
    assert np.signbit(_eval(0, [-0.0])[0])


def test_powf_gamma_domain():
    rng = np.random.default_rng(11)
    x = rng.uniform(0.0031308, 1.5, 300_000).astype(np.float32)
    got = _eval(3, x)
    ref = np.power(x.astype(np.float64), np.float64(np.float32(1 / 2.4))).astype(np.float32)
    assert np.count_nonzero(got != ref) == 0


def test_sincos_equals_sin_and_cos(tmp_path):
    """rt_sincosf (one reduction for both, the shading code's form) gives
    rt_sinf's and rt_cosf's bits: every 3rd float of [-8, 8], every 4096th
    float up to 1e6 (tests/native/sincos_check.c; the full [-8, 8] sweep, 2.2
    billion floats, was run too: 0 mismatches)."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "sincos_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fopenmp", "-I",
                    os.path.join(root, "isaklm-raytracer_amd", "csrc"),
                    os.path.join(root, "tests", "native", "sincos_check.c"), "-o", exe, "-lm"], check=True)
    r = subprocess.run([exe, "3"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="8"))
    assert r.returncode == 0 and " mismatches 0" in r.stdout and int(r.stdout.split()[1]) > 300_000_000, r.stdout
