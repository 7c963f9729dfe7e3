"""Arithmetic identities the kernels rely on to skip work bit-exactly.

GEOM_AXIS_FLAT (csrc/scene_layout.h): for a triangle whose three vertex normals
are one axis-aligned unit vector n, Triangle::getNormal (scene_basics.h:100-109)
blends n*w0 + n*w1 + n*w2 and renormalises.  The zero components stay signed
zeros; the +-1 component becomes +-s with s > 0, and normalisation divides by
RN(sqrt(RN(s*s))).  The shortcut is exact iff that equals s, which is checked
here exhaustively over every float in the range s can take, and end to end on
random hit points (numpy float32 is IEEE round-to-nearest; with zero
components the fused ops of the kernel reduce to these plain ops exactly).
"""
import numpy as np


def test_sqrt_of_square_is_identity_exhaustive():
    # s = w0 + w1 + w2 ~= 1 for points on the triangle; cover [2^-4, 2^4)
    lo = np.float32(2.0 ** -4).view(np.uint32)
    hi = np.float32(2.0 ** 4).view(np.uint32)
    for start in range(int(lo), int(hi), 1 << 22):
        s = np.arange(start, min(int(hi), start + (1 << 22)), dtype=np.uint32).view(np.float32)
        r = np.sqrt(s * s)
        assert np.array_equal(r.view(np.uint32), s.view(np.uint32))


def _get_normal_f32(v, vn, q, area):
    f = np.float32

    def cross(a, b):
        return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], f)

    c0 = cross(v[1] - q, v[2] - q)
    c1 = cross(v[2] - q, v[0] - q)
    c2 = cross(v[0] - q, v[1] - q)
    w = [f(0.5) * np.sqrt((c * c).sum(dtype=f)) / area for c in (c0, c1, c2)]
    n = vn[0] * w[0] + vn[1] * w[1] + vn[2] * w[2]
    s = np.sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2])
    return n / s


def test_axis_flat_normal_is_exact_on_random_points():
    rng = np.random.RandomState(0)
    f = np.float32
    for axis in range(3):
        for sign in (1.0, -1.0):
            for _ in range(200):
                n = np.zeros(3, f)
                n[axis] = f(sign)
                if rng.rand() < 0.5:  # signed zeros
                    n[(axis + 1) % 3] = f(-0.0)
                v = rng.uniform(-3, 3, (3, 3)).astype(f)
                v[:, axis] = f(rng.uniform(-3, 3))
                a, b = rng.dirichlet([1, 1, 1]).astype(f)[:2]
                q = (v[0] + a * (v[1] - v[0]) + b * (v[2] - v[0])).astype(f)
                e = np.cross(v[1] - v[0], v[2] - v[1]).astype(f)
                area = np.sqrt((e * e).sum(dtype=f)) / f(2)
                if not area > 0:
                    continue
                got = _get_normal_f32(v, np.stack([n, n, n]), q, area)
                assert np.array_equal(got.view(np.uint32), n.view(np.uint32)), (n, got)


def test_lemire_division_exact():
    """csrc/ipt_hip.hip udiv32: q = mulhi64(ceil(2^64/d), n) == n // d for 32-bit
    n and 1 < d < 2^32 (the kernels' g / spp and pixel / W)."""
    rng = np.random.RandomState(3)
    ds = [2, 3, 5, 7, 64, 100, 255, 500, 512, 1000, 1023, 4096, 65535, 2**31 - 1, 2**31, 2**32 - 1]
    ds += [int(x) for x in rng.randint(2, 2**31, 200)]
    ns = [0, 1, 2**32 - 1, 2**32 - 2, 2**31] + [int(x) for x in rng.randint(0, 2**32, 2000, dtype=np.uint64)]
    for d in ds:
        m = (2**64 - 1) // d + 1
        for n in ns + [d - 1, d, d + 1, 2 * d - 1, (2**32 - 1) // d * d, (2**32 - 1) // d * d - 1]:
            if 0 <= n < 2**32:
                assert (m * n) >> 64 == n // d, (n, d)


def test_div_const_equals_ieee_exhaustive(tmp_path):
    """ipt_device.h::div_const (x / b for b = 1/pi, 0.9, pi in three VALU
    operations) equals the IEEE quotient for every float 2^-100 <= x < 2^100:
    tools/check_div_const.c, compiled here (gcc -mfma -fopenmp), ~3 s."""
    import os
    import shutil
    import subprocess

    gcc = shutil.which("gcc")
    assert gcc, "gcc is needed for the exhaustive check"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "check_div_const")
    subprocess.run([gcc, "-O2", "-mfma", "-fopenmp", os.path.join(root, "tools", "check_div_const.c"), "-o", exe,
                    "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.count(": 0 mismatches") == 3, out.stdout
