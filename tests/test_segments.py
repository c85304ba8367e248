"""The exactness claim behind the kernel's segment-bounded crossings (svo_cast.hip: seg_cap), checked
on the CPU: from a DDA state (T, a) as dda_axis and later additions produce it, the crossings
0 .. seg_cap + 1 computed in closed form — one rounding of the exact T + i*a, as fma(i, a, T) does —
equal castRayFromCam's iterated double sums T += a (ray_caster.cpp:70-80).  seg_cap is restated here
bit for bit (f32 rounding through numpy; the reciprocal perturbed by up to 1 ulp, as v_rcp_f32 may be)."""
import struct
from fractions import Fraction

import numpy as np


def _bits(d):
    return struct.unpack("<Q", struct.pack("<d", d))[0]


def _lsb_exp(T):
    b = _bits(T)
    lo, hi = b & 0xFFFFFFFF, b >> 32
    e = (hi >> 20) & 0x7FF
    if lo:
        tz = (lo & -lo).bit_length() - 1
    else:
        m = (hi & 0xFFFFF) | 0x100000
        tz = 32 + (m & -m).bit_length() - 1
    if e:
        return e - 1075 + tz
    return (1 << 20) if (b << 1) & ((1 << 64) - 1) == 0 else -1074


def _seg_cap(T, af, inva):
    ab = struct.unpack("<I", struct.pack("<f", af))[0]
    m = ab | 0x800000
    la = ((ab >> 23) & 0xFF) - 150 + ((m & -m).bit_length() - 1)
    be = min(max(min(_lsb_exp(T), la) + 53 + 1023, 1), 0x7FF)
    B = struct.unpack("<d", struct.pack("<Q", (be << 20) << 32))[0]
    x = np.float32(np.float32(np.float32(B - T) * np.float32(inva)) * np.float32(0.99999905))
    if not np.isfinite(x):
        return 1 << 30
    return int(min(max(np.floor(float(x)), 0), 1 << 30))


def _closed(i, a, T):
    return float(Fraction(i) * Fraction(a) + Fraction(T))  # the exact sum rounded once


def test_segment_cap_is_exact():
    rng = np.random.default_rng(7)
    checked = 0
    for trial in range(1500):
        o = float(np.float32(rng.uniform(-300, 300)))
        d = float(np.float32(rng.uniform(-1, 1)))
        if d == 0.0:
            continue
        delta = float(np.float32(np.float32(1.0) / np.float32(d)))
        a = abs(delta)
        af = float(np.float32(a))
        cell = int(np.trunc(np.float32(o)))
        ex = o - 1.0 if d < 0 else o
        T = a - (ex - cell) * delta  # deltaPos (dda_axis)
        for _ in range(int(rng.choice([0, 1, 2, 5, 50, 300, 3000]))):
            T = T + a  # some iterated steps first
        inva = float(np.float32(1.0 / af)) * (1 + int(rng.integers(-1, 2)) * 2.0 ** -23)
        c = _seg_cap(T, af, float(np.float32(inva)))
        t, n = T, min(c + 1, 5000)
        for i in range(n + 1):
            if i:
                t = t + a
            if i in (0, 1, 2, n - 1, n) or i % 61 == 0:
                assert _closed(i, a, T) == t, (o, d, c, i)
                checked += 1
    assert checked > 10000


def _count_est(T, af, inva, V):
    # svo_cast.hip count_est: m = cvt_u32(fma_f32(f32(V) - f32(T), inva, 0.5)) (the f32 fma emulated
    # as the exact product plus 1/2 in double, rounded to f32 once more; v_cvt_u32_f32 truncates and
    # saturates at 0)
    x = np.float32(np.float32(V) - np.float32(T))
    y = np.float32(float(x) * float(np.float32(inva)) + 0.5)
    return int(max(np.trunc(float(y)), 0.0))


def test_count_estimate_within_one():
    """skip_box's crossing counts start from an f32 estimate m of #{j >= 0 : T + j*a < V} (or <=):
    m must be the count c or c - 1 (one exact f64 test then settles it).  States as the kernel reaches
    them: T a crossing value of an axis after up to 2^20 crossings, V any value up to T + steps * a
    (budget < 2^20 in all), the reciprocal off by up to 1 ulp (v_rcp_f32)."""
    rng = np.random.default_rng(11)
    for _ in range(20000):
        a = float(np.float32(2.0 ** rng.uniform(-2, 12)))
        af = np.float32(a)
        inva = np.float32(1.0) / af
        inva = np.nextafter(inva, np.float32(rng.choice([0.0, np.inf]))) if rng.random() < 0.5 else inva
        budget = int(rng.choice([300, 16384, (1 << 20) - 1]))
        j = int(rng.integers(0, budget))
        T = float(Fraction(a) * (j + 1) - Fraction(a) * Fraction(float(np.float32(rng.random()))))
        steps = budget - j
        V = T + float(rng.random()) * steps * a
        if rng.random() < 0.3:  # V on a crossing of this axis, or next to one
            i = int(rng.integers(0, steps + 1))
            V = float(np.nextafter(_closed(i, a, T), rng.choice([-np.inf, np.inf]))) if rng.random() < 0.5 else _closed(i, a, T)
        m = _count_est(T, af, inva, V)
        xs = (Fraction(V) - Fraction(T)) / Fraction(a)
        c_lt = max(0, -(-xs.numerator // xs.denominator))  # #{j >= 0 : T + j a < V} = ceil(x)
        c_le = max(0, xs.numerator // xs.denominator + 1)  # #{j >= 0 : T + j a <= V} = floor(x) + 1
        assert m in (c_lt - 1, c_lt) or c_lt == 0 and m == 0, (T, a, V, m, c_lt)
        assert m in (c_le - 1, c_le) or c_le == 0 and m == 0, (T, a, V, m, c_le)
