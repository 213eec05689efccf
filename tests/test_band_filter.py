"""The band re-check's candidate filter of k_vote_mfma (PVM_BANDV 2,
pvnet_amd/csrc/pvvote.hip), checked in float32
arithmetic on the CPU.

Round 5 queued a pair of a flagged MFMA for the reference's sequence (KU:116-125)
when |z| <= g, g = fma(kx, |X|, fma(ky, |Y|, G)), z = X - |Y|, with
G = gzf B s 1.001.  Round 6 queues it when t = fma(-K, |X|, |z|) <= G', with
K = (kx + ky) c and G' = gb gzf / (gzf + gzr) 1.0011 c, c = 1.0002 / (1 - 1.0001 ky),
derived from the
hot loop's bound gb = (gzf + gzr) B s 1.00001.  Every decision stays the
reference's only if the new queue contains the old one: this test draws pairs
on and around the old band's edge (the worst case for the inequality
|Y| <= |X| + |z| it rests on) and asserts that every pair the old test queues,
the new one queues too.  The constants are the kernel's (fast_constants,
mfma_gz); fma is emulated in float64 (exact products of float32 values)."""
import numpy as np
import pytest

U = 1.0 / 16777216.0
f32 = np.float32


def fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def constants(thr):
    tau = np.sqrt(1.0 - thr * thr) / thr
    gzr = f32(2.0 * 9.5 * (tau + 1.0 / tau) * U * 1.0001)          # fast_constants
    gzf = f32(2.0 * (41.5 * float(f32(tau)) + 38.7) * U * 1.0001)   # mfma_gz
    return f32(tau), gzf, gzr


@pytest.mark.parametrize("thr", [0.99, 0.9, 0.5, 0.05, 0.999999])
def test_new_queue_contains_old(thr):
    rng = np.random.default_rng(int(thr * 1e6))
    tau, gzf, gzr = constants(thr)
    kx = f32(f32(gzr / tau) * f32(1.0001))
    ky = f32(gzr * f32(1.0001))
    inv1k = f32(f32(1.0002) / f32(f32(1.0) - f32(ky * f32(1.0001))))
    K = f32((kx + ky) * inv1k)
    gq = f32(f32(f32(gzf / f32(gzf + gzr)) * f32(1.0011)) * inv1k)
    n = 400_000
    # per-hypothesis bound B and scale s as hscale makes them (s a power of two)
    Bv = f32(10.0) ** rng.uniform(-1, 4.5, n).astype(f32)
    s = np.ldexp(f32(1.0), -rng.integers(0, 10, n)).astype(f32)
    G = f32(f32(gzf * Bv) * s) * f32(1.001)                          # round 5's per-pair constant
    gb = f32(f32(f32(gzf + gzr) * Bv) * s) * f32(1.00001)            # the hot loop's bound
    Gn = f32(gb * gq)                                                # round 6's
    # X, Y of the pair (scaled, as the MFMA forms): |h - c| up to B, any angle
    d = (Bv * s * rng.uniform(0, 1, n).astype(f32)).astype(f32)
    X = (d * rng.uniform(-1, 1, n).astype(f32)).astype(f32)
    Yabs = np.abs(X) * rng.uniform(0, 3, n).astype(f32)
    Y = np.where(rng.random(n) < 0.5, Yabs, -Yabs).astype(f32)
    g = fma32(kx, np.abs(X), fma32(ky, np.abs(Y), G))
    # put z on the old band's edge (and just inside / outside): X = |Y| + z
    frac = rng.choice(np.array([1.0, 0.999999, 1.000001, 0.5, -1.0, -0.999999, -1.000001], dtype=f32), n)
    z_target = (g * frac).astype(f32)
    X = (np.abs(Y) + z_target).astype(f32)
    g = fma32(kx, np.abs(X), fma32(ky, np.abs(Y), G))                # g of the final X
    z = (X - np.abs(Y)).astype(f32)
    old = np.abs(z) <= g
    t = fma32(-K, np.abs(X), np.abs(z))
    new = t <= Gn
    assert old.sum() > n // 4
    bad = old & ~new
    assert not bad.any(), f"{bad.sum()} pairs queued by the round-5 test but not by the filter (thr {thr})"


def test_inequality_y_le_x_plus_z():
    """|Y| <= |X| + |z| for z = X - |Y| in exact arithmetic, both signs of X."""
    rng = np.random.default_rng(7)
    X = rng.normal(size=100_000) * 10 ** rng.uniform(-3, 3, 100_000)
    Y = rng.normal(size=100_000) * 10 ** rng.uniform(-3, 3, 100_000)
    z = X - np.abs(Y)
    assert np.all(np.abs(Y) <= np.abs(X) + np.abs(z) + 1e-12 * (np.abs(X) + np.abs(Y)))
