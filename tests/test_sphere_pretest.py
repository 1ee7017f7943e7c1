"""The exact sphere pre-test (intersect.h sphere_surely_misses) restated in binary64 numpy
(no contraction, the device build's -ffp-contract=off) against the reference's sphere test
(geometry.cpp:47-67 after Ray::direction's normalized(), intersect.h sphere_hit): whenever the
pre-test says "certainly no hit", the reference's arithmetic finds none.  Adversarial samples:
rays starting on the sphere (the shadow and secondary rays of its own hits), grazing rays,
rays from inside, and object-space directions scaled by 1e-40...1e40."""
import numpy as np
import pytest


def sq4(x, y, z):
    return (x * x + z * z) + y * y


def dot4z(ax, ay, az, bx, by, bz):
    return (ax * bx + az * bz) + ay * by


def reference_hits(oo, draw, c, rr, reverse):
    n = np.sqrt(sq4(*draw))
    dd = [v / n for v in draw]
    oc = [oo[k] - c[k] for k in range(3)]
    a = sq4(*dd)
    b = 2 * dot4z(*dd, *oc)
    cc = sq4(*oc) - rr
    disc = b * b - (4 * a) * cc
    with np.errstate(invalid="ignore"):
        s = np.sqrt(disc)
        t = np.where(reverse, (-b + s) / (2 * a), (-b - s) / (2 * a))
    return (disc >= 0) & (t >= 0)


def surely_misses(oo, draw, c, rr, reverse):
    oc = [oo[k] - c[k] for k in range(3)]
    A = sq4(*draw)
    B = 2 * dot4z(*draw, *oc)
    oc2 = sq4(*oc)
    C = oc2 - rr
    D = B * B - (4 * A) * C
    scale = B * B + (4 * A) * (oc2 + np.abs(rr))
    ranged = (scale >= 1e-200) & (scale <= 1e200) & (A >= 1e-100) & (A <= 1e100)
    b_pos = B > 1e-10 * np.sqrt(scale)
    return ranged & ((D < -1e-10 * scale) | (b_pos & (~reverse | ((4 * A) * C > 1e-9 * scale))))


def samples(rng, n):
    c = rng.normal(size=(3, n)) * 10.0 ** rng.uniform(-3, 3, n)
    r = 10.0 ** rng.uniform(-3, 3, n)
    rr = (r.astype(np.float32) * r.astype(np.float32)).astype(np.float64)  # fp32 r*r (geometry.cpp:53)
    u = rng.normal(size=(3, n))
    u /= np.sqrt((u ** 2).sum(0))
    kind = rng.integers(0, 4, n)
    # origins: on the sphere (its own hits), near it, inside, far
    f = np.select([kind == 0, kind == 1, kind == 2], [np.ones(n), 1 + 10.0 ** rng.uniform(-12, -1, n),
                                                     rng.uniform(0, 1, n)], 10.0 ** rng.uniform(0.5, 3, n))
    f = f * (1 + rng.normal(size=n) * 1e-15)
    oo = c + u * (np.sqrt(rr) * f)
    # directions: random, tangent-ish to the sphere at the origin, along the normal
    v = rng.normal(size=(3, n))
    v /= np.sqrt((v ** 2).sum(0))
    tang = v - u * (v * u).sum(0)
    tang /= np.sqrt((tang ** 2).sum(0))
    eps = 10.0 ** rng.uniform(-14, 0, n) * rng.choice([-1, 1], n)
    dkind = rng.integers(0, 3, n)
    d = np.where(dkind == 0, v, np.where(dkind == 1, tang + u * eps, u * rng.choice([-1, 1], n)))
    d = d * 10.0 ** rng.uniform(-40, 40, n)  # the object-space length of a unit world direction
    reverse = rng.random(n) < 0.5
    return list(oo), list(d), list(c), rr, reverse


@pytest.mark.parametrize("seed", range(8))
def test_pretest_never_drops_a_hit(seed):
    rng = np.random.default_rng(1000 + seed)
    oo, draw, c, rr, reverse = samples(rng, 500_000)
    with np.errstate(all="ignore"):
        hit = reference_hits(oo, draw, c, rr, reverse)
        skip = surely_misses(oo, draw, c, rr, reverse)
    assert not np.any(hit & skip), int(np.sum(hit & skip))
    # and it decides most of the misses (what it is for)
    assert np.sum(skip) > 0.5 * np.sum(~hit)


def test_pretest_on_the_surface_outwards():
    """A ray leaving its own sphere's surface: the pre-test decides it without the reference's
    arithmetic unless it grazes; from inside (reverse) it never decides it."""
    rng = np.random.default_rng(7)
    n = 200_000
    c = [np.zeros(n)] * 3
    u = rng.normal(size=(3, n))
    u /= np.sqrt((u ** 2).sum(0))
    rr = np.ones(n)
    oo = list(u * (1 + rng.normal(size=n) * 1e-16))
    v = rng.normal(size=(3, n))
    v /= np.sqrt((v ** 2).sum(0))
    out = np.where((v * u).sum(0) > 0, v, -v)
    with np.errstate(all="ignore"):
        hit = reference_hits(oo, list(out), c, rr, np.zeros(n, bool))
        skip = surely_misses(oo, list(out), c, rr, np.zeros(n, bool))
        skip_rev = surely_misses(oo, list(out), c, rr, np.ones(n, bool))
    assert not np.any(hit & skip)
    assert np.mean(skip) > 0.99
    assert not np.any(skip_rev & reference_hits(oo, list(out), c, rr, np.ones(n, bool)))
