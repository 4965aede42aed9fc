"""Unit checks of oracle building blocks against independent references (CPU)."""
import matplotlib

matplotlib.use("Agg")
import matplotlib.path as mpath  # noqa: E402
import numpy as np  # noqa: E402
import pytest  # noqa: E402

from helpers import POLYS  # noqa: E402
from oracle import sit_oracle as so  # noqa: E402


def test_philox_known_answer_vectors():
    """Random123 kat_vectors for philox4x32_10."""
    out = so.philox4x32_10((0, 0, 0, 0), (0, 0))
    assert [int(x) for x in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    m = 0xFFFFFFFF
    out = so.philox4x32_10((m, m, m, m), (m, m))
    assert [int(x) for x in out] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    out = so.philox4x32_10((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0))
    assert [int(x) for x in out] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_sampler_uniform_range_and_spread():
    u = so.sampler_uniform(25450, np.arange(20000), np.zeros(20000))
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01


def test_point_in_polygon_matches_matplotlib_off_boundary():
    rng = np.random.default_rng(1)
    n = rng.uniform(-100, 10100, 20000)
    e = rng.uniform(-100, 10100, 20000)
    got = so.point_in_polygons(POLYS, n, e)
    want = np.zeros_like(got)
    for p in POLYS:
        want |= mpath.Path(np.vstack([p, p[:1]])).contains_points(np.stack([e, n], axis=1))
    d = so.distance_to_polygons(POLYS, n, e)
    far = d > 1e-6
    assert np.array_equal(got[far], want[far])


def test_point_in_polygon_boundary_is_not_contained():
    # vertices and points on edges are on the boundary: Polygon.contains is False
    p = POLYS[3]
    assert not so.point_in_polygons(POLYS, p[:, 1], p[:, 0]).any()
    mid_e = (p[0, 0] + p[1, 0]) / 2
    mid_n = (p[0, 1] + p[1, 1]) / 2
    assert not so.point_in_polygons(POLYS, np.array([mid_n]), np.array([mid_e]))[0]
    # axis-aligned map-edge segment of island 1: east = 0, north in (2350, 10000)
    assert not so.point_in_polygons(POLYS, np.array([5000.0]), np.array([0.0]))[0]
    assert so.point_in_polygons(POLYS, np.array([5000.0]), np.array([1e-9]))[0]


def test_distance_to_polygons_brute_force():
    rng = np.random.default_rng(2)
    n = rng.uniform(0, 10000, 3000)
    e = rng.uniform(0, 10000, 3000)
    got = so.distance_to_polygons(POLYS, n, e)
    best = np.full(n.shape, np.inf)
    for p in POLYS:
        a = p
        b = np.roll(p, -1, axis=0)
        for (ax, ay), (bx, by) in zip(a, b):
            dx, dy = bx - ax, by - ay
            t = np.clip(((e - ax) * dx + (n - ay) * dy) / (dx * dx + dy * dy), 0, 1)
            best = np.minimum(best, np.hypot(e - (ax + t * dx), n - (ay + t * dy)))
    np.testing.assert_allclose(got, best, rtol=1e-9, atol=1e-9)


def test_exact_orientation_fallback():
    # collinear by construction: q on the line through p1 p2 with exact binary coordinates
    s = so.orientation_index(np.array([0.0]), np.array([0.0]), np.array([4.0]), np.array([2.0]),
                             np.array([2.0]), np.array([1.0]))
    assert s[0] == 0
    s = so.orientation_index(np.array([0.0]), np.array([0.0]), np.array([4.0]), np.array([2.0]),
                             np.array([2.0]), np.array([1.0 + 2 ** -40]))
    assert s[0] == 1


@pytest.mark.parametrize("bits,expect", [
    (0, " |Test ship not in terminal state| |Obstacle ship not in terminal state| "),
    (so.ST_OBS_ENDPOINT, " |Test ship not in terminal state| |Obstacle ship reaches endpoint|"
                         "|Obstacle ship not in terminal state| "),
    (so.ST_COLLISION, " |Test ship not in terminal state| |Obstacle ship not in terminal state| |Ship collision|"),
])
def test_status_strings(bits, expect):
    assert so.status_string(bits) == expect
