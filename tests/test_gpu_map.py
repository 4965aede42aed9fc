"""GPU parity of the island-map predicates (sit_probe_map) against the oracle's GEOS restatement.

The step kernel decides terrain hits and the boundary-distance reward term through a spatial
index (nearest-edge grid, class grid, per-cell crossing records; sit_device.h).  The index must
reproduce the full scans of the reference's predicates exactly:
  * Polygon.contains               obstacle.py:126-129   (GEOS RayCrossingCounter)
  * exterior.distance              obstacle.py:138-141   (GEOS Distance::pointToSegment)
  * is_pos_inside_obstacles        MSRL_env_ex.py:490-515 (four hull corners at +-l/2)
Points: uniform over the map and its margin, dense bands along every edge (offsets from 1e-9 m
to 80 m on both sides), exact vertices, edge midpoints, and rays through vertex latitudes
(GEOS's degenerate cases).  float64: identical booleans everywhere, distance within 1e-12.
float32 (the probes run in the float32 step kernels' translation unit, device fast-math): the
oracle evaluates the same float32 points in float64; containment and the hull test are identical
everywhere, on the boundary band included — the kernel decides containment in float64 from the
float32 point (count_segment) and forms the hull corners n +- l/2 in float64 as the reference
does — and the distance is within 1e-5 relative (floor 10 m).
"""
import numpy as np
import pytest
import torch

from helpers import POLYS
from oracle import sit_oracle as so

pytestmark = pytest.mark.gpu

sit = pytest.importorskip("sac_maritime_ast_amd")
from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402

DEV = "cuda:0"
HALF = 40.0   # l/2 of the reference ship (test_policy.py ShipConfiguration length 80 m)


def probe_points(seed=7):
    rng = np.random.default_rng(seed)
    pts = [np.stack([rng.uniform(-600, 10600, 200_000), rng.uniform(-600, 10600, 200_000)], 1)]
    for ring in POLYS:
        a = ring
        b = np.roll(ring, -1, axis=0)
        for (ax, ay), (bx, by) in zip(a, b):
            m = 1500
            t = rng.uniform(0, 1, m)
            ex, ey = bx - ax, by - ay
            L = np.hypot(ex, ey)
            nx, ny = -ey / L, ex / L
            off = np.exp(rng.uniform(np.log(1e-9), np.log(80.0), m)) * rng.choice([-1.0, 1.0], m)
            x = ax + t * ex + off * nx
            y = ay + t * ey + off * ny
            pts.append(np.stack([y, x], 1))                            # (north, east)
            pts.append(np.array([[ay, ax], [(ay + by) / 2, (ax + bx) / 2]]))   # vertex, midpoint
            # rays through the vertex latitude (horizontal-ray degeneracies), left and right
            xs = np.concatenate([rng.uniform(-600, 10600, 40), [ax - 1.0, ax + 1.0, ax - 1e-7, ax + 1e-7]])
            pts.append(np.stack([np.full(xs.shape, ay), xs], 1))
            # hull corners landing exactly on the vertex
            pts.append(np.array([[ay + s1 * HALF, ax + s2 * HALF] for s1 in (-1, 1) for s2 in (-1, 1)]))
    return np.concatenate(pts)


def oracle_predicates(pts):
    n, e = pts[:, 0], pts[:, 1]
    dist = so.distance_to_polygons(POLYS, n, e)
    inside = so.point_in_polygons(POLYS, n, e)
    hull = np.zeros(len(n), bool)
    for s1 in (-1, 1):
        for s2 in (-1, 1):
            hull |= so.point_in_polygons(POLYS, n + s1 * HALF, e + s2 * HALF)
    return dist, inside, hull


def corner_margin(pts):
    """Smallest boundary distance over the point and its four hull corners."""
    m = so.distance_to_polygons(POLYS, pts[:, 0], pts[:, 1])
    for s1 in (-1, 1):
        for s2 in (-1, 1):
            m = np.minimum(m, so.distance_to_polygons(POLYS, pts[:, 0] + s1 * HALF, pts[:, 1] + s2 * HALF))
    return m


@pytest.fixture(scope="module")
def points():
    return probe_points()


def make_env(precision):
    sc = make_scenario(64, cap=32)
    return VecMultiShipRLEnv(scenario=sc, precision=precision, device=DEV)


def test_map_index_in_use():
    info = make_env(32).map_info()
    assert info["use_index"] == 1 and info["use_cells"] == 1, info
    assert info["mixed_cells"] > 0 and info["lds_bytes"] <= 72 * 1024, info
    print(info)


def test_f64_map_predicates_exact(points):
    env = make_env(64)
    dist, inside, hull = (x.cpu().numpy() for x in env.probe_map(torch.from_numpy(points)))
    d_ref, in_ref, hull_ref = oracle_predicates(points)
    err = np.abs(dist - d_ref) / np.maximum(d_ref, 1.0)
    assert err.max() <= 1e-12, f"distance rel err {err.max():.3e}"
    bad = np.nonzero(inside != in_ref)[0]
    assert bad.size == 0, f"{bad.size} contains mismatches, e.g. {points[bad[:5]].tolist()}"
    bad = np.nonzero(hull != hull_ref)[0]
    assert bad.size == 0, f"{bad.size} hull mismatches, e.g. {points[bad[:5]].tolist()}"


def test_f32_map_predicates(points):
    env = make_env(32)
    p32 = points.astype(np.float32)
    dist, inside, hull = (x.cpu().numpy() for x in env.probe_map(torch.from_numpy(p32)))
    p = p32.astype(np.float64)          # the float32 state, evaluated in float64 by the oracle
    d_ref, in_ref, hull_ref = oracle_predicates(p)
    # float32 coordinates near 1e4 m carry ~5e-4 m of rounding: 1e-5 relative with a 10 m floor
    # (the reward uses d / 1e6, so this is 1e-10 of reward)
    err = np.abs(dist.astype(np.float64) - d_ref) / np.maximum(d_ref, 10.0)
    assert err.max() <= 1e-5, f"distance rel err {err.max():.3e}"
    bad = np.nonzero(inside != in_ref)[0]
    assert bad.size == 0, f"{bad.size} contains mismatches, e.g. {p[bad[:5]].tolist()}"
    bad_h = np.nonzero(hull != hull_ref)[0]
    assert bad_h.size == 0, f"{bad_h.size} hull mismatches, e.g. {p[bad_h[:5]].tolist()}"
    near = int((corner_margin(p) < 0.05).sum())
    print(f"float32 probes: {len(p)} points, {near} within 5 cm of a boundary (hull corners included), 0 mismatches")
