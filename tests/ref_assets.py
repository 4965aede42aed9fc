"""Stand-ins for the reference's ShipAssets / PolygonObstacle objects, built from the attribute paths
the reference's own objects hold (tests/golden/asset_paths.json, written by
tests/golden/make_golden.py --only assets from test_beds/test_policy.py-style objects).  Each stand-in
carries exactly the attributes ``compat.MultiShipRLEnv`` reads, with the reference's names, so the
drop-in is driven the way a user of the reference drives it (the reference itself never runs here
or on the GPU box)."""
from __future__ import annotations

import json
import math
import os
from types import SimpleNamespace

import numpy as np

from helpers import GOLDEN, MAP

SG_NAME = {0: "MOTOR", 1: "GEN", 2: "OFF"}


def asset_paths():
    with open(os.path.join(GOLDEN, "asset_paths.json")) as f:
        return json.load(f)


def tree(values: dict):
    """Nested SimpleNamespace objects from {"a.b.c": value}."""
    root = SimpleNamespace()
    for path, v in values.items():
        cur = root
        parts = path.split(".")
        for p in parts[:-1]:
            if not hasattr(cur, p):
                setattr(cur, p, SimpleNamespace())
            cur = getattr(cur, p)
        setattr(cur, parts[-1], v)
    return root


def polygon_obstacle(vertex_lists=MAP):
    """A PolygonObstacle as obstacle.py:98-109 builds it: shapely Polygons whose exterior.coords is
    the ring closed by its first vertex."""
    polys = [SimpleNamespace(exterior=SimpleNamespace(coords=[tuple(map(float, v)) for v in vl] + [tuple(map(float, vl[0]))]))
             for vl in vertex_lists]
    return SimpleNamespace(polygons=polys, num_obstacles=len(polys))


def fixture_assets(d, snapshot="constructed"):
    """[test, obs] ShipAssets stand-ins for an env fixture (tests/golden/env_*.npz): the recorded
    reference objects' values with the fixture's machinery mode, poses and routes."""
    ap = asset_paths()
    mode = int(d["mode"][0])
    base = ap["cases"]["PTO" if mode == 1 else "PTI"][snapshot]
    assets = []
    for t, who in enumerate(("test", "obs")):
        v = dict(base[who])
        pose = [float(x) for x in d["pose"][t]]
        for j, f in enumerate(("north", "east", "yaw_angle", "forward_speed", "sideways_speed", "yaw_rate")):
            v[f"ship_model.init_{f}"] = pose[j]
            v[f"ship_model.{f}"] = pose[j]
        nw = int(d["n_wpt"][t])
        route = [[float(a), float(b)] for a, b in d["routes"][t, :nw]]
        v["auto_pilot.navigate.init_route"] = route
        v["auto_pilot.navigate.north"] = [r[0] for r in route]
        v["auto_pilot.navigate.east"] = [r[1] for r in route]
        mm = "ship_model.ship_machinery_model.mode."
        v[mm + "shaft_generator_state"] = SG_NAME[mode]
        v[mm + "main_engine_capacity"] = float(d["mode"][1])
        v[mm + "electrical_capacity"] = float(d["mode"][2])
        a = tree(v)
        a.type_tag = who + "_ship"
        a.integrator_term, a.time_list = [], []
        assets.append(a)
    return assets


def args(sampling_frequency=7, theta=2):
    return SimpleNamespace(sampling_frequency=sampling_frequency, theta=theta)


# the set-ups the fixtures applied after reset() + init_step() (tests/golden/make_golden.py
# gen_env_cases): attribute assignments on the reference's objects
SETUPS = {
    "env_obs_arrival": [("obs", "ship_model.north", 8450.0), ("obs", "ship_model.east", 5203.0),
                        ("obs", "ship_model.forward_speed", 8.0)],
    "env_collision": [("test", "ship_model.north", 2100.0), ("test", "ship_model.east", 5300.0),
                      ("test", "ship_model.yaw_angle", 0.0), ("test", "ship_model.forward_speed", 8.0),
                      ("obs", "ship_model.north", 2200.0), ("obs", "ship_model.east", 5300.0),
                      ("obs", "ship_model.yaw_angle", np.pi), ("obs", "ship_model.forward_speed", 1.0)],
    "env_test_arrival": [("test", "auto_pilot.next_wpt", 4), ("test", "ship_model.north", 9150.0),
                         ("test", "ship_model.east", 9010.0), ("test", "ship_model.yaw_angle", 0.0),
                         ("test", "ship_model.forward_speed", 8.0)],
    "env_mechanical": [("test", "ship_model.ship_machinery_model.omega", 2001.0 * math.pi / 30 + 0.5)],
    "env_test_terrain": [("test", "ship_model.north", 1820.0), ("test", "ship_model.east", 3400.0),
                         ("test", "ship_model.yaw_angle", 0.5), ("test", "ship_model.forward_speed", 8.0)],
}


def apply_setup(env, name):
    for who, path, value in SETUPS.get(name, []):
        obj = getattr(env, who)
        parts = path.split(".")
        for p in parts[:-1]:
            obj = getattr(obj, p)
        setattr(obj, parts[-1], value)


def route_state(d, prefix, i):
    """The fixture's recorded route lists (north, east) of both ships at row i."""
    out = []
    for t in range(2):
        nw = int(d[prefix + "n_wpt"][i][t])
        end = d["routes"][t, int(d["n_wpt"][t]) - 1]
        n = [float(x) for x in d[prefix + "wpt_north"][i][t, :nw - 1]] + [float(end[0])]
        e = [float(x) for x in d[prefix + "wpt_east"][i][t, :nw - 1]] + [float(end[1])]
        out.append((n, e))
    return out

