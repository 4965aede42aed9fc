"""Float64 NumPy restatement of the ship-in-transit two-ship env step.

TEST INFRASTRUCTURE ONLY — imported by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``; never by the product path.

What it restates (reference = AndreasKing-Goks/sac-maritime-ast @ 2025-06-29):
  * ship dynamics      simulators/ship_in_transit/ship_model.py:211-306, 576-643
  * machinery          simulators/ship_in_transit/ship_engine.py:32-76, 316-395
  * controllers        simulators/ship_in_transit/controllers.py:52-62, 81-93, 138-151, 180-189,
                       298-314, 333-350
  * LOS guidance       simulators/ship_in_transit/LOS_guidance.py:88-136
  * env step/reset     RLEnv/MSRL_Env.py:147-442 (reward/failures RLEnv/MSRL_env_ex.py:453-980)
  * polygon map        simulators/ship_in_transit/obstacle.py:92-141, whose shapely calls are
                       restated from GEOS's published algorithms: Polygon.contains(Point) via
                       RayCrossingCounter::countSegment with the orientationIndexFilter +
                       exact fallback, exterior.distance(Point) via Distance::pointToSegment.
Vectorised over envs; ship axis 0 = ship under test, 1 = obstacle ship.

Pinning: tests/golden/make_golden.py runs the reference simulator itself (imported read-only
from /root/reference in the build container) and commits its outputs as fixtures;
tests/test_oracle_golden.py checks this module against every one of them.  The polygon
predicates are pinned against the reference env run with a shapely stand-in (shapely is not
installed and not version-pinned by the reference): parity of contains/distance against real
shapely is *unpinned* (see DESIGN.md).
"""
from __future__ import annotations

import numpy as np

# ------------------------------------------------------------------------------------
# configuration: the reference's NamedTuple values (test_beds/test_policy.py:94-226)
# ------------------------------------------------------------------------------------
SG_MOTOR, SG_GEN, SG_OFF = 0, 1, 2
MACH_SHAFT, MACH_SIMPLIFIED = 0, 1

DEFAULT_PARAMS = dict(
    # ShipConfiguration (test_policy.py:102-118)
    dead_weight_tonnage=3850000.0,
    coefficient_of_deadweight_to_displacement=0.7,
    bunkers=200000.0,
    ballast=200000.0,
    length_of_ship=80.0,
    width_of_ship=16.0,
    added_mass_coefficient_in_surge=0.4,
    added_mass_coefficient_in_sway=0.4,
    added_mass_coefficient_in_yaw=0.4,
    mass_over_linear_friction_coefficient_in_surge=130.0,
    mass_over_linear_friction_coefficient_in_sway=18.0,
    mass_over_linear_friction_coefficient_in_yaw=90.0,
    nonlinear_friction_coefficient_in_surge=2400.0,
    nonlinear_friction_coefficient_in_sway=4000.0,
    nonlinear_friction_coefficient_in_yaw=400.0,
    # EnvironmentConfiguration (test_policy.py:119-124)
    current_velocity_component_from_north=-2.0,
    current_velocity_component_from_east=-2.0,
    wind_speed=2.0,
    wind_direction=-np.pi / 4,
    # BaseShipModel constants (ship_model.py:123-130)
    rho_air=1.2, front_height=8.0, side_height=8.0, cx=0.5, cy=0.7, cn=0.08,
    integration_step=0.5,
    # MachinerySystemConfiguration + PTI mode (test_policy.py:132-168)
    hotel_load=200000.0,
    main_engine_capacity=0.0,
    electrical_capacity=2 * 510e3,
    shaft_generator_state=SG_MOTOR,
    rated_speed_main_engine_rpm=1000.0,
    linear_friction_main_engine=68.0,
    linear_friction_hybrid_shaft_generator=57.0,
    gear_ratio_between_main_engine_and_propeller=0.6,
    gear_ratio_between_hybrid_shaft_generator_and_propeller=0.6,
    propeller_inertia=6000.0,
    propeller_speed_to_torque_coefficient=7.5,
    propeller_diameter=3.1,
    propeller_speed_to_thrust_force_coefficient=1.7,
    rudder_angle_to_sway_force_coefficient=50e3,
    rudder_angle_to_yaw_force_coefficient=500e3,
    max_rudder_angle_degrees=30.0,
    # ThrottleControllerGains / HeadingControllerGains / LosParameters (test_policy.py:199-217)
    kp_ship_speed=7.0, ki_ship_speed=0.13, kp_shaft_speed=0.05, ki_shaft_speed=0.005,
    heading_kp=1.0, heading_kd=90.0, heading_ki=0.01,
    radius_of_acceptance=300.0, lookahead_distance=1000.0,
    los_integral_gain=0.002, integrator_windup_limit=4000.0,
    # env args + reward constants (test_policy.py:39-42; MSRL_env_ex.py:119, 557, 592, 754)
    theta=2.0, sampling_frequency=7, collision_bias=1,
    e_tolerance=1000.0, arrival_radius=200.0, shaft_rpm_max=2000.0, minimum_ship_distance=50.0,
    bias_throttle_scale=0.5, bias_throttle_max=1.1, bias_rudder_degrees=3.0,
    # specific fuel consumption coefficients (test_policy.py:162-163: Wartsila 6L26 main engine,
    # Baudouin 6M26.3 diesel generators; ship_engine.py:89-115)
    fuel_me_a=128.9, fuel_me_b=-168.9, fuel_me_c=246.8,
    fuel_dg_a=108.7, fuel_dg_b=-289.9, fuel_dg_c=324.9,
    # machinery model: ShipMachineryModel (the reference's ShipModelAST) or SimplifiedMachineryModel
    # (ship_engine.py:398-433, with ThrottleFromSpeedSetPointSimplifiedPropulsion, controllers.py:
    # 154-172, whose kp / ki are kp_ship_speed / ki_ship_speed); the reference configures no time
    # constant for it, 30 s is this library's default
    machinery_model=MACH_SHAFT, thrust_force_dynamic_time_constant=30.0,
)

# ShipModelAST.store_simulation_data keys, in order (ship_model.py:645-684)
LOG_KEYS = ("time [s]", "north position [m]", "east position [m]", "yaw angle [deg]", "rudder angle [deg]",
            "forward speed [m/s]", "sideways speed [m/s]", "yaw rate [deg/sec]", "propeller shaft speed [rpm]",
            "commanded load fraction me [-]", "commanded load fraction hsg [-]", "power me [kw]",
            "available power me [kw]", "power electrical [kw]", "available power electrical [kw]", "power [kw]",
            "propulsion power [kw]", "fuel rate me [kg/s]", "fuel rate hsg [kg/s]", "fuel rate [kg/s]",
            "fuel consumption me [kg]", "fuel consumption hsg [kg]", "fuel consumption [kg]", "motor torque [Nm]",
            "thrust force [kN]", "cross track error [m]", "heading error [deg]")
# per-step terms behind MultiShipRLEnv.reward_results (MSRL_env_ex.py:628-731, 926-964); the
# reference keeps their per-episode running sums
REWARD_TERMS = ("test reward_e_ct", "test reward_near_col", "test total_non_terminal", "obs reward_base",
                "obs reward_e_ct", "obs reward_near_col", "obs total_non_terminal", "shared total_non_terminal")

# initial-value columns (same order as SIT_INIT_* in include/sit.h)
INIT_FIELDS = ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed",
               "desired_speed", "ship_speed_i", "shaft_speed_i")

SHIP_REAL = ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed",
             "ship_speed_i", "shaft_speed_i", "heading_i", "heading_prev", "e_ct_int",
             "last_rpm", "last_e_ct", "last_power_me")
SHIP_INT = ("next_wpt", "n_wpt", "ticks", "stop")
ENV_REAL = ("sampling_dist", "eps_dist", "prev_pre_north", "prev_pre_east", "iw_north", "iw_east")
ENV_INT = ("ep_step", "event", "episodes")

ST_TEST_ENDPOINT, ST_TEST_HORIZON, ST_TEST_TERRAIN = 1 << 0, 1 << 1, 1 << 2
ST_TEST_MECHANICAL, ST_TEST_NAVIGATION, ST_TEST_BLACKOUT = 1 << 3, 1 << 4, 1 << 5
ST_OBS_ENDPOINT, ST_OBS_HORIZON, ST_OBS_TERRAIN = 1 << 6, 1 << 7, 1 << 8
ST_OBS_IW_TERMINAL, ST_OBS_NAVIGATION, ST_COLLISION = 1 << 9, 1 << 10, 1 << 11
ST_TEST_DONE, ST_OBS_DONE, ST_ROUTE_OVERFLOW = 1 << 12, 1 << 13, 1 << 31


def derive(p: dict) -> dict:
    """Constants the reference derives in its constructors, in its own operation order."""
    c = dict(p)
    dwt = p["dead_weight_tonnage"]
    payload = 0.9 * (dwt - p["bunkers"])                                   # ship_model.py:71
    lsw = dwt / p["coefficient_of_deadweight_to_displacement"] - dwt        # :72-73
    mass = lsw + payload + p["bunkers"] + p["ballast"]                      # :74
    l, w = p["length_of_ship"], p["width_of_ship"]
    i_z = mass * (l ** 2 + w ** 2) / 12                                     # :80
    c.update(mass=mass, i_z=i_z,
             x_du=mass * p["added_mass_coefficient_in_surge"],              # :206-208
             y_dv=mass * p["added_mass_coefficient_in_sway"],
             n_dr=i_z * p["added_mass_coefficient_in_yaw"])
    c["proj_area_f"] = w * p["front_height"]                                # :126
    c["proj_area_l"] = l * p["side_height"]                                 # :127
    # MachineryMode.update_available_propulsion_power (ship_engine.py:32-44); the base class
    # only calls it when hotel_load is truthy (ship_engine.py:190-193)
    me, el, hotel = p["main_engine_capacity"], p["electrical_capacity"], p["hotel_load"]
    sg = p["shaft_generator_state"]
    if not hotel:
        avail = avail_me = avail_el = 0.0
    elif sg == SG_MOTOR:
        avail, avail_me, avail_el = me + el - hotel, me, el - hotel
    elif sg == SG_GEN:
        avail, avail_me, avail_el = me - hotel, me - hotel, 0.0
    else:
        avail, avail_me, avail_el = me, me, 0.0
    c.update(avail_prop=avail, avail_me=avail_me, avail_el=avail_el)
    c["rudder_max"] = p["max_rudder_angle_degrees"] * np.pi / 180           # ship_engine.py:203
    c["bias_rudder"] = float(np.deg2rad(p["bias_rudder_degrees"]))           # MSRL_Env.py:250
    c["thrust_coeff"] = p["propeller_diameter"] ** 4 * p["propeller_speed_to_thrust_force_coefficient"]
    # SimplifiedMachineryModel (ship_engine.py:420-428)
    c["simplified"] = p.get("machinery_model", MACH_SHAFT) == MACH_SIMPLIFIED
    c["p_simpl"] = avail_me + avail_el
    c["k_thrust"] = 2160 / 790
    return c


# ------------------------------------------------------------------------------------
# polygon predicates (obstacle.py:92-141 -> GEOS algorithms)
# ------------------------------------------------------------------------------------
def _two_prod(a, b):
    """Exact product a*b = p + e (Dekker/Veltkamp split; identical to the fma form)."""
    p = a * b
    split = 134217729.0  # 2**27 + 1
    t = split * a
    ah = t - (t - a)
    al = a - ah
    t = split * b
    bh = t - (t - b)
    bl = b - bh
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return p, e


def _two_sum(a, b):
    s = a + b
    bb = s - a
    e = (a - (s - bb)) + (b - bb)
    return s, e


def _exact_sign_diff(a, b, c, d):
    """sign(a*b - c*d) computed exactly (4-term expansion)."""
    p1, e1 = _two_prod(a, b)
    p2, e2 = _two_prod(c, d)
    # grow expansion [e1, p1] by -e2 then by -p2 (Shewchuk GROW-EXPANSION)
    q, h0 = _two_sum(-e2, e1)
    q, h1 = _two_sum(q, p1)
    comps = [h0, h1, q]
    q2, g0 = _two_sum(-p2, comps[0])
    q2, g1 = _two_sum(q2, comps[1])
    q2, g2 = _two_sum(q2, comps[2])
    out = np.sign(q2)
    for g in (g2, g1, g0):
        out = np.where(out == 0, np.sign(g), out)
    return out


def orientation_index(p1x, p1y, p2x, p2y, qx, qy):
    """GEOS CGAlgorithmsDD::orientationIndex: filter, then exact sign."""
    detleft = (p1x - qx) * (p2y - qy)
    detright = (p1y - qy) * (p2x - qx)
    det = detleft - detright
    detsum = np.abs(detleft) + np.abs(detright)
    same_sign = ((detleft > 0) & (detright > 0)) | ((detleft < 0) & (detright < 0))
    uncertain = same_sign & (np.abs(det) < 1e-15 * detsum)
    out = np.sign(det)
    if np.any(uncertain):
        ex = _exact_sign_diff(p1x - qx, p2y - qy, p1y - qy, p2x - qx)
        out = np.where(uncertain, ex, out)
    return out


def point_in_polygons(polys, n, e):
    """Any polygon strictly contains Point(e, n)  (obstacle.py:126-129; GEOS RayCrossingCounter)."""
    n = np.asarray(n, dtype=np.float64)
    e = np.asarray(e, dtype=np.float64)
    shape = n.shape
    qx, qy = e.reshape(-1, 1), n.reshape(-1, 1)
    inside_any = np.zeros(qx.shape[0], dtype=bool)
    for ring in polys:
        p1x, p1y = ring[:, 0][None, :], ring[:, 1][None, :]
        p2x, p2y = np.roll(ring[:, 0], -1)[None, :], np.roll(ring[:, 1], -1)[None, :]
        left = (p1x < qx) & (p2x < qx)
        on_vertex = (qx == p2x) & (qy == p2y)
        horiz = (p1y == qy) & (p2y == qy)
        on_horiz = horiz & (np.minimum(p1x, p2x) <= qx) & (qx <= np.maximum(p1x, p2x))
        straddle = ((p1y > qy) & (p2y <= qy)) | ((p2y > qy) & (p1y <= qy))
        orient = orientation_index(p1x, p1y, p2x, p2y, qx, qy)
        on_edge = straddle & (orient == 0)
        o = np.where(p2y < p1y, -orient, orient)
        consider = ~left & ~on_vertex & ~horiz
        crossing = consider & straddle & (o > 0)
        boundary = ~left & (on_vertex | on_horiz | (consider & on_edge))
        ncross = crossing.sum(axis=1)
        inside_any |= ((ncross % 2) == 1) & ~boundary.any(axis=1)
    return inside_any.reshape(shape)


def distance_to_polygons(polys, n, e):
    """min over polygons of poly.exterior.distance(Point(e, n)) (obstacle.py:138-141;
    GEOS Distance::pointToSegment)."""
    n = np.asarray(n, dtype=np.float64)
    e = np.asarray(e, dtype=np.float64)
    shape = n.shape
    px, py = e.reshape(-1, 1), n.reshape(-1, 1)
    best = np.full(px.shape[0], np.inf)
    for ring in polys:
        ax, ay = ring[:, 0][None, :], ring[:, 1][None, :]
        bx, by = np.roll(ring[:, 0], -1)[None, :], np.roll(ring[:, 1], -1)[None, :]
        len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay)
        with np.errstate(divide="ignore", invalid="ignore"):
            r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2
            s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2
        da = np.sqrt((px - ax) * (px - ax) + (py - ay) * (py - ay))
        db = np.sqrt((px - bx) * (px - bx) + (py - by) * (py - by))
        dseg = np.abs(s) * np.sqrt(len2)
        d = np.where(len2 == 0, da, np.where(r <= 0.0, da, np.where(r >= 1.0, db, dseg)))
        best = np.minimum(best, d.min(axis=1))
    return best.reshape(shape)


# ------------------------------------------------------------------------------------
# Philox4x32-10 (Salmon et al., SC'11; Random123) for the synthetic sampler
# ------------------------------------------------------------------------------------
_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF
SAMPLER_TAG = 0x5A4D


def philox4x32_10(ctr, key):
    c = [np.asarray(x, dtype=np.uint64) & _MASK for x in ctr]
    k0 = np.asarray(key[0], dtype=np.uint64) & _MASK
    k1 = np.asarray(key[1], dtype=np.uint64) & _MASK
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & _MASK
            k1 = (k1 + _W1) & _MASK
        p0 = np.uint64(_M0) * c[0]
        p1 = np.uint64(_M1) * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(_MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(_MASK)
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
    return [x.astype(np.uint32) for x in c]


def sampler_uniform(seed, env_id, event):
    """53-bit uniform in [0, 1) from Philox(key=seed, ctr=(env_id, event, TAG, 0))."""
    env_id = np.asarray(env_id, dtype=np.uint64)
    event = np.asarray(event, dtype=np.uint64)
    seed = int(seed)
    key = (np.uint64(seed & _MASK), np.uint64((seed >> 32) & _MASK))
    x = philox4x32_10((env_id & np.uint64(_MASK), event & np.uint64(_MASK),
                       np.uint64(SAMPLER_TAG), np.uint64(0)), key)
    hi = (x[0] >> np.uint32(5)).astype(np.float64)
    lo = (x[1] >> np.uint32(6)).astype(np.float64)
    return (hi * 67108864.0 + lo) * (1.0 / 9007199254740992.0)


POLICY_TAG = 0x504F


def sampler_normal(seed, env_id, event):
    """Standard normal from Philox(key=seed, ctr=(env_id, event, 0x504F, 0)) by Box-Muller:
    u1 in (0, 1], u2 in [0, 1) from 53 bits each (the policy's reparameterisation noise)."""
    env_id = np.asarray(env_id, dtype=np.uint64)
    event = np.asarray(event, dtype=np.uint64)
    seed = int(seed)
    key = (np.uint64(seed & _MASK), np.uint64((seed >> 32) & _MASK))
    x = philox4x32_10((env_id & np.uint64(_MASK), event & np.uint64(_MASK),
                       np.uint64(POLICY_TAG), np.uint64(0)), key)
    u1 = ((x[0] >> np.uint32(5)).astype(np.float64) * 67108864.0
          + (x[1] >> np.uint32(6)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)
    u2 = ((x[2] >> np.uint32(5)).astype(np.float64) * 67108864.0
          + (x[3] >> np.uint32(6)).astype(np.float64)) * (1.0 / 9007199254740992.0)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


# ------------------------------------------------------------------------------------
# the env
# ------------------------------------------------------------------------------------
class OracleEnvs:
    """N two-ship MultiShipRLEnv instances, float64 throughout.

    routes: float64[n_env, 2, cap, 2] (north, east); n_wpt: int[n_env, 2];
    init: float64[n_env, 2, len(INIT_FIELDS)]; polys: list of float64[m, 2] (east, north).
    """

    def __init__(self, params, routes, n_wpt, init, polys, cap=None):
        self.c = derive(params)
        routes = np.asarray(routes, dtype=np.float64)
        self.n_env = routes.shape[0]
        self.cap = int(cap if cap is not None else routes.shape[2])
        n_wpt = np.asarray(n_wpt, dtype=np.int64)
        self.n_wpt0 = n_wpt.T.copy()                                  # [2, n_env]
        ar = np.arange(self.n_env)
        self.end_n = np.stack([routes[ar, t, n_wpt[:, t] - 1, 0] for t in (0, 1)])
        self.end_e = np.stack([routes[ar, t, n_wpt[:, t] - 1, 1] for t in (0, 1)])
        self.start_n = routes[:, :, 0, 0].T.copy()
        self.start_e = routes[:, :, 0, 1].T.copy()
        self.init = np.asarray(init, dtype=np.float64).transpose(1, 2, 0).copy()  # [2, NF, n_env]
        self.polys = [np.asarray(p, dtype=np.float64) for p in polys]
        allv = np.concatenate(self.polys)
        # PolygonObstacle.map_boundaries (obstacle.py:111-124): vertices are (east, north)
        self.min_east, self.max_east = allv[:, 0].min(), allv[:, 0].max()
        self.min_north, self.max_north = allv[:, 1].min(), allv[:, 1].max()
        # reward_function_params (MSRL_Env.py:119-128) from the obstacle ship's route
        ab_n = self.end_n[1] - self.start_n[1]
        ab_e = self.end_e[1] - self.start_e[1]
        self.ab_len = np.sqrt(ab_n ** 2 + ab_e ** 2) / self.c["sampling_frequency"]
        self.ab_alpha = np.arctan2(ab_e, ab_n)
        # construction-time observation, float32 (MSRL_Env.py:88-91)
        i = self.init
        self.initial_state = np.zeros((self.n_env, 10), dtype=np.float32)
        self.initial_state[:, 0], self.initial_state[:, 1], self.initial_state[:, 2] = i[0, 0], i[0, 1], i[0, 2]
        self.initial_state[:, 6], self.initial_state[:, 7], self.initial_state[:, 8] = i[1, 0], i[1, 1], i[1, 2]
        self.tab_n = np.zeros((2, self.cap, self.n_env))
        self.tab_e = np.zeros((2, self.cap, self.n_env))
        for t in (0, 1):
            for e in range(self.n_env):
                k = n_wpt[e, t] - 1
                self.tab_n[t, :k, e] = routes[e, t, :k, 0]
                self.tab_e[t, :k, e] = routes[e, t, :k, 1]
        self.s = {}
        self.restart()

    # ---------------- state ----------------
    def restart(self):
        """Construction-time state (ship_model.py:102-116, ship_engine.py:327, controllers.py:45-79)."""
        n = self.n_env
        i = self.init
        s = {}
        for name in SHIP_REAL:
            s[name] = np.zeros((2, n))
        for j, name in enumerate(("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed")):
            s[name] = i[:, j].copy()
        s["ship_speed_i"] = i[:, INIT_FIELDS.index("ship_speed_i")].copy()
        s["shaft_speed_i"] = i[:, INIT_FIELDS.index("shaft_speed_i")].copy()
        s["next_wpt"] = np.ones((2, n), dtype=np.int64)
        s["n_wpt"] = self.n_wpt0.copy()
        s["ticks"] = np.zeros((2, n), dtype=np.int64)
        s["stop"] = np.zeros((2, n), dtype=np.int64)
        for name in ENV_REAL:
            s[name] = np.zeros(n)
        for name in ENV_INT:
            s[name] = np.zeros(n, dtype=np.int64)
        s["last_obs"] = self.initial_state.T.astype(np.float64).copy()   # sampler's `state`
        # logging-only machinery state: accumulated fuel (ship_engine.py:283-289) and the last
        # logged row (store_last_simulation_data repeats it on the obstacle's stop path)
        for name in ("fuel_me", "fuel_el", "fuel"):
            s[name] = np.zeros((2, n))
        s["last_log"] = np.zeros((len(LOG_KEYS), n))          # the obstacle ship's last row
        self.s = s
        self.log = None          # list of per-step rows when logging (start_log)

    # ---------------- trajectory log (ship_model.py:645-700) ----------------
    def start_log(self):
        """Record the reference's simulation_results rows ([2, 27] per env and step) and the
        reward terms from the next step on; fuel accumulates over logged steps."""
        self.log = {"ship": [], "reward": []}

    def _distribute_load(self, thr):
        """MachineryMode.distribute_load(load_perc=thr, hotel_load) (ship_engine.py:46-76)."""
        c = self.c
        me, el, hotel = c["main_engine_capacity"], c["electrical_capacity"], c["hotel_load"]
        total = thr * c["avail_prop"]
        sg = c["shaft_generator_state"]
        with np.errstate(divide="ignore", invalid="ignore"):
            if sg == SG_MOTOR:
                load_me = np.minimum(total, me)
                load_el = total + hotel - load_me
                lp_el = load_el / el
                lp_me = np.zeros_like(total) if me == 0 else load_me / me
            elif sg == SG_GEN:
                load_el = np.full_like(total, min(hotel, el))
                load_me = total + hotel - load_el
                lp_me = load_me / me
                lp_el = np.zeros_like(total) if el == 0 else load_el / el
            else:
                load_me = total
                load_el = np.full_like(total, hotel)
                lp_me = load_me / me
                lp_el = load_el / el
        return load_me, load_el, lp_me, lp_el

    def _log_row(self, t, thr, rudder, ect, psi_ref, pre, m):
        """store_simulation_data(load_perc=thr, rudder, e_ct, e_psi) from the pre-integration
        state `pre`; accumulates fuel (BaseMachineryModel.fuel_consumption) where m is set."""
        c, s = self.c, self.s
        dt = c["integration_step"]
        load_me, load_el, lp_me, lp_el = self._distribute_load(thr)

        def spec(x, a, b, cc):                                    # spec_fuel_cons (:257-261)
            return (a * x ** 2 + b * x + cc) / 3.6e9
        with np.errstate(invalid="ignore"):
            rate_me = np.where(load_me == 0, 0.0, load_me * spec(lp_me, c["fuel_me_a"], c["fuel_me_b"], c["fuel_me_c"]))
            rate_el = np.where(lp_el == 0, 0.0, load_el * spec(lp_el, c["fuel_dg_a"], c["fuel_dg_b"], c["fuel_dg_c"]))
        s["fuel_me"][t] = np.where(m, s["fuel_me"][t] + rate_me * dt, s["fuel_me"][t])
        s["fuel_el"][t] = np.where(m, s["fuel_el"][t] + rate_el * dt, s["fuel_el"][t])
        s["fuel"][t] = np.where(m, s["fuel"][t] + (rate_me + rate_el) * dt, s["fuel"][t])
        w = pre["shaft_speed"]
        torque = np.minimum(thr * c["avail_me"] / (w + 0.1), c["avail_me"] / 5 * np.pi / 30)   # ship_engine.py:369-376
        thrust = c["thrust_coeff"] * w * np.abs(w)
        if c["simplified"]:
            # no reference row (store_simulation_data reads the shaft speed, which the simplified
            # model lacks): shaft speed and torque 0, thrust force from the thrust state
            torque, thrust = np.zeros_like(w), w
        row = np.stack([
            s["ticks"][t] * dt, pre["north"], pre["east"], pre["yaw"] * 180 / np.pi, rudder * 180 / np.pi,
            pre["surge"], pre["sway"], pre["yaw_rate"] * 180 / np.pi, self._rpm(w), lp_me, lp_el,
            load_me / 1000, np.full_like(thr, c["main_engine_capacity"] / 1000), load_el / 1000,
            np.full_like(thr, c["electrical_capacity"] / 1000), (load_el + load_me) / 1000,
            (thr * c["avail_prop"]) / 1000, rate_me, rate_el, rate_me + rate_el,
            s["fuel_me"][t], s["fuel_el"][t], s["fuel"][t], torque,
            thrust / 1000, ect,
            np.abs(pre["yaw"] - psi_ref)])                          # get_heading_error: radians (label says deg)
        return row

    def get_state(self):
        out = {k: v.copy() for k, v in self.s.items()}
        out["wpt_north"] = self.tab_n.copy()
        out["wpt_east"] = self.tab_e.copy()
        return out

    def set_state(self, st):
        for k in self.s:
            if k in st:
                self.s[k] = np.asarray(st[k]).astype(self.s[k].dtype).copy()
        if "wpt_north" in st:
            self.tab_n = np.asarray(st["wpt_north"], dtype=np.float64).copy()
            self.tab_e = np.asarray(st["wpt_east"], dtype=np.float64).copy()

    def _rpm(self, w):
        """Observed shaft speed omega * 30 / pi (ship_model.py:652); SimplifiedMachineryModel has no
        shaft (its state slot holds the thrust force): 0."""
        return np.zeros_like(w) if self.c["simplified"] else w * 30 / np.pi

    def _wpt(self, t, idx):
        ar = np.arange(self.n_env)
        last = idx == self.s["n_wpt"][t] - 1
        j = np.clip(idx, 0, self.cap - 1)
        wn = np.where(last, self.end_n[t], self.tab_n[t, j, ar])
        we = np.where(last, self.end_e[t], self.tab_e[t, j, ar])
        return wn, we

    # ---------------- one ship: guidance + control ----------------
    def _guidance_control(self, t, m, trace=None):
        """rudder_angle_from_sampled_route (controllers.py:306-314) and throttle (:138-143).
        Updates state only where mask m is set.  Returns (rudder, throttle, |e_ct|)."""
        c, s = self.c, self.s
        n, e, psi, u = (s[f][t].copy() for f in ("north", "east", "yaw", "surge"))
        k = s["next_wpt"][t].copy()
        # NavigationSystem.next_wpt (LOS_guidance.py:88-103)
        wn, we = self._wpt(t, k)
        adv = ((wn - n) ** 2 + (we - e) ** 2 <= c["radius_of_acceptance"] ** 2) & (s["n_wpt"][t] > k + 1)
        k = np.where(adv, k + 1, k)
        # NavigationSystem.los_guidance (LOS_guidance.py:105-121)
        pn, pe = self._wpt(t, k - 1)
        nn, ne_ = self._wpt(t, k)
        alpha = np.arctan2(ne_ - pe, nn - pn)
        ect = -(n - pn) * np.sin(alpha) + (e - pe) * np.cos(alpha)
        ect_abs = np.abs(ect)
        r = c["lookahead_distance"]
        ect = np.where(ect ** 2 >= r ** 2, 0.99 * r, ect)
        delta = np.sqrt(r ** 2 - ect ** 2)
        ei = s["e_ct_int"][t]
        ei = np.where(np.abs(ei + ect / delta) <= c["integrator_windup_limit"], ei + ect / delta, ei)
        chi = np.arctan(-ect / delta - ei * c["los_integral_gain"])
        psi_ref = alpha + chi
        # PidController.pid_ctrl via rudder_angle_from_heading_setpoint (controllers.py:81-93, 180-189)
        dt = c["integration_step"]
        err = psi_ref - psi
        d_err = (err - s["heading_prev"][t]) / dt
        hi = s["heading_i"][t] + err * dt
        out = err * c["heading_kp"] + d_err * c["heading_kd"] + hi * c["heading_ki"]
        rudder = np.maximum(-c["rudder_max"], np.minimum(-out, c["rudder_max"]))
        # EngineThrottleFromSpeedSetPoint.throttle: measured_shaft_speed := forward speed
        # (MSRL_Env.py:235-239; controllers.py:52-62, no saturation)
        e1 = self.init[t, INIT_FIELDS.index("desired_speed")] - u
        i1 = s["ship_speed_i"][t] + e1 * dt
        w_des = e1 * c["kp_ship_speed"] + i1 * c["ki_ship_speed"]
        if c["simplified"]:
            # ThrottleFromSpeedSetPointSimplifiedPropulsion.throttle (controllers.py:170-172)
            i2 = s["shaft_speed_i"][t]
            thr = np.maximum(0.0, np.minimum(w_des, 1.1))
        else:
            e2 = w_des - u
            i2 = s["shaft_speed_i"][t] + e2 * dt
            thr = e2 * c["kp_shaft_speed"] + i2 * c["ki_shaft_speed"]
        if trace is not None:
            trace["heading_ref"] = psi_ref
        s["next_wpt"][t] = np.where(m, k, s["next_wpt"][t])
        s["e_ct_int"][t] = np.where(m, ei, s["e_ct_int"][t])
        s["heading_prev"][t] = np.where(m, err, s["heading_prev"][t])
        s["heading_i"][t] = np.where(m, hi, s["heading_i"][t])
        s["ship_speed_i"][t] = np.where(m, i1, s["ship_speed_i"][t])
        s["shaft_speed_i"][t] = np.where(m, i2, s["shaft_speed_i"][t])
        return rudder, thr, ect_abs

    def _power_me_kw(self, thr):
        """distribute_load(...).load_on_main_engine / 1000 (ship_engine.py:46-76; ship_model.py:659-662)."""
        c = self.c
        total = thr * c["avail_prop"]
        sg = c["shaft_generator_state"]
        if sg == SG_MOTOR:
            load_me = np.minimum(total, c["main_engine_capacity"])
        elif sg == SG_GEN:
            load_el = min(c["hotel_load"], c["electrical_capacity"])
            load_me = total + c["hotel_load"] - load_el
        else:
            load_me = total
        return load_me / 1000

    # ---------------- one ship: dynamics + Euler step ----------------
    def _dynamics(self, t, thr, rudder, m):
        """update_differentials + integrate_differentials (ship_model.py:624-643)."""
        c, s = self.c, self.s
        n, e, psi, u, v, r, w = (s[f][t].copy() for f in
                                 ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed"))
        cps, sps = np.cos(psi), np.sin(psi)
        # three_dof_kinematics (ship_model.py:233-250)
        d_n = cps * u - sps * v
        d_e = sps * u + cps * v
        d_psi = r
        if c["simplified"]:
            # SimplifiedMachineryModel.update_thrust_force (ship_engine.py:423-428); w is the thrust
            power = thr * c["p_simpl"]
            d_w = (-c["k_thrust"] * w + power) / c["thrust_force_dynamic_time_constant"]
            thrust = w
        else:
            # ShipMachineryModel.update_shaft_equation (ship_engine.py:355-395)
            tq_me = np.minimum(thr * c["avail_me"] / (w + 0.1), c["avail_me"] / 5 * np.pi / 30)
            tq_hsg = np.minimum(thr * c["avail_el"] / (w + 0.1), c["avail_el"] / 5 * np.pi / 30)
            eq_me = (tq_me - c["linear_friction_main_engine"] * w) / c["gear_ratio_between_main_engine_and_propeller"]
            eq_hsg = (tq_hsg - c["linear_friction_hybrid_shaft_generator"] * w) / \
                c["gear_ratio_between_hybrid_shaft_generator_and_propeller"]
            d_w = (eq_me + eq_hsg - c["propeller_speed_to_torque_coefficient"] * w ** 2) / c["propeller_inertia"]
            thrust = c["thrust_coeff"] * w * np.abs(w)                       # ship_engine.py:363-366
        # ShipModelAST.three_dof_kinetics (ship_model.py:576-606)
        vcn, vce = c["current_velocity_component_from_north"], c["current_velocity_component_from_east"]
        vc_u = cps * vcn + sps * vce              # inv(rotation()) . vel_c
        vc_v = -sps * vcn + cps * vce
        u_r, v_r = u - vc_u, v - vc_v
        # rudder (ship_model.py:608-622)
        f_rv = -c["rudder_angle_to_sway_force_coefficient"] * rudder * (u - vc_u)
        f_rr = -c["rudder_angle_to_yaw_force_coefficient"] * rudder * (u - vc_u)
        # get_wind_force (ship_model.py:211-231)
        uw = c["wind_speed"] * np.cos(c["wind_direction"] - psi)
        vw = c["wind_speed"] * np.sin(c["wind_direction"] - psi)
        u_rw, v_rw = uw - u, vw - v
        gamma = -np.arctan2(v_rw, u_rw)
        w2 = u_rw ** 2 + v_rw ** 2
        q = 0.5 * c["rho_air"] * w2
        tau_u = q * (-c["cx"] * np.cos(gamma)) * c["proj_area_f"]
        tau_v = q * (c["cy"] * np.sin(gamma)) * c["proj_area_l"]
        tau_n = q * (c["cn"] * np.sin(2 * gamma)) * c["proj_area_l"] * c["length_of_ship"]
        mass, x_du, y_dv = c["mass"], c["x_du"], c["y_dv"]
        # coriolis_matrix . vel  (x_g = 0)
        crb0 = -(mass * v) * r
        crb1 = (mass * u) * r
        crb2 = (mass * v) * u + (-(mass * u)) * v
        # coriolis_added_mass_matrix(u_r, v_r) . (vel - v_c)
        ca0 = (y_dv * v_r) * r
        ca1 = (-(x_du * u_r)) * r
        ca2 = (-(y_dv * v_r)) * u_r + (x_du * u_r) * v_r
        # (linear + non_linear damping) . (vel - v_c)
        dd0 = (mass / c["mass_over_linear_friction_coefficient_in_surge"]
               + c["nonlinear_friction_coefficient_in_surge"] * u) * u_r
        dd1 = (mass / c["mass_over_linear_friction_coefficient_in_sway"]
               + c["nonlinear_friction_coefficient_in_sway"] * v) * v_r
        dd2 = (c["i_z"] / c["mass_over_linear_friction_coefficient_in_yaw"]
               + c["nonlinear_friction_coefficient_in_yaw"] * r) * r
        f0 = -crb0 - ca0 - dd0 + tau_u + thrust
        f1 = -crb1 - ca1 - dd1 + tau_v + f_rv
        f2 = -crb2 - ca2 - dd2 + tau_n + f_rr
        # inv(mass_matrix()) is diagonal for x_g = 0
        d_u = (1.0 / (mass + x_du)) * f0
        d_v = (1.0 / (mass + y_dv)) * f1
        d_r = (1.0 / (c["i_z"] + c["n_dr"])) * f2
        # integrate_differentials (EulerInt.integrate, utils.py:50-53)
        dt = c["integration_step"]
        for name, x, dx in (("north", n, d_n), ("east", e, d_e), ("yaw", psi, d_psi),
                            ("surge", u, d_u), ("sway", v, d_v), ("yaw_rate", r, d_r),
                            ("shaft_speed", w, d_w)):
            s[name][t] = np.where(m, x + dx * dt, x)
        return dict(d_north=d_n, d_east=d_e, d_yaw=d_psi, d_surge=d_u, d_sway=d_v,
                    d_yaw_rate=d_r, d_shaft_speed=d_w, thrust=thrust)

    # ---------------- env API ----------------
    def sim_step(self, t, bias=False):
        """One simulator step of ship type t for all envs, as MSRL_Env.obs_step's non-stop path
        (MSRL_Env.py:347-375), or test_step's (:223-262) when bias is set; no reward."""
        c, s = self.c, self.s
        allm = np.ones(self.n_env, bool)
        tr = {}
        rudder, thr, ect = self._guidance_control(t, allm, tr)
        if bias:
            thr = np.clip(thr * c["bias_throttle_scale"], 0.0, c["bias_throttle_max"])
            rudder = np.clip(rudder + c["bias_rudder"], -c["rudder_max"], c["rudder_max"])
        rpm = self._rpm(s["shaft_speed"][t])
        pme = self._power_me_kw(thr)
        s["last_rpm"][t], s["last_e_ct"][t], s["last_power_me"][t] = rpm, ect, pme
        pre = {k: s[k][t].copy() for k in ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed")}
        log = self._log_row(t, thr, rudder, ect, tr["heading_ref"], pre, allm)
        d = self._dynamics(t, thr, rudder, allm)
        s["ticks"][t] += 1
        return dict(rudder=rudder, throttle=thr, heading_ref=tr["heading_ref"], e_ct=ect, rpm=rpm,
                    power_me=pme, log=log, **d)

    def reset(self, mask=None):
        """MultiShipRLEnv.reset (MSRL_Env.py:147-188): pose/velocity/time/route/LOS state back to
        construction values; shaft speed and PI/PID integrators are kept (Q6)."""
        m = np.ones(self.n_env, bool) if mask is None else np.asarray(mask, bool)
        s = self.s
        for j, name in enumerate(("north", "east", "yaw", "surge", "sway", "yaw_rate")):
            s[name][:, m] = self.init[:, j][:, m]
        s["e_ct_int"][:, m] = 0.0
        s["next_wpt"][:, m] = 1
        s["n_wpt"][:, m] = self.n_wpt0[:, m]
        s["ticks"][:, m] = 0
        s["stop"][:, m] = 0
        for name in ("sampling_dist", "eps_dist"):
            s[name][m] = 0.0
        s["ep_step"][m] = 0
        s["last_obs"][:, m] = self.initial_state[m].T
        return self.initial_state.copy()

    def init_step(self, mask=None):
        """MultiShipRLEnv.init_step (MSRL_Env.py:190-217): no store, no time advance, no bias."""
        m = np.ones(self.n_env, bool) if mask is None else np.asarray(mask, bool)
        for t in (0, 1):
            rudder, thr, _ = self._guidance_control(t, m)
            self._dynamics(t, thr, rudder, m)

    def step(self, action_ne, sac_update, init, trace=None):
        """MultiShipRLEnv.step (MSRL_Env.py:404-442) + reward_function (MSRL_env_ex.py:906-980)."""
        c, s = self.c, self.s
        n_env = self.n_env
        allm = np.ones(n_env, bool)
        action_ne = np.asarray(action_ne, dtype=np.float64).reshape(n_env, 2)
        sac_update = np.asarray(sac_update, bool).reshape(n_env)
        init = np.asarray(init, bool).reshape(n_env)
        status = np.zeros(n_env, dtype=np.uint32)

        # ---- test_step (MSRL_Env.py:219-285) ----
        tr0 = {}
        rudder, thr, ect0 = self._guidance_control(0, allm, tr0)
        if c["collision_bias"]:  # is_collision_imminent on the all-zero next_states: always True (Q1)
            thr = np.clip(thr * c["bias_throttle_scale"], 0.0, c["bias_throttle_max"])
            rudder = np.clip(rudder + c["bias_rudder"], -c["rudder_max"], c["rudder_max"])
        rpm0 = self._rpm(s["shaft_speed"][0])
        pme0 = self._power_me_kw(thr)
        s["last_rpm"][0], s["last_e_ct"][0], s["last_power_me"][0] = rpm0, ect0, pme0
        if self.log is not None:       # store_simulation_data before update/integrate (:256-260)
            pre0 = {k: s[k][0].copy() for k in ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed")}
            log0 = self._log_row(0, thr, rudder, ect0, tr0["heading_ref"], pre0, allm)
        d0 = self._dynamics(0, thr, rudder, allm)
        s["ticks"][0] += 1
        if trace is not None:
            trace.update(test_rudder=rudder, test_throttle=thr, **{"test_" + k: v for k, v in d0.items()})

        # ---- obs_step (MSRL_Env.py:287-402) ----
        stopped = s["stop"][1].astype(bool)
        run = ~stopped
        ins = run & sac_update
        # update_route: insert at index -1 (controllers.py:298-303)
        nw = s["n_wpt"][1]
        fits = nw < self.cap
        do_ins = ins & fits
        idx = np.where(do_ins, nw - 1, 0)
        ar = np.arange(n_env)
        self.tab_n[1, idx[do_ins], ar[do_ins]] = action_ne[do_ins, 0]
        self.tab_e[1, idx[do_ins], ar[do_ins]] = action_ne[do_ins, 1]
        s["n_wpt"][1] = np.where(do_ins, nw + 1, nw)
        status |= np.where(ins & ~fits, np.uint32(ST_ROUTE_OVERFLOW), np.uint32(0))
        s["sampling_dist"] = np.where(ins, 0.0, s["sampling_dist"])
        pre_n, pre_e = s["north"][1].copy(), s["east"][1].copy()
        tr1 = {}
        rudder1, thr1, ect1 = self._guidance_control(1, run, tr1)
        if self.log is not None:       # store_simulation_data / store_last_simulation_data (:294, :367)
            pre1 = {k: s[k][1].copy() for k in ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed")}
            row1 = self._log_row(1, thr1, rudder1, ect1, tr1["heading_ref"], pre1, run)
            last = s["last_log"].copy()
            last[0] = s["ticks"][1] * c["integration_step"]
            log1 = np.where(run[None, :], row1, last)
            s["last_log"] = log1
        rpm1 = self._rpm(s["shaft_speed"][1])
        pme1 = self._power_me_kw(thr1)
        s["last_rpm"][1] = np.where(run, rpm1, s["last_rpm"][1])
        s["last_e_ct"][1] = np.where(run, ect1, s["last_e_ct"][1])
        s["last_power_me"][1] = np.where(run, pme1, s["last_power_me"][1])
        d1 = self._dynamics(1, thr1, rudder1, run)
        # travelled distance from the last two stored pre-integration positions (:392-397)
        acc = run & ~init
        dist = np.sqrt((pre_n - s["prev_pre_north"]) ** 2 + (pre_e - s["prev_pre_east"]) ** 2)
        s["eps_dist"] = np.where(acc, s["eps_dist"] + dist, s["eps_dist"])
        s["sampling_dist"] = np.where(acc, s["sampling_dist"] + dist, s["sampling_dist"])
        s["prev_pre_north"] = np.where(run, pre_n, s["prev_pre_north"])
        s["prev_pre_east"] = np.where(run, pre_e, s["prev_pre_east"])
        s["ticks"][1] += np.where(stopped, 2, 1)          # stop path advances time twice (Q10)
        if trace is not None:
            trace.update(obs_rudder=rudder1, obs_throttle=thr1, **{"obs_" + k: v for k, v in d1.items()})

        ns = np.zeros((n_env, 10))
        ns[:, 0], ns[:, 1], ns[:, 2] = s["north"][0], s["east"][0], s["yaw"][0]
        ns[:, 3], ns[:, 4], ns[:, 5] = rpm0, ect0, pme0
        ns[:, 6], ns[:, 7], ns[:, 8] = s["north"][1], s["east"][1], s["yaw"][1]
        ns[:, 9] = s["last_e_ct"][1]
        reward, done, st = self._reward(ns, action_ne)
        if self.log is not None:
            self.log["ship"].append(np.stack([log0, log1]))          # [2, 27, n_env]
            self.log["reward"].append(self._terms)                   # [8, n_env]
        status |= st
        s["ep_step"] += 1
        s["last_obs"] = ns.T.copy()
        return ns, reward, done, status

    # ---------------- reward_function (MSRL_env_ex.py:906-980) ----------------
    def _outside(self, n, e, margin):
        """is_pos_outside_horizon / is_route_outside_horizon (MSRL_env_ex.py:460-488, 517-542)."""
        return ((n < self.min_north + margin) | (n > self.max_north - margin)
                | (e < self.min_east + margin) | (e > self.max_east - margin))

    def _hull_in_terrain(self, n, e):
        """is_pos_inside_obstacles: 4 corners of a +-l/2 square (MSRL_env_ex.py:490-515)."""
        h = self.c["length_of_ship"] / 2
        hit = np.zeros(n.shape, bool)
        for cn_, ce_ in ((n - h, e - h), (n - h, e + h), (n + h, e - h), (n + h, e + h)):
            hit |= point_in_polygons(self.polys, cn_, ce_)
        return hit

    def _reward(self, ns, action_ne):
        c, s = self.c, self.s
        tol = c["e_tolerance"]
        maxn = self.max_north
        tn, te, t_rpm, t_ect, t_pme = ns[:, 0], ns[:, 1], ns[:, 3], ns[:, 4], ns[:, 5]
        on, oe, o_ect = ns[:, 6], ns[:, 7], ns[:, 9]
        st = np.zeros(self.n_env, dtype=np.uint32)
        margin = c["length_of_ship"] / 2
        # test ship non-terminal (:628-664)
        d_t = distance_to_polygons(self.polys, tn, te)
        r_ntt = np.abs(t_ect) / tol + (1 - d_t / maxn) / 100
        # test ship terminal (:734-809): first satisfied predicate wins the reward
        stop = s["stop"][0].astype(bool)
        rt = np.zeros(self.n_env)
        done_t = np.zeros(self.n_env, bool)
        preds = [
            (np.sqrt((tn - self.end_n[0]) ** 2 + (te - self.end_e[0]) ** 2) <= c["arrival_radius"], 0.0, ST_TEST_ENDPOINT),
            (self._outside(tn, te, margin), 0.0, ST_TEST_HORIZON),
            (self._hull_in_terrain(tn, te), 1000.0, ST_TEST_TERRAIN),
            (np.abs(t_rpm) > c["shaft_rpm_max"], 1000.0, ST_TEST_MECHANICAL),
            (np.abs(t_ect) > tol, 1000.0, ST_TEST_NAVIGATION),
            (t_pme > c["main_engine_capacity"] / 1000, 1000.0, ST_TEST_BLACKOUT),
        ]
        for hit, rew, bit in preds:
            rt = np.where(hit & ~stop, rt + rew, rt)
            stop |= hit
            done_t |= hit
            st |= np.where(hit, np.uint32(bit), np.uint32(0))
        s["stop"][0] = stop.astype(np.int64)
        # obstacle ship non-terminal (:666-710), gated on the stop flag before this call
        ostop = s["stop"][1].astype(bool)
        d_o = distance_to_polygons(self.polys, on, oe)
        r_nto = np.where(ostop, 0.0,
                         0.1 + (-(np.abs(o_ect) / tol)) / 100
                         + (-(1 - d_o / maxn)) / 100)
        terms_obs = (np.where(ostop, 0.0, 0.1), np.where(ostop, 0.0, -(np.abs(o_ect) / tol) / 100),
                     np.where(ostop, 0.0, -(1 - d_o / maxn) / 100), r_nto)
        # obstacle ship terminal (:811-881)
        ro = np.zeros(self.n_env)
        done_o = np.zeros(self.n_env, bool)
        arrive = np.sqrt((on - self.end_n[1]) ** 2 + (oe - self.end_e[1]) ** 2) <= c["arrival_radius"]
        ostop |= arrive
        st |= np.where(arrive, np.uint32(ST_OBS_ENDPOINT), np.uint32(0))
        hz = self._outside(on, oe, margin)
        ostop |= hz
        done_o |= hz
        st |= np.where(hz, np.uint32(ST_OBS_HORIZON), np.uint32(0))
        terr = self._hull_in_terrain(on, oe)                  # done, but no stop flag (Q12)
        ro = np.where(terr & ~ostop, ro - 1000.0, ro)
        done_o |= terr
        st |= np.where(terr, np.uint32(ST_OBS_TERRAIN), np.uint32(0))
        iw_n, iw_e = action_ne[:, 0], action_ne[:, 1]      # converted_action even without a sample (Q11)
        iw = self._outside(iw_n, iw_e, 0.0) | point_in_polygons(self.polys, iw_n, iw_e)
        ro = np.where(iw & ~ostop, ro - 1000.0, ro)
        ostop |= iw
        done_o |= iw
        st |= np.where(iw, np.uint32(ST_OBS_IW_TERMINAL), np.uint32(0))
        nav = (np.abs(o_ect) > tol) | (s["sampling_dist"] > self.ab_len * c["theta"])
        ro = np.where(nav & ~ostop, ro - 1000.0, ro)
        ostop |= nav
        done_o |= nav
        st |= np.where(nav, np.uint32(ST_OBS_NAVIGATION), np.uint32(0))
        # shared non-terminal (:712-731): uses the stop flag as just updated
        dist = np.sqrt((tn - on) ** 2 + (te - oe) ** 2)
        r_snt = np.where(ostop, 0.0, (1 - dist / maxn) / 1000)
        self._terms = np.stack([np.abs(t_ect) / tol, (1 - d_t / maxn) / 100, r_ntt, *terms_obs, r_snt])
        # shared terminal (:883-904)
        coll = (tn - on) ** 2 + (te - oe) ** 2 < c["minimum_ship_distance"] ** 2
        rs = np.where(coll, 2000.0, 0.0)
        st |= np.where(coll, np.uint32(ST_COLLISION), np.uint32(0))
        stop_t = s["stop"][0].astype(bool) | coll
        ostop |= coll
        s["stop"][0] = stop_t.astype(np.int64)
        s["stop"][1] = ostop.astype(np.int64)
        st |= np.where(done_t, np.uint32(ST_TEST_DONE), np.uint32(0))
        st |= np.where(done_o, np.uint32(ST_OBS_DONE), np.uint32(0))
        reward = r_ntt + rt + r_nto + ro + r_snt + rs
        done = done_t | done_o | coll
        return reward, done, st

    # ---------------- synthetic sampler rollout ----------------
    def sampler_actions(self, seed, env_id_offset=0):
        """Decide this step's (iw, sac_update, init, angle) for every env and advance counters."""
        s = self.s
        init = s["ep_step"] == 0
        stopped = s["stop"][1].astype(bool)
        sample = init | ((s["sampling_dist"] >= self.ab_len) & ~stopped)
        env_id = np.arange(self.n_env, dtype=np.uint64) + np.uint64(env_id_offset)
        u = sampler_uniform(seed, env_id, s["event"])
        act_n = u * 2.0 - 1.0                    # mode-0 action U[-1, 1] (uniform_policy.py:20-22)
        a = act_n * (np.pi / 6.0)
        self.last_action_n = np.where(sample, act_n, np.nan)   # the SAC action of the event
        iw_n = s["north"][1] + self.ab_len * np.cos(self.ab_alpha + a)
        iw_e = s["east"][1] + self.ab_len * np.sin(self.ab_alpha + a)
        s["iw_north"] = np.where(sample, iw_n, s["iw_north"])
        s["iw_east"] = np.where(sample, iw_e, s["iw_east"])
        s["event"] = np.where(sample, s["event"] + 1, s["event"])
        act = np.stack([s["iw_north"], s["iw_east"]], axis=1)
        return act, sample, init, np.where(sample, a, np.nan)

    def policy_rollout(self, n_steps, seed, policy, env_id_offset=0, mask_horizon=600):
        """The synchronous loop of test_beds/main_ast.py:310-412 with a policy choosing the IW
        (agent.select_action mode 1, :344-349): at every sampling event (episode start, or the
        sampling distance reaching AB_len while the obstacle ship runs) policy(state[m, 10],
        noise[m]) -> action[m] in [-1, 1] with noise = sampler_normal(seed, env_id, event); the
        route angle is a = action * pi / 6 and IW = obstacle position + AB_len (cos, sin)(AB_alpha
        + a).  Auto-reset on done.  Returns dict of [K, n_env, ...] arrays (action rows hold IW
        north, IW east, a, SAC_update) and the per-event policy actions."""
        s = self.s
        out = dict(next_state=[], reward=[], done=[], status=[], action=[])
        trans = []
        env_id = np.arange(self.n_env, dtype=np.uint64) + np.uint64(env_id_offset)
        for _ in range(n_steps):
            init = s["ep_step"] == 0
            stopped = s["stop"][1].astype(bool)
            sample = init | ((s["sampling_dist"] >= self.ab_len) & ~stopped)
            ang = np.full(self.n_env, np.nan)
            act_n = np.full(self.n_env, np.nan)
            idx = np.nonzero(sample)[0]
            state_all = self.s["last_obs"].T.copy()
            t_after = s["ep_step"] + 1
            if idx.size:
                state = self.s["last_obs"].T[idx]
                noise = sampler_normal(seed, env_id[idx], s["event"][idx])
                a = np.asarray(policy(state, noise), dtype=np.float64).reshape(-1)
                act_n[idx] = a
                ang[idx] = a * (np.pi / 6.0)
                s["iw_north"][idx] = s["north"][1][idx] + self.ab_len[idx] * np.cos(self.ab_alpha[idx] + ang[idx])
                s["iw_east"][idx] = s["east"][1][idx] + self.ab_len[idx] * np.sin(self.ab_alpha[idx] + ang[idx])
                s["event"][idx] = s["event"][idx] + 1
            act = np.stack([s["iw_north"], s["iw_east"]], axis=1)
            ns, rew, done, st = self.step(act, sample, init)
            if idx.size:          # memory.push on sampling events (main_ast.py:385-396)
                trans.append(self._transitions(idx, state_all, act_n, rew, ns, done, t_after, mask_horizon,
                                               env_id_offset))
            out["next_state"].append(ns)
            out["reward"].append(rew)
            out["done"].append(done)
            out["status"].append(st)
            out["action"].append(np.stack([act[:, 0], act[:, 1], ang, sample.astype(float)], axis=1))
            if done.any():
                self.reset(done)
                self.s["episodes"] = self.s["episodes"] + done.astype(np.int64)
                self.init_step(done)
        res = {k: np.stack(v) for k, v in out.items()}
        res["transitions"] = np.concatenate(trans) if trans else np.zeros((0, 24))
        return res

    @staticmethod
    def _transitions(idx, state, act_n, rew, ns, done, t_after, mask_horizon, env_id_offset):
        """Replay records [state 10, action, reward, next_state 10, mask, env id] of the envs idx:
        memory.push(state, action, reward, next_state, mask) with mask = 1 at the episode-length
        horizon, else not done (test_beds/main_ast.py:385-396)."""
        mask = np.where((mask_horizon > 0) & (t_after + 1 == mask_horizon), 1.0, 1.0 - done)
        return np.concatenate([state[idx], act_n[idx, None], rew[idx, None], ns[idx], mask[idx, None],
                               (idx + env_id_offset)[:, None].astype(np.float64)], axis=1)

    def rollout(self, n_steps, seed, auto_reset=True, env_id_offset=0, actions=None, mask_horizon=600):
        """K steps of the test_beds/main_ast.py:310-412 loop: reset+init_step on done, synthetic
        (or explicit) IW actions.  Returns dict of [K, n_env, ...] arrays plus the replay
        transitions pushed on sampling events (main_ast.py:385-396) as rows of
        [state 10, a, reward, next_state 10, mask, env id]."""
        out = dict(next_state=[], reward=[], done=[], status=[], action=[])
        trans = []
        for k in range(n_steps):
            if actions is None:
                act, sac, init, ang = self.sampler_actions(seed, env_id_offset)
                act_n = self.last_action_n
            else:
                act, sac, init = actions["action_ne"][k], actions["sac_update"][k], actions["init"][k]
                ang = np.full(self.n_env, np.nan)
            state = self.s["last_obs"].T.copy()
            t_after = self.s["ep_step"] + 1
            ns, rew, done, st = self.step(act, sac, init)
            if actions is None and np.any(sac):
                trans.append(self._transitions(np.nonzero(sac)[0], state, act_n, rew, ns, done, t_after,
                                               mask_horizon, env_id_offset))
            out["next_state"].append(ns)
            out["reward"].append(rew)
            out["done"].append(done)
            out["status"].append(st)
            out["action"].append(np.stack([act[:, 0], act[:, 1], ang, sac.astype(float)], axis=1))
            if auto_reset and done.any():
                self.reset(done)
                self.s["episodes"] = self.s["episodes"] + done.astype(np.int64)
                self.init_step(done)
        res = {k: np.stack(v) for k, v in out.items()}
        res["transitions"] = np.concatenate(trans) if trans else np.zeros((0, 24))
        return res


def status_string(bits: int) -> str:
    """Rebuild the reference's concatenated status string (MSRL_env_ex.py:742-807, 817-879, 890-899)."""
    t = " "
    for bit, txt in ((ST_TEST_ENDPOINT, "|Test ship reaches endpoint|"),
                     (ST_TEST_HORIZON, "|Test ship hits map horizon|"),
                     (ST_TEST_TERRAIN, "|Test ship collides with the terrain|"),
                     (ST_TEST_MECHANICAL, "|Test ship mechanical failure|"),
                     (ST_TEST_NAVIGATION, "|Test ship navigation failure|"),
                     (ST_TEST_BLACKOUT, "|Test ship blackout failure|")):
        if bits & bit:
            t += txt
    if not bits & ST_TEST_DONE:
        t += "|Test ship not in terminal state|"
    o = " "
    for bit, txt in ((ST_OBS_ENDPOINT, "|Obstacle ship reaches endpoint|"),
                     (ST_OBS_HORIZON, "|Obstacle ship hits map horizon|"),
                     (ST_OBS_TERRAIN, "|Obstacle ship collides with the terrain|"),
                     (ST_OBS_IW_TERMINAL, "|Obstacle ship IW sampled in terminal state|"),
                     (ST_OBS_NAVIGATION, "|Obstacle ship navigation failure|")):
        if bits & bit:
            o += txt
    if not bits & ST_OBS_DONE:
        o += "|Obstacle ship not in terminal state|"
    sh = " " + ("|Ship collision|" if bits & ST_COLLISION else "")
    return t + o + sh

