"""Batched two-ship environment on one MI355X: ``VecMultiShipRLEnv``.

N independent copies of the reference's ``MultiShipRLEnv`` (RLEnv/MSRL_Env.py:37-450 with the
reward/termination of RLEnv/MSRL_env_ex.py:450-980) stepped by the HIP kernels of libsit.so.
All per-step tensors live on the GPU; PyTorch is used only for device memory and streams.

Method              reference counterpart
  reset(mask)         MultiShipRLEnv.reset        MSRL_Env.py:147-188
  init_step(mask)     MultiShipRLEnv.init_step    MSRL_Env.py:190-217
  step(a, sac, init)  MultiShipRLEnv.step         MSRL_Env.py:404-442
  rollout(K, seed)    K steps of test_beds/main_ast.py:310-412 with the synthetic sampler
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_char_p, c_int32, c_int64, c_size_t, c_void_p

import numpy as np
import torch

from . import _lib
from .config import params as default_params
from .scenario import Scenario, make_scenario


def _ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


# float32 handles keep these fields as double-float values (hi + lo; csrc/sit_device.h comp_add): the
# reference integrates them in float64, and a float32 running sum loses up to half an ulp a step
LO_FIELDS = {"north": "north_lo", "east": "east_lo", "yaw": "yaw_lo", "ship_speed_i": "ship_speed_i_lo",
             "shaft_speed_i": "shaft_speed_i_lo", "heading_i": "heading_i_lo", "e_ct_int": "e_ct_int_lo",
             "surge": "surge_lo", "sway": "sway_lo", "yaw_rate": "yaw_rate_lo", "shaft_speed": "shaft_speed_lo",
             "sampling_dist": "sampling_dist_lo", "prev_pre_north": "prev_pre_north_lo",
             "prev_pre_east": "prev_pre_east_lo"}


class VecMultiShipRLEnv:
    """N two-ship environments resident in HBM.

    precision 32 (default, BASELINE fp32) or 64 (bit-faithful float64 arithmetic of the reference).
    """

    def __init__(self, n_env: int | None = None, scenario: Scenario | None = None, params=None,
                 precision: int = 32, wpt_capacity: int = 32, device=None):
        if scenario is None:
            if n_env is None:
                raise ValueError("give n_env or a scenario")
            scenario = make_scenario(n_env, cap=wpt_capacity)
        self.scenario = scenario
        self.n_env = int(scenario.n_env)
        self.cap = int(scenario.routes.shape[2])
        if precision not in (32, 64):
            raise ValueError("precision must be 32 or 64")
        self.precision = precision
        self.dtype = torch.float32 if precision == 32 else torch.float64
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("VecMultiShipRLEnv runs on a ROCm GPU device")
        self.params = params if params is not None else default_params()
        self.lib = _lib.load()
        self.handle = c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.sit_create(byref(self.params), self.n_env, self.cap, precision,
                                           byref(self.handle)))
            self._load(scenario)
            self._call("sit_restart", self._stream())
        self._layout = self._read_layout()
        self._zero_i32 = None

    # ---------------- plumbing ----------------
    def _stream(self):
        return c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _call(self, name, *args):
        return _lib.check(getattr(self.lib, name)(self.handle, *args), self.handle)

    def _load(self, sc: Scenario):
        polys = [np.ascontiguousarray(p, dtype=np.float64) for p in sc.polys]
        offs = np.zeros(len(polys) + 1, dtype=np.int32)
        offs[1:] = np.cumsum([len(p) for p in polys])
        verts = np.ascontiguousarray(np.concatenate(polys), dtype=np.float64)
        self._call("sit_load_map", len(polys), offs.ctypes.data_as(c_void_p), verts.ctypes.data_as(c_void_p))
        routes = np.ascontiguousarray(sc.routes, dtype=np.float64)
        nw = np.ascontiguousarray(sc.n_wpt, dtype=np.int32)
        self._call("sit_load_routes", routes.ctypes.data_as(c_void_p), nw.ctypes.data_as(c_void_p))
        init = np.ascontiguousarray(sc.init, dtype=np.float64)
        self._call("sit_load_initial", init.ctypes.data_as(c_void_p))

    def _read_layout(self):
        out = []
        n = self.lib.sit_state_nfields()
        for i in range(n):
            name, off, dt, cnt = c_char_p(), c_size_t(), c_int32(), c_int64()
            self._call("sit_state_field", i, byref(name), byref(off), byref(dt), byref(cnt))
            out.append((name.value.decode(), off.value, dt.value, cnt.value))
        nb = c_size_t()
        self._call("sit_state_bytes", byref(nb))
        self._state_bytes = nb.value
        return out

    def _field_shape(self, name, count):
        if name == "last_obs":
            return (_lib.SIT_OBS_DIM, self.n_env)
        if name == "last_log":
            return (_lib.SIT_LOG_KEYS, self.n_env)
        if count == 2 * self.n_env:
            return (2, self.n_env)
        if count == self.n_env:
            return (self.n_env,)
        return (2, self.cap, self.n_env)

    def _dev(self, t, dtype, shape, name):
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(np.asarray(t))
        if t.dtype == torch.bool:
            t = t.to(torch.uint8)
        t = t.to(device=self.device, dtype=dtype).reshape(shape).contiguous()
        return t

    def _mask(self, mask):
        if mask is None:
            return None
        return self._dev(mask, torch.uint8, (self.n_env,), "mask")

    # ---------------- map diagnostics ----------------
    def map_info(self) -> dict:
        """Spatial-index statistics of the loaded island map (sit_map_info)."""
        info = (c_int64 * 6)()
        self._call("sit_map_info", info, 6)
        keys = ("map_bytes", "mixed_cells", "live_edges", "use_index", "use_cells", "lds_bytes")
        return dict(zip(keys, (int(v) for v in info)))

    def probe_map(self, pts_ne):
        """The step kernel's map predicates at arbitrary (north, east) points: boundary distance,
        Polygon.contains and the 4-corner hull test (sit_probe_map)."""
        pts = self._dev(pts_ne, self.dtype, (-1, 2), "pts_ne")
        n = pts.shape[0]
        dist = torch.empty(n, dtype=self.dtype, device=self.device)
        inside = torch.empty(n, dtype=torch.uint8, device=self.device)
        hull = torch.empty(n, dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            self._call("sit_probe_map", n, _ptr(pts), _ptr(dist), _ptr(inside), _ptr(hull), self._stream())
        return dist, inside.bool(), hull.bool()

    # ---------------- env API ----------------
    def restart(self):
        """Construction-time state (as if freshly built)."""
        with torch.cuda.device(self.device):
            self._call("sit_restart", self._stream())

    def reset(self, mask=None):
        """MultiShipRLEnv.reset; returns the construction-time observation [n_env, 10]."""
        out = torch.empty((self.n_env, _lib.SIT_OBS_DIM), dtype=self.dtype, device=self.device)
        m = self._mask(mask)
        with torch.cuda.device(self.device):
            self._call("sit_reset", _ptr(m), _ptr(out), self._stream())
        return out

    def init_step(self, mask=None):
        m = self._mask(mask)
        with torch.cuda.device(self.device):
            self._call("sit_init_step", _ptr(m), self._stream())

    def step(self, action_ne, sac_update, init, done_count: torch.Tensor | None = None):
        """One MultiShipRLEnv.step for every env.  Returns (next_state [n,10], reward [n],
        done [n] bool, status [n] int64 bitmask)."""
        n = self.n_env
        a = self._dev(action_ne, self.dtype, (n, 2), "action_ne")
        s = self._dev(sac_update, torch.uint8, (n,), "sac_update")
        i = self._dev(init, torch.uint8, (n,), "init")
        ns = torch.empty((n, _lib.SIT_OBS_DIM), dtype=self.dtype, device=self.device)
        rew = torch.empty((n,), dtype=self.dtype, device=self.device)
        done = torch.empty((n,), dtype=torch.uint8, device=self.device)
        st = torch.empty((n,), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            self._call("sit_step", _ptr(a), _ptr(s), _ptr(i), _ptr(ns), _ptr(rew), _ptr(done), _ptr(st),
                       _ptr(done_count), self._stream())
        return ns, rew, done.bool(), st.to(torch.int64) & 0xFFFFFFFF

    def rollout(self, n_steps: int, seed: int = 25450, auto_reset: bool = True, env_id_offset: int = 0,
                actions: dict | None = None, out: dict | None = None, want=("next_state", "reward", "done",
                                                                              "status", "action", "done_count"),
                transition_capacity: int = 0, mask_horizon: int = 600, policy_io: dict | None = None,
                log: bool = False, reset_transitions: bool = True):
        """K fused steps (one kernel launch).  actions=None: synthetic AST sampler on device.
        Returns a dict of [K, n_env, ...] tensors (reused from `out` when given).  With
        transition_capacity > 0 the sampling-event replay transitions are appended to
        out["transitions"] ([capacity, 24]) and counted in out["transition_count"] ([1]); the count
        is zeroed first unless reset_transitions=False (several launches appending to one buffer).
        policy_io: the policy-mode buffers (see samplers.PolicySampler): actions of sampling events
        come from a policy; waiting envs' rows carry status ST_NO_STEP.  With "actor_weights" (the
        packed float32 actor, samplers.pack_actor_weights) the launch serves its waiting envs itself
        at its end (in-kernel serving; optional "actor_served" int64[1], "actor_deterministic");
        otherwise after the launch the library admits waiting envs into the request queue
        ("request_*"), oldest request first, ties by env id (include/sit.h, sit_rollout_args)."""
        n, K = self.n_env, int(n_steps)
        out = {} if out is None else out
        shapes = {"next_state": ((K, n, _lib.SIT_OBS_DIM), self.dtype), "reward": ((K, n), self.dtype),
                  "done": ((K, n), torch.uint8), "status": ((K, n), torch.int32),
                  "action": ((K, n, 4), self.dtype), "done_count": ((K,), torch.int32)}
        for k in want:
            shp, dt = shapes[k]
            t = out.get(k)
            if t is None or tuple(t.shape) != shp or t.dtype != dt:
                out[k] = torch.empty(shp, dtype=dt, device=self.device)
        if "done_count" in want:
            out["done_count"].zero_()
        ra = _lib.RolloutArgs()
        ra.n_steps, ra.auto_reset, ra.seed, ra.env_id_offset = K, int(bool(auto_reset)), int(seed), int(env_id_offset)
        keep = []
        if actions is not None:
            a = self._dev(actions["action_ne"], self.dtype, (K, n, 2), "action_ne")
            s = self._dev(actions["sac_update"], torch.uint8, (K, n), "sac_update")
            i = self._dev(actions["init"], torch.uint8, (K, n), "init")
            keep += [a, s, i]
            ra.action_ne, ra.sac_update, ra.init = a.data_ptr(), s.data_ptr(), i.data_ptr()
        for field, key in (("next_state", "next_state"), ("reward", "reward"), ("done", "done"),
                           ("status", "status"), ("action_out", "action"), ("done_count", "done_count")):
            t = out.get(key) if key in want else None
            setattr(ra, field, None if t is None else t.data_ptr())
        if transition_capacity > 0:
            tr = out.get("transitions")
            if tr is None or tr.shape != (transition_capacity, _lib.SIT_TRANSITION_DIM) or tr.dtype != self.dtype:
                out["transitions"] = torch.zeros((transition_capacity, _lib.SIT_TRANSITION_DIM),
                                                 dtype=self.dtype, device=self.device)
            if out.get("transition_count") is None:
                out["transition_count"] = torch.zeros(1, dtype=torch.int32, device=self.device)
            if reset_transitions:
                out["transition_count"].zero_()
            ra.transitions = out["transitions"].data_ptr()
            ra.transition_count = out["transition_count"].data_ptr()
            ra.transition_capacity = int(transition_capacity)
        ra.mask_horizon = int(mask_horizon)
        if log:                                  # trajectory log [K, SIT_LOG_ROWS, n_env]
            lg = out.get("log")
            if lg is None or tuple(lg.shape) != (K, _lib.SIT_LOG_ROWS, n) or lg.dtype != self.dtype:
                out["log"] = torch.empty((K, _lib.SIT_LOG_ROWS, n), dtype=self.dtype, device=self.device)
            ra.log = out["log"].data_ptr()
        if policy_io is not None:
            if actions is not None:
                raise ValueError("policy mode and explicit actions are exclusive")
            serve = policy_io.get("actor_weights") is not None
            for k in ("policy_action", "policy_ready", "request_env", "request_noise", "request_obs",
                      "request_count", "request_age", "env_steps", "actor_weights", "actor_served"):
                t = policy_io.get(k)
                if t is None and not (serve and k.startswith("request_")) and k not in ("env_steps", "actor_served",
                                                                                        "actor_weights"):
                    raise ValueError(f"policy_io needs {k}")
                setattr(ra, k, None if t is None else t.data_ptr())
            if serve and (policy_io["actor_weights"].dtype != torch.float32 or
                          policy_io["actor_weights"].numel() != _lib.SIT_ACTOR_WEIGHTS):
                raise ValueError("actor_weights: float32[SIT_ACTOR_WEIGHTS] (samplers.pack_actor_weights)")
            ra.actor_deterministic = int(bool(policy_io.get("actor_deterministic", False)))
            req = policy_io.get("request_env")
            ra.request_capacity = 0 if req is None else int(req.numel())
        with torch.cuda.device(self.device):
            _lib.check(self.lib.sit_rollout(self.handle, byref(ra), self._stream()), self.handle)
        return out

    # ---------------- state ----------------
    def state_blob(self):
        blob = torch.empty(self._state_bytes, dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            self._call("sit_get_state", _ptr(blob), self._stream())
        return blob

    def load_state_blob(self, blob):
        if blob.numel() != self._state_bytes or blob.dtype != torch.uint8:
            raise ValueError("state blob size/dtype mismatch")
        blob = blob.to(self.device).contiguous()
        with torch.cuda.device(self.device):
            self._call("sit_set_state", _ptr(blob), self._stream())

    def _views(self, blob):
        views = {}
        for name, off, dt, cnt in self._layout:
            tdt = self.dtype if dt == _lib.SIT_DT_REAL else torch.int32
            el = torch.tensor([], dtype=tdt).element_size()
            v = blob[off:off + cnt * el].view(tdt).reshape(self._field_shape(name, cnt))
            views[name] = v
        return views

    def get_state(self, combined: bool = False):
        """Named tensors (copies): ship fields [2, n_env], env fields [n_env], route tables
        [2, cap, n_env].  Unsigned fields are returned as int32.  A float32 handle holds the fields of
        LO_FIELDS as hi + lo (the `<name>_lo` fields); combined=True returns them as float64 values
        hi + lo, without the `_lo` fields."""
        st = self._views(self.state_blob())
        if combined:
            for hi, lo in LO_FIELDS.items():
                st[hi] = st[hi].to(torch.float64) + st.pop(lo).to(torch.float64)
        return st

    def set_state(self, state: dict):
        """Writes the given fields.  A field of LO_FIELDS given without its `_lo` part gets it from the
        value (float32 handles: the value's float64 rounding residual, so a float64 state is held
        exactly as hi + lo; float64 handles: 0)."""
        blob = self.state_blob()
        views = self._views(blob)
        for k, v in state.items():
            if k not in views:
                continue
            t = torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v).reshape(views[k].shape)
            views[k].copy_(t.to(dtype=views[k].dtype, device=self.device))
            lo = LO_FIELDS.get(k)
            if lo is not None and lo in views and lo not in state:
                x = t.to(dtype=torch.float64, device=self.device)
                views[lo].copy_((x - x.to(torch.float32).to(torch.float64)).to(views[lo].dtype)
                                if self.precision == 32 else torch.zeros_like(views[lo]))
        self.load_state_blob(blob)

    def close(self):
        if getattr(self, "handle", None) and self.handle.value:
            self.lib.sit_destroy(self.handle)
            self.handle = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_ = ctypes  # ctypes types are used through the _lib signatures
