"""Build-owned AST samplers: the counterpart of the reference's (empty)
``ast_core/samplers/intermediate_waypoint_sampler.py`` and of the episode loop of
``test_beds/main_ast.py:310-412``, driving the HIP env step.

Two action sources, as in ``agent.select_action(state, done, init, mode)`` (main_ast.py:337-349):

* mode 0 (``start_steps``, random sampling): the route scoping angle a ~ U[-pi/6, pi/6] drawn on
  device (the synthetic sampler of ``sit_rollout``; ``UniformPolicy``, uniform_policy.py:18-21,
  gives actions U[-1, 1], scaled by the action bound pi/6).
* mode 1 (policy sampling): the SAC actor, a squashed Gaussian MLP (``GaussianPolicy`` below),
  evaluated in PyTorch-ROCm between fused K-step launches of the env kernel.

Policy mode on the GPU: an env whose next step is a sampling event and that holds no fresh
action stops for the rest of the launch.  Its action is computed from its observation and a
standard-normal draw keyed by (seed, env id, event), in one of two ways:

* in-kernel serving (``serve="kernel"``, the default for the reference's actor architecture): the
  step kernel itself evaluates the fused actor for every env of a block that ends the launch
  waiting (csrc/sit_serve.h), so every waiting env steps again from the next launch;
* the request queue (``serve="queue"``): after the launch the library admits the waiting envs,
  oldest request first and ties by env id, at most ``request_capacity`` of them; the actor runs
  on the queued observations (one HIP kernel, or PyTorch-ROCm for other architectures) and
  scatters the squashed actions into per-env slots (an env waiting since launch L is served by
  round L + ceil(n_env / capacity) - 1).

The next launch consumes the actions.  Each env's trajectory is the one the synchronous per-step
loop produces (oracle/sit_oracle.py ``OracleEnvs.policy_rollout``; tests/test_gpu_policy.py),
independent of how envs are batched into launches, and how many rows each env executes is a
function of the data, the chunk and the capacity, never of GPU scheduling; both serving paths give
the same rows bit for bit at capacity n_env.
``OverlappedPolicySampler`` splits the envs into groups on separate HIP streams so one group's
actor runs while the others' env kernels run.

The converter from action to simulator input (``agent.convert_action_to_simu_input``) is absent
from the reference; the build defines it: route angle a = action * pi/6 and
IW = obstacle position + AB_len (cos, sin)(AB_alpha + a), inserted at index -1 of the obstacle
ship's route with SAC_update on sampling events only.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib
from .env import VecMultiShipRLEnv

LOG_SIG_CAP_MIN, LOG_SIG_CAP_MAX = -20.0, 2.0   # ast_core/distributions/normal.py:15-16
EPS = 1e-6                                      # ast_core/policies/gaussian_policy.py:18


class GaussianPolicy(nn.Module):
    """Squashed Gaussian policy: ast_core/policies/gaussian_policy.py:19-148 with the Normal head of
    ast_core/distributions/normal.py:17-133 and the MLP of ast_core/nn_models/mlp.py:95-148.

    obs [N, obs_dim] -> ReLU hidden layers -> [mu, log_sigma] ([N, 2*Da], no output nonlinearity);
    log_sigma clipped to [-20, 2]; x = mu + exp(log_sigma) * noise (reparameterised sample,
    normal.py:96-101); action = tanh(x) (squash=True); log_pi = sum_d log N(x_d; mu_d, sigma_d)
    - sum_d log(1 - tanh(x_d)^2 + 1e-6) (gaussian_policy.py:88-94, 141-144).  The reference's
    TF1 graph (tensorflow/tfp/rllab) is not importable here: parity of this head is pinned to its
    formulas (tests/test_samplers.py), not to a reference run.  Hidden size 256 x 2 is
    main_ast.py:67's default."""

    def __init__(self, obs_dim: int = _lib.SIT_OBS_DIM, act_dim: int = 1, hidden=(256, 256)):
        super().__init__()
        layers, d = [], obs_dim
        for h in hidden:
            layers += [nn.Linear(d, h), nn.ReLU()]
            d = h
        layers.append(nn.Linear(d, 2 * act_dim))
        self.net = nn.Sequential(*layers)
        self.act_dim = act_dim

    def forward(self, obs: torch.Tensor, noise: torch.Tensor | None = None, deterministic: bool = False):
        out = self.net(obs)
        mu, log_sig = out[..., :self.act_dim], out[..., self.act_dim:]
        log_sig = log_sig.clamp(LOG_SIG_CAP_MIN, LOG_SIG_CAP_MAX)
        if deterministic:                     # GaussianPolicy.get_actions, _is_deterministic (:114-126)
            x = mu
        else:
            if noise is None:
                noise = torch.randn_like(mu)
            x = mu + log_sig.exp() * noise.reshape(mu.shape)
        action = torch.tanh(x)
        sig = log_sig.exp()
        log_prob = (-0.5 * ((x - mu) / sig) ** 2 - log_sig - 0.5 * math.log(2 * math.pi)).sum(-1)
        log_pi = log_prob - torch.log(1 - action ** 2 + EPS).sum(-1)
        return action, log_pi, mu, log_sig


def pack_actor_weights(policy: nn.Module, out: torch.Tensor | None = None) -> torch.Tensor | None:
    """The float32 weight block of sit_policy_actor (include/sit.h) from a GaussianPolicy whose trunk
    is the reference's default MLP (obs 10 -> 256 -> ReLU -> 256 -> ReLU -> 2; mlp.py:95-148,
    main_ast.py:67), or None for any other architecture (those take the generic path)."""
    net = getattr(policy, "net", None)
    if net is None or getattr(policy, "act_dim", 1) != 1 or len(net) != 5:
        return None
    l1, r1, l2, r2, l3 = net
    H = _lib.SIT_ACTOR_HIDDEN
    shapes_ok = (isinstance(l1, nn.Linear) and isinstance(l2, nn.Linear) and isinstance(l3, nn.Linear)
                 and isinstance(r1, nn.ReLU) and isinstance(r2, nn.ReLU)
                 and tuple(l1.weight.shape) == (H, _lib.SIT_OBS_DIM) and tuple(l2.weight.shape) == (H, H)
                 and tuple(l3.weight.shape) == (2, H) and l1.bias is not None and l2.bias is not None
                 and l3.bias is not None)
    if not shapes_ok:
        return None
    with torch.no_grad():
        if out is None:
            parts = [l1.weight.reshape(-1), l1.bias, l2.weight.t().reshape(-1), l2.bias, l3.weight.reshape(-1), l3.bias]
            return torch.cat([t.detach().to(torch.float32).reshape(-1) for t in parts]).contiguous()
        # in place, one copy per parameter into its segment of the block (no concatenated temporary:
        # half the host work of a refresh after each optimizer step)
        if out.numel() != _lib.SIT_ACTOR_WEIGHTS or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"pack_actor_weights: out must be a contiguous float32 tensor of "
                             f"{_lib.SIT_ACTOR_WEIGHTS} elements (got {tuple(out.shape)} {out.dtype}, "
                             f"contiguous={out.is_contiguous()})")
        o = 0
        for t, shape in ((l1.weight, (H, _lib.SIT_OBS_DIM)), (l1.bias, (H,)), (l2.weight.t(), (H, H)), (l2.bias, (H,)),
                         (l3.weight, (2, H)), (l3.bias, (2,))):
            n = t.numel()
            out[o:o + n].view(shape).copy_(t.detach())
            o += n
        return out


def _trunk(net: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """net(x) for an nn.Sequential trunk, each Linear followed by a ReLU evaluated as one GEMM with
    the bias and the ReLU in its epilogue (torch._addmm_activation: hipBLASLt's fused epilogue on ROCm)
    instead of a GEMM and a separate elementwise kernel; any other layer as itself."""
    layers = list(net) if isinstance(net, nn.Sequential) else None
    if layers is None or x.dim() != 2 or not hasattr(torch, "_addmm_activation"):
        return net(x)
    i = 0
    while i < len(layers):
        m = layers[i]
        if (isinstance(m, nn.Linear) and m.bias is not None and i + 1 < len(layers)
                and isinstance(layers[i + 1], nn.ReLU)):
            x = torch._addmm_activation(m.bias, x, m.weight.t())
            i += 2
        else:
            x = m(x)
            i += 1
    return x


class PolicySampler:
    """Fused K-step launches in policy mode.

    serve="kernel" (the default when the actor is fused and no request_capacity is given): the
    step kernel serves every env that ends a launch waiting, in the same launch (no queue, no
    capacity).  serve="queue": the actor runs between launches on the request queue;
    request_capacity bounds the envs served per launch (default n_env: every waiting env) and envs
    beyond it keep waiting, oldest first, for the next admission round.  The queued actor runs on a
    fixed number of rows (no host synchronisation); rows past the device-side request count are
    scattered into a dummy slot.

    With the reference's default actor architecture (``pack_actor_weights``) the whole actor runs as
    HIP code (in the step kernel, or sit_policy_actor); ``fused_actor=False`` or any other
    architecture evaluates the network with PyTorch-ROCm (queue only).  The fused path reads a packed
    copy of the weights: after an optimizer step call ``refresh_weights()`` (``launch()`` does it by
    itself outside HIP-graph replays)."""

    def __init__(self, env: VecMultiShipRLEnv, policy: nn.Module, chunk: int = 32, seed: int = 25450,
                 env_id_offset: int = 0, request_capacity: int | None = None, mask_horizon: int = 600,
                 transition_capacity: int = 0, deterministic: bool = False, actor_dtype=None,
                 fused_actor: bool = True, serve: str | None = None, actor_stream: bool = False):
        self.env, self.policy, self.chunk, self.seed = env, policy, int(chunk), int(seed)
        # queue serving: the actor on a HIP stream of its own, forked after the env launch and joined
        # before the next (north_star's "actor forward interleaved with the HIP env step on separate
        # streams"; with one group the two kernels still run in order: the next launch needs the actions)
        self.actor_stream = torch.cuda.Stream(device=env.device) if actor_stream else None
        self.env_id_offset, self.mask_horizon = int(env_id_offset), int(mask_horizon)
        self.transition_capacity, self.deterministic = int(transition_capacity), deterministic
        n, dev, dt = env.n_env, env.device, env.dtype
        self.actor_dtype = actor_dtype or next(policy.parameters()).dtype
        self._w = pack_actor_weights(policy) if fused_actor and self.actor_dtype == torch.float32 else None
        if serve is None:
            serve = "kernel" if self._w is not None and request_capacity is None else "queue"
        if serve not in ("kernel", "queue"):
            raise ValueError("serve must be 'kernel' or 'queue'")
        if serve == "kernel" and (self._w is None or request_capacity is not None):
            raise ValueError("in-kernel serving needs the fused actor (the reference's architecture, float32) "
                             "and serves every waiting env (no request_capacity)")
        self.serve = serve
        self.served = torch.zeros(1, dtype=torch.int64, device=dev)   # policy evaluations used
        self.io = {
            "policy_action": torch.zeros(n + 1, dtype=dt, device=dev),      # slot n: dummy
            "policy_ready": torch.zeros(n + 1, dtype=torch.int32, device=dev),
            "env_steps": torch.zeros(1, dtype=torch.int64, device=dev),
        }
        if self._w is not None:
            self._w = self._w.to(dev)
            self._w_version = self._weights_version()
        if serve == "kernel":
            self.io.update(actor_weights=self._w, actor_served=self.served, actor_deterministic=bool(deterministic))
        else:
            cap = int(request_capacity or n)
            if cap <= 0:
                raise ValueError("request_capacity must be positive")
            self.io.update({
                "request_env": torch.zeros(cap, dtype=torch.int32, device=dev),
                "request_noise": torch.zeros(cap, dtype=dt, device=dev),
                "request_obs": torch.zeros((cap, _lib.SIT_OBS_DIM), dtype=dt, device=dev),
                # rows admitted by the last launch (written by the library's admission kernel)
                "request_count": torch.zeros(1, dtype=torch.int32, device=dev),
                # admission rounds each waiting env has waited (kept by the admission kernel)
                "request_age": torch.zeros(n, dtype=torch.int32, device=dev),
            })
            self._rows = torch.arange(cap, device=dev, dtype=torch.int32)
            self._one = torch.full((cap,), _lib.SIT_POLICY_READY, dtype=torch.int32, device=dev)
        self.out: dict = {}

    @property
    def fused(self) -> bool:
        return self._w is not None

    def _weights_version(self):
        return tuple((p.data_ptr(), p._version) for p in self.policy.parameters())

    def refresh_weights(self):
        """Re-pack the actor weights (after the policy's parameters changed)."""
        if self._w is not None:
            pack_actor_weights(self.policy, out=self._w)
            self._w_version = self._weights_version()

    @property
    def env_steps(self) -> torch.Tensor:
        """Env-steps executed so far (device int64[1])."""
        return self.io["env_steps"]

    def launch(self, want=("next_state", "reward", "done", "status", "action"), events=None,
               first: bool = True):
        """One fused launch of `chunk` steps, serving its waiting envs in the kernel, or followed by
        the actor on the queued requests.
        Returns the launch's [K, n_env, ...] outputs (rows of waiting envs: status ST_NO_STEP).
        events: optional (start, end) torch.cuda.Event pair recorded around the env kernel.
        first: the launch starts a new batch of replay transitions (their count is zeroed); later
        launches of a batch append to it, so a HIP graph of several launches keeps all of them."""
        if (self.serve == "kernel" and not torch.cuda.is_current_stream_capturing()
                and self._weights_version() != self._w_version):
            self.refresh_weights()
        if events is not None:
            events[0].record(torch.cuda.current_stream(self.env.device))
        self.env.rollout(self.chunk, seed=self.seed, env_id_offset=self.env_id_offset, out=self.out,
                         want=want, transition_capacity=self.transition_capacity,
                         mask_horizon=self.mask_horizon, policy_io=self.io, reset_transitions=first)
        if events is not None:
            events[1].record(torch.cuda.current_stream(self.env.device))
        if self.serve == "queue":
            if self.actor_stream is None:
                self.act()
            else:
                cur = torch.cuda.current_stream(self.env.device)
                self.actor_stream.wait_stream(cur)
                with torch.cuda.stream(self.actor_stream):
                    self.act()
                cur.wait_stream(self.actor_stream)
        return self.out

    def capture(self, n_launch: int = 2, want=("next_state", "reward", "done", "status", "action")):
        """Record `n_launch` launches (env kernel [+ admission + actor]) into one HIP graph; replay()
        then runs them with a single submission (the per-launch host work of ctypes and ~10 torch
        ops otherwise bounds short chunks).  The output buffers are those of the last launch."""
        if n_launch < 1:
            raise ValueError("capture at least one launch")
        self.launch(want)                     # allocate every buffer outside the capture
        self.launch(want)
        torch.cuda.synchronize(self.env.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for i in range(n_launch):
                self.launch(want, first=(i == 0))
        return self

    def replay(self):
        self.graph.replay()
        return self.out

    @torch.no_grad()
    def act(self):
        """The actor on the queued observations and the scatter into the per-env action slots:
        one HIP kernel (sit_policy_actor) for the default architecture; otherwise the network in
        PyTorch-ROCm, then the squashed Gaussian head and the scatter in one HIP kernel
        (sit_policy_apply), or for policies without a `.net` (mu, log_sigma) trunk forward() and a
        device-side scatter.  (Queue serving only: in-kernel serving has nothing left to do.)"""
        io, env = self.io, self.env
        if self.serve == "kernel":
            return
        if self._w is not None:
            if not torch.cuda.is_current_stream_capturing() and self._weights_version() != self._w_version:
                self.refresh_weights()
            with torch.cuda.device(env.device):
                env._call("sit_policy_actor", int(self._rows.numel()), self._w.data_ptr(), io["request_obs"].data_ptr(),
                          io["request_noise"].data_ptr(), io["request_env"].data_ptr(),
                          io["request_count"].data_ptr(), int(bool(self.deterministic)),
                          io["policy_action"].data_ptr(), io["policy_ready"].data_ptr(), self.served.data_ptr(),
                          None, env._stream())
            return
        obs = io["request_obs"] if self.actor_dtype == env.dtype else io["request_obs"].to(self.actor_dtype)
        net = getattr(self.policy, "net", None)
        if net is not None and getattr(self.policy, "act_dim", 1) == 1:
            head = _trunk(net, obs)
            if head.dtype != env.dtype:
                head = head.to(env.dtype)
            head = head.contiguous()
            with torch.cuda.device(env.device):
                env._call("sit_policy_apply", int(self._rows.numel()), head.data_ptr(), int(head.shape[1]),
                          io["request_noise"].data_ptr(), io["request_env"].data_ptr(),
                          io["request_count"].data_ptr(), int(bool(self.deterministic)),
                          io["policy_action"].data_ptr(), io["policy_ready"].data_ptr(), self.served.data_ptr(),
                          env._stream())
            return
        count = io["request_count"].clamp(max=self._rows.numel())
        idx = torch.where(self._rows < count, io["request_env"], env.n_env).long()
        action, _, _, _ = self.policy(obs, io["request_noise"].to(self.actor_dtype),
                                      deterministic=self.deterministic)
        io["policy_action"].index_put_((idx,), action[:, 0].to(io["policy_action"].dtype))
        io["policy_ready"].index_put_((idx,), self._one)
        self.served += count


class OverlappedPolicySampler:
    """Envs split into groups, each with its own HIP stream: while one group's actor runs, the
    other groups' env kernels keep the CUs busy (BASELINE config 5)."""

    def __init__(self, samplers: list[PolicySampler], device=None):
        self.samplers = samplers
        dev = device or samplers[0].env.device
        self.streams = [torch.cuda.Stream(device=dev) for _ in samplers]

    def launch(self, want=("next_state", "reward", "done", "status", "action"), events=None, first: bool = True):
        """One launch of every group on its stream; events: optional per-group (start, end) pairs."""
        cur = torch.cuda.current_stream(self.streams[0].device)
        outs = []
        for g, (sm, st) in enumerate(zip(self.samplers, self.streams)):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                outs.append(sm.launch(want, events=None if events is None else events[g], first=first))
        for st in self.streams:
            cur.wait_stream(st)
        return outs

    def env_steps(self) -> torch.Tensor:
        return sum(sm.env_steps for sm in self.samplers)

    def capture(self, n_launch: int = 2, want=("next_state", "reward", "done", "status", "action")):
        """One HIP graph holding `n_launch` rounds of every group (forked onto the groups'
        streams inside the capture, joined at the end)."""
        if n_launch < 1:
            raise ValueError("capture at least one launch")
        self.launch(want)
        self.launch(want)
        torch.cuda.synchronize(self.streams[0].device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for i in range(n_launch):
                self.launch(want, first=(i == 0))
        return self

    def replay(self):
        self.graph.replay()
        return [sm.out for sm in self.samplers]


class IntermediateWaypointSampler:
    """The AST sampler the reference leaves empty: mode 0 (random IWs, on-device Philox draws)
    until `start_steps` env-steps, then mode 1 (policy) — main_ast.py:337-349."""

    def __init__(self, env: VecMultiShipRLEnv, policy: nn.Module | None = None, chunk: int = 32,
                 seed: int = 25450, start_steps: int = 0, env_id_offset: int = 0, **kw):
        self.env, self.chunk, self.seed, self.env_id_offset = env, int(chunk), int(seed), int(env_id_offset)
        self.start_steps = int(start_steps)
        self.total = 0
        self.policy_sampler = PolicySampler(env, policy, chunk, seed, env_id_offset, **kw) if policy is not None else None
        self.out: dict = {}

    def launch(self):
        if self.policy_sampler is None or self.total < self.start_steps:
            self.env.rollout(self.chunk, seed=self.seed, env_id_offset=self.env_id_offset, out=self.out)
            self.total += self.chunk * self.env.n_env
            return self.out
        out = self.policy_sampler.launch()
        self.total += self.chunk * self.env.n_env
        return out
