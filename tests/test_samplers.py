"""CPU tests of the build-owned sampler's host logic: the squashed Gaussian policy head
(ast_core/distributions/normal.py, ast_core/policies/gaussian_policy.py) against its formulas,
and the oracle's policy-noise draw.  The TF1 reference policy is not importable here (tensorflow,
tfp and rllab are absent), so this head's parity is pinned to the published formulas only."""
import math

import numpy as np
import torch

from oracle import sit_oracle as so
from sac_maritime_ast_amd.samplers import EPS, LOG_SIG_CAP_MAX, LOG_SIG_CAP_MIN, GaussianPolicy


def test_policy_shapes_and_squash():
    torch.manual_seed(0)
    pol = GaussianPolicy(hidden=(256, 256)).double()
    obs = torch.randn(512, 10, dtype=torch.float64) * 100
    noise = torch.randn(512, dtype=torch.float64)
    a, logp, mu, ls = pol(obs, noise)
    assert a.shape == (512, 1) and logp.shape == (512,)
    assert torch.all(a.abs() <= 1)
    assert torch.all((ls >= LOG_SIG_CAP_MIN) & (ls <= LOG_SIG_CAP_MAX))
    # reparameterised sample, tanh squash
    x = mu + ls.exp() * noise[:, None]
    assert torch.allclose(a, torch.tanh(x))
    # log-likelihood of the pre-squash sample minus the squash correction (gaussian_policy.py:141-144)
    ref = torch.distributions.Normal(mu, ls.exp()).log_prob(x).sum(-1) - torch.log(1 - torch.tanh(x) ** 2 + EPS).sum(-1)
    assert torch.allclose(logp, ref, rtol=1e-12, atol=1e-12)


def test_policy_deterministic_mean_action():
    torch.manual_seed(1)
    pol = GaussianPolicy(hidden=(32,)).double()
    obs = torch.randn(16, 10, dtype=torch.float64)
    a, _, mu, _ = pol(obs, deterministic=True)
    assert torch.allclose(a, torch.tanh(mu))      # GaussianPolicy.get_actions, deterministic


def test_log_sigma_clip():
    pol = GaussianPolicy(hidden=(8,)).double()
    with torch.no_grad():
        pol.net[-1].bias[1] = 50.0
        pol.net[-1].weight.zero_()
    _, _, _, ls = pol(torch.zeros(3, 10, dtype=torch.float64))
    assert torch.all(ls == LOG_SIG_CAP_MAX)


def test_oracle_policy_noise_is_standard_normal_and_keyed():
    z = so.sampler_normal(7, np.arange(200_000), np.zeros(200_000, dtype=np.int64))
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert np.isfinite(z).all()
    z2 = so.sampler_normal(7, np.arange(10), np.ones(10, dtype=np.int64))
    assert not np.allclose(z[:10], z2)                 # the event index changes the draw
    assert np.array_equal(so.sampler_normal(7, np.arange(10), np.zeros(10, dtype=np.int64)), z[:10])
    # tails of Box-Muller with u1 in (0, 1]
    assert np.abs(z).max() < math.sqrt(-2 * math.log(1 / 2 ** 53)) + 1e-9


def test_oracle_policy_rollout_constant_policy_matches_explicit_actions():
    """policy_rollout with a constant action equals the explicit-action loop fed the same IWs."""
    from sac_maritime_ast_amd.scenario import make_scenario
    sc = make_scenario(8, cap=32, seed=3)
    mk = lambda: so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)  # noqa: E731
    o1 = mk()
    o1.reset()
    o1.init_step()
    r1 = o1.policy_rollout(120, 5, lambda s, n: np.full(len(s), 0.3))
    o2 = mk()
    o2.reset()
    o2.init_step()
    acts = {"action_ne": r1["action"][..., :2], "sac_update": r1["action"][..., 3] > 0.5,
            "init": np.zeros(r1["action"].shape[:2], bool)}
    # init flags: the first step of each episode
    ep0 = np.ones(8, bool)
    for k in range(120):
        acts["init"][k] = ep0
        ep0 = r1["done"][k]
    r2 = o2.rollout(120, 5, actions=acts)
    assert np.array_equal(r1["next_state"], r2["next_state"])
    assert np.array_equal(r1["status"], r2["status"])
    ang = r1["action"][..., 2]
    assert np.allclose(ang[~np.isnan(ang)], 0.3 * np.pi / 6)


def test_pack_actor_weights_in_place_equals_fresh_pack():
    """The in-place refresh (one copy per parameter into its segment, PolicySampler.refresh_weights)
    gives the same block as a fresh pack, before and after the parameters change (include/sit.h:
    W1 [256][10], b1, W2 transposed [256 in][256 out], b2, W3 [2][256], b3)."""
    from sac_maritime_ast_amd import _lib
    from sac_maritime_ast_amd.samplers import pack_actor_weights
    torch.manual_seed(3)
    pol = GaussianPolicy(hidden=(256, 256))
    fresh = pack_actor_weights(pol)
    assert fresh.numel() == _lib.SIT_ACTOR_WEIGHTS and fresh.dtype == torch.float32
    out = torch.full_like(fresh, float("nan"))
    assert pack_actor_weights(pol, out=out) is out
    assert torch.equal(out, fresh)
    with torch.no_grad():
        for p in pol.parameters():
            p.add_(torch.randn_like(p))
    pack_actor_weights(pol, out=out)
    assert torch.equal(out, pack_actor_weights(pol))
    l2 = pol.net[2]
    H = _lib.SIT_ACTOR_HIDDEN
    w2t = out[H * _lib.SIT_OBS_DIM + H:H * _lib.SIT_OBS_DIM + H + H * H].view(H, H)
    assert torch.equal(w2t, l2.weight.detach().t())
    assert pack_actor_weights(GaussianPolicy(hidden=(64, 64))) is None   # other architectures: generic path


def test_pack_actor_weights_rejects_a_wrong_out_buffer():
    """pack_actor_weights(out=...) checks the buffer before writing: its size, dtype and contiguity
    (a larger buffer was partly written with a stale tail, a wrong dtype failed late)."""
    import pytest

    from sac_maritime_ast_amd import _lib
    from sac_maritime_ast_amd.samplers import _trunk, pack_actor_weights
    pol = GaussianPolicy()
    n = _lib.SIT_ACTOR_WEIGHTS
    for bad in (torch.zeros(n + 1), torch.zeros(n - 1), torch.zeros(n, dtype=torch.float64), torch.zeros(2 * n)[::2]):
        with pytest.raises(ValueError):
            pack_actor_weights(pol, out=bad)
    # the PyTorch actor's trunk with fused ReLU epilogues is the network itself
    x = torch.randn(33, 10, dtype=torch.float64)
    p64 = GaussianPolicy().double()
    assert torch.equal(_trunk(p64.net, x), p64.net(x))
