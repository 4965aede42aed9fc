import sys, torch
sys.path.insert(0, "/root/repo")
from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario
n_env, chunk = 32768, 5000
sc = make_scenario(n_env, cap=48, seed=25450)
env = VecMultiShipRLEnv(scenario=sc, precision=32, device="cuda:0")
env.reset(); env.init_step()
out = {}
cap = n_env * chunk // 64
for i in range(12):
    env.rollout(chunk, seed=25450, out=out, transition_capacity=cap)
    c = int(out["transition_count"].item())
    print(f"launch {i}: transitions {c} = 1 per {n_env*chunk/c:.0f} env-steps (cap {cap})", flush=True)
