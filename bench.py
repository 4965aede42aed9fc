#!/usr/bin/env python3
"""Benchmark: env-steps/s of the two-ship SAC-AST environment on MI355X (BASELINE.json metric).

A bench "step" is one MultiShipRLEnv.step (RLEnv/MSRL_Env.py:404-442 + MSRL_env_ex.py:906-980)
of every env: both ships (guidance, control, machinery, 3-DOF hull, Euler) plus reward,
termination and status, with the synthetic random-IW sampler and auto-reset.
Config C3: 65 536 ships = 32 768 two-ship envs per GPU (weak scaling over ranks).  Steps run as
fused launches of --chunk steps; every step's full output (next_state[10], reward, done,
status, IW action) is written to HBM.  Inputs (env state) are resident in HBM before timing.

Multi-GPU: one process per GPU.  ``bench.py --gpus N`` started without torchrun's environment
re-launches itself under ``torch.distributed.run`` (N rank processes, 127.0.0.1 rendezvous)
before anything touches a GPU; under torchrun (WORLD_SIZE set) --gpus must equal WORLD_SIZE.
Each rank owns an independent env shard (global env ids offset by rank, no data-path
collective); per launch the replay transitions of its sampling events (the only data the SAC
learner consumes, test_beds/main_ast.py:395-396) go to rank 0 (the learner) over RCCL: the
per-rank counts are all-gathered, then exactly the valid records move point-to-point
(sac_maritime_ast_amd/shard.py).

Timing: W warm-up steps (at least 8 launches: the env population starts synchronised and needs
~40 000 steps to reach the steady state of desynchronised episodes), then K timed steps in
whole launches (at least 3), bracketed by barrier + synchronize, max over ranks.  A "step" is one
env step of every env; with --steps below 3 launches the used count is reported beside the
requested one.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "env-steps/sec at 64k parallel ships, 1/2/4/8 MI355X; fp32 match vs NumPy"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=40000, help="steps before timing (the env population "
                    "starts synchronised; ~40k steps reach the steady state of desynchronised episodes)")
    ap.add_argument("--min-launches", type=int, default=3, help="timed launches at least")
    ap.add_argument("--min-warmup-launches", type=int, default=8, help="warm-up launches at least")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/collective self-check without a GPU (gloo, CPU tensors, synthetic records)")
    ap.add_argument("--n-env", type=int, default=32768, help="two-ship envs per GPU (32768 = 64k ships)")
    ap.add_argument("--chunk", type=int, default=None,
                    help="env steps fused per kernel launch (default 40000; 32 in policy mode): a launch "
                         "ends with its slowest block, so longer launches average the blocks' near-shore "
                         "work (K = 5000 / 10000 / 20000 / 40000: 1.46e10 / 1.54e10 / 1.59e10 / 1.61e10 "
                         "env-steps/s; outputs of every step are written: 85 GB per launch at 40000)")
    ap.add_argument("--precision", type=int, default=32, choices=(32, 64))
    ap.add_argument("--seed", type=int, default=25450)
    ap.add_argument("--mode", default="rollout", choices=("rollout", "step", "policy"),
                    help="rollout: fused K-step launches (synthetic sampler); step: one sit_step launch "
                         "per env step; policy: Gaussian-policy actor between launches (config C5)")
    ap.add_argument("--groups", type=int, default=2, help="policy mode: env groups on separate streams")
    ap.add_argument("--request-div", type=int, default=4,
                    help="policy mode, --serve queue: request capacity = envs / this")
    ap.add_argument("--serve", choices=("kernel", "queue"), default="kernel",
                    help="policy mode: the step kernel serves its waiting envs itself (default), or the request "
                         "queue + sit_policy_actor between launches")
    ap.add_argument("--graph-launches", type=int, default=16, help="policy mode: launches per HIP graph")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=2.5,
                    help="CPU work per baseline process (the whole leg takes ~2 s more for the imports)")
    ap.add_argument("--cpu-baseline-workers", type=int, default=16,
                    help="single-threaded oracle processes (the GPU box's CPU share is 16 cores per GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the replay-transition stream (by default every rank, N = 1 included, writes "
                         "its sampling events' transitions and the learner gathers them)")
    ap.add_argument("--launch-trace", action="store_true", help="print every launch's kernel ms to stderr")
    ap.add_argument("--no-c5", action="store_true", help="rollout mode: skip the config C5 (policy) line")
    ap.add_argument("--c5-steps", type=int, default=32 * 16 * 16, help="timed steps of the C5 line")
    ap.add_argument("--c5-warmup", type=int, default=32 * 16 * 60, help="warm-up steps of the C5 line")
    ap.add_argument("--c5-groups", type=int, default=1, help="C5 line: stream groups (1 measured fastest)")
    ap.add_argument("--c5-chunk", type=int, default=80,
                    help="C5 line: env steps per launch (an env that stops at a sampling event waits for the launch's "
                         "end, so the idle share depends on the launch length against the events' spacing: K = 64 / 72 / "
                         "76 / 80 / 84 / 96 measured 1.57 / 1.66 / 1.56 / 1.66 / 1.64 / 1.53e10, DESIGN.md §9)")
    ap.add_argument("--no-extra-lines", action="store_true",
                    help="rollout mode: skip the secondary lines (C3 in float64, C5 with the PyTorch-ROCm actor)")
    ap.add_argument("--trajectory-stride", type=int, default=0,
                    help="rollout mode: also gather every S-th step's trajectory rows (next_state, reward, done, "
                         "status) of every rank to rank 0 per launch (shard.TrajectoryGather; 0 = off)")
    ap.add_argument("--actor-stream", action="store_true",
                    help="policy mode, --serve queue: the actor on a HIP stream of its own (fork / join per launch)")
    ap.add_argument("--torch-actor", action="store_true",
                    help="policy mode: the actor forward in PyTorch-ROCm on the request queue (north_star's C5 "
                         "wording) instead of the fused HIP actor")
    args = ap.parse_args()
    if args.chunk is None:
        args.chunk = 32 if args.mode == "policy" else 40000
    return args


def algorithmic_bytes_per_launch(n_env, k, rs, mean_nw_obs, mean_nw_test, mode):
    """Bytes a launch must move (no padding, no redundant reloads).  rs = bytes per real."""
    ship_state = 15 * rs + 4 * 4            # 15 reals + next_wpt, n_wpt, ticks, stop
    env_state = 6 * rs + 3 * 4              # sampling/eps dist, prev pos, IW + ep_step, event, episodes
    scen = 2 * 3 * rs + 2 * 8               # per env: end wpt + desired speed per ship, AB len/alpha
    routes = 2 * rs * ((mean_nw_obs - 1) * 2 + (mean_nw_test - 1))   # obs read+write back, test read
    out_step = 15 * rs + 1 + 4              # next_state 10 + reward + IW action 4, done u8, status u32
    # float32: the double-float low parts, 11 per ship and 3 per env (csrc/sit_impl.h kShipLo / kEnvLo)
    lo = (2 * 11 + 3) * rs if rs == 4 else 0
    if mode == "rollout":
        per_env = 2 * (2 * ship_state + env_state + lo) + scen + routes + k * out_step
    else:  # per-step launch: state in and out every step, explicit action in
        per_env = k * (2 * (2 * ship_state + env_state + lo) + scen + 2 * rs * 3 + 2 * rs + 2 + out_step - 4 * rs)
    return n_env * per_env


def latest_pmc(precision, mode, n_env, chunk, serve="kernel"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this exact launch
    configuration (precision, mode, envs, steps per launch; policy mode: in-kernel serving or the
    request queue), if any; the newest round's file wins."""
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if (d.get("precision") == precision and d.get("mode") == mode and d.get("n_env") == n_env
                and d.get("steps_per_launch") == chunk and (mode != "policy" or d.get("serve", "kernel") == serve)):
            best = d
    return best


CPU_WORKER = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
from oracle import sit_oracle as so  # CPU baseline leg only
from sac_maritime_ast_amd.scenario import make_scenario
n_env, seconds, seed, part = int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
sc = make_scenario(n_env, cap=32, seed=seed, env_offset=part * n_env)
o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
o.reset()
o.init_step()
o.rollout(2, seed, env_id_offset=part * n_env)
steps, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < seconds:
    o.rollout(10, seed, env_id_offset=part * n_env)
    steps += 10
print(json.dumps({"env_steps": n_env * steps, "steps": steps, "seconds": time.perf_counter() - t0}))
"""


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, seed, workers):
    """The oracle (float64 NumPy restatement, vectorised over envs) on a bounded sample of the same
    workload: per worker process 2048 envs (its own global env-id range), synthetic sampler,
    auto-reset, ~`seconds` of CPU work; `workers` single-threaded processes on the host cores
    (one process per core), one of them the scalar loop below, all at once (the leg
    takes ~`seconds` + the imports).  Workers are fresh interpreters started as child processes
    (nothing of this GPU process is forked into them); value = the env-steps all vectorised workers
    did / the slowest worker's time."""
    n_env = 2048
    share = max(1, min(workers, len(os.sched_getaffinity(0))))
    cores = max(1, share - 1)
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1",
               PYTHONDONTWRITEBYTECODE="1")
    # BASELINE.md CPU plan 2(a): the reference-equivalent scalar loop (one env, one process, one
    # core), and through the calibration ratio measured in the build container
    # (oracle/calibrate.py: reference / restatement at one env on one core) the reference's own
    # estimated speed on this host, where the reference cannot run
    sp = subprocess.Popen([sys.executable, "-c", CPU_WORKER, ROOT, "1", str(seconds), str(seed), "0"],
                          stdout=subprocess.PIPE, env=env, text=True)
    procs = [subprocess.Popen([sys.executable, "-c", CPU_WORKER, ROOT, str(n_env), str(seconds), str(seed), str(p)],
                              stdout=subprocess.PIPE, env=env, text=True) for p in range(cores)]
    res = []
    for p in procs:
        outp, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"cpu baseline worker failed (exit {p.returncode})")
        res.append(json.loads(outp.strip().splitlines()[-1]))
    total = sum(r["env_steps"] for r in res)
    dt = max(r["seconds"] for r in res)
    sp_out, _ = sp.communicate()
    scalar = None
    if sp.returncode == 0:
        r1 = json.loads(sp_out.strip().splitlines()[-1])
        scalar = {"value": r1["env_steps"] / r1["seconds"], "unit": "env-steps/s", "cores": 1,
                  "sample": f"oracle/sit_oracle.py with one env, {r1['steps']} steps, {r1['seconds']:.1f} s"}
        cal = latest_calibration()
        if cal:
            ratio = cal["env_steps_per_s"]["ratio_reference_over_restatement"]
            scalar["reference_estimate"] = scalar["value"] * ratio
            scalar["calibration"] = {"ratio_reference_over_restatement": ratio, "source": cal["_file"],
                                     "measured_on": cal["cpu_model"]}
    return {"value": total / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "per_core_value": float(np.mean([r["env_steps"] / r["seconds"] for r in res])),
            "cpu_model": _cpu_model(),
            "sample": f"oracle/sit_oracle.py float64 NumPy, {cores} single-threaded processes x {n_env} envs x "
                      f"~{int(np.mean([r['steps'] for r in res]))} steps each (synthetic sampler, auto-reset), "
                      f"{dt:.1f} s wall",
            "scalar_1core": scalar}


def latest_calibration():
    """The newest profiles/*cpu_calibration.json (oracle/calibrate.py), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*cpu_calibration.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    d["_file"] = os.path.relpath(files[-1], ROOT)
    return d


def stats_of(launch_ms):
    v = np.asarray(launch_ms, dtype=np.float64)
    return {"min": float(v.min()), "median": float(np.median(v)), "max": float(v.max())}


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args) -> int:
    """--gpus N without torchrun's environment: run this script as N rank processes under
    torch.distributed.run (a child process, started before anything here touched a GPU), and
    return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch with --gpus equal to the "
                         f"number of rank processes (or without torchrun: bench.py starts them itself)")
    if args.dry_run:
        dev = torch.device("cpu")
        if world > 1:
            torch.distributed.init_process_group("gloo")
        return rank, world, dev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
    return rank, world, dev


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed(dev, world, fn):
    """Barrier + synchronize on both sides of fn(); max over ranks of the wall time."""
    _sync(dev)
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    fn()
    _sync(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def dry_run(args, rank, world, dev):
    """The multi-rank skeleton of bench_rollout on CPU (gloo): the same launcher, shard offsets,
    pipelined transition gather to the learner and max-over-ranks timing, with synthetic records
    (rank r writes 3 + launch + r records per launch) instead of the GPU kernel."""
    from sac_maritime_ast_amd.shard import AsyncTransitionGather, shard_offset
    cap = 64
    g = AsyncTransitionGather(cap, 24, torch.float64, dev, world)
    n_launch = max(args.min_launches, 3)
    got = []

    def run():
        for i in range(n_launch):
            rec, cnt = g.buffers(i)
            n = 3 + i + rank
            rec.zero_()
            rec[:n, 0] = float(i)
            rec[:n, 23] = float(shard_offset(rank, 1000) + rank)
            cnt.fill_(n)
            g.start(i)
            g.progress(i - 1)
            if rank == 0 and i > 0:
                got.append(int(g.records(i - 1).shape[0]))
        g.finish()
        if rank == 0:
            got.append(int(g.records(n_launch - 1).shape[0]))
    elapsed = timed(dev, world, run)
    want = [sum(3 + i + r for r in range(world)) for i in range(n_launch)]
    return {"dry_run": True, "n_gpus": world, "world_size": world, "launches": n_launch, "seconds": elapsed,
            "gathered": g.gathered, "dropped": g.dropped(), "records_per_launch_ok": got == want if rank == 0 else None}


def roofline(alg_bytes, kern_ms, pmc, kernel):
    """kernel: the instantiation the timed launches ran (sit_step_kernel of the handle)."""
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": (pmc["hbm_bytes_per_launch"] if pmc else None),
            "kernel": kernel, "kernel_ms_per_launch": kern_ms,
            "algorithmic_bytes_per_launch": alg_bytes}


def kernel_name(env):
    return env.lib.sit_step_kernel(env.handle).decode()


# VALU issue peak of the chip: 256 CUs x 4 SIMD-32 x one wave64 VALU instruction per 2 cycles at
# 2.4 GHz (MI355X_MICROARCH.md: v_fma_f32 2 cyc/SIMD; one wave alone issues at most every 4)
VALU_PEAK_INST_S = 256 * 4 * 2.4e9 / 2


def roofline_valu(kern_ms, pmc, n_env, chunk):
    """The kernel's binding resource: wave64 VALU instructions issued per second
    against the chip's VALU issue peak.  Instructions per launch from the committed rocprofv3 PMC
    summary of this launch configuration (SQ_INSTS_VALU), time from this run's HIP events."""
    per = (pmc or {}).get("per_wave_step", {}).get("SQ_INSTS_VALU")
    if per is None:
        return {"bound": "valu-issue", "achieved": None, "peak": VALU_PEAK_INST_S, "unit": "wave-instr/s",
                "frac": None, "note": "no PMC summary for this configuration under profiles/"}
    waves = pmc.get("waves") or 2 * ((n_env + 63) // 64)   # the profiled kernel's waves (SQ_WAVES)
    inst = per * waves * chunk
    achieved = inst / (kern_ms * 1e-3)
    return {"bound": "valu-issue", "achieved": achieved, "peak": VALU_PEAK_INST_S, "unit": "wave-instr/s",
            "frac": achieved / VALU_PEAK_INST_S, "valu_per_wave_step": per, "waves": waves,
            "source": pmc.get("source")}


def launch_plan(args, chunk):
    """(timed steps, warm-up steps) in whole launches: >= min_launches timed, >= the requested
    steps; warm-up >= min_warmup_launches and >= the requested warm-up."""
    steps = max(args.min_launches * chunk, -(-args.steps // chunk) * chunk)
    warm = max(args.min_warmup_launches * chunk, -(-args.warmup // chunk) * chunk)
    return steps, warm


def bench_rollout(args, rank, world, dev):
    """Configs C3/C4: synthetic random-IW sampler on device, fused `chunk`-step launches."""
    from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario
    from sac_maritime_ast_amd.shard import AsyncTransitionGather, TrajectoryGather, shard_offset

    n_env = args.n_env
    offset = shard_offset(rank, n_env)
    sc = make_scenario(n_env, cap=48, seed=args.seed, env_offset=offset)
    env = VecMultiShipRLEnv(scenario=sc, precision=args.precision, device=dev)
    env.reset()
    env.init_step()
    chunk = args.chunk if args.mode == "rollout" else 1
    if args.mode == "step":
        steps = max(args.min_launches, args.steps)
        warm = max(args.min_warmup_launches, args.warmup)
    else:
        steps, warm = launch_plan(args, chunk)
    stream = torch.cuda.current_stream(dev)
    # replay transitions of sampling events, written by the kernel with a device-side count and
    # gathered to the learner (rank 0) per launch.  Capacity per rank and launch: the measured
    # steady-state rate is 1 transition per ~390 env-steps (C3; tools/tcount.py), so 1 per 192 is 2x
    # headroom; floor n_env so the synchronised episode start (one event per env) always fits.
    # Records beyond it are counted and reported ("dropped").
    tcap = max(n_env, n_env * chunk // 192)
    # every N, N = 1 included, times the same work: the kernel writes the transitions and the learner
    # gathers them (at N = 1 rank 0 is the learner: the count crosses to the host, no record moves)
    gather = AsyncTransitionGather(tcap, 24, env.dtype, dev, world) if (args.mode == "rollout" and not args.no_gather) \
        else None
    # optional: strided trajectory rows of every rank to the learner, behind each launch
    tgather = (TrajectoryGather(chunk, n_env, args.trajectory_stride, env.dtype, dev, world)
               if args.mode == "rollout" and getattr(args, "trajectory_stride", 0) > 0 else None)
    out = {}
    launch_no = [0]

    if args.mode == "step":   # one sit_step launch per env step, explicit (precomputed) random IWs
        g = torch.Generator(device=dev).manual_seed(args.seed)
        st = env.get_state()
        act = torch.stack([st["north"][1], st["east"][1]], 1) + torch.randn(n_env, 2, device=dev, dtype=env.dtype,
                                                                           generator=g) * 500
        sac = (torch.rand(n_env, device=dev, generator=g) < 0.005).to(torch.uint8)
        init = torch.zeros(n_env, dtype=torch.uint8, device=dev)
        bufs = [torch.empty((n_env, 10), dtype=env.dtype, device=dev), torch.empty(n_env, dtype=env.dtype, device=dev),
                torch.empty(n_env, dtype=torch.uint8, device=dev), torch.empty(n_env, dtype=torch.int32, device=dev),
                torch.zeros(1, dtype=torch.int32, device=dev)]

        def one(ev_pair=None):
            if ev_pair:
                ev_pair[0].record(stream)
            env._call("sit_step", act.data_ptr(), sac.data_ptr(), init.data_ptr(), *[b.data_ptr() for b in bufs],
                      env._stream())
            if ev_pair:
                ev_pair[1].record(stream)
    else:
        def one(ev_pair=None):
            i = launch_no[0]
            if gather:     # this launch's slot of the pipelined transition gather
                out["transitions"], out["transition_count"] = gather.buffers(i)
            if ev_pair:
                ev_pair[0].record(stream)
            env.rollout(chunk, seed=args.seed, env_id_offset=offset, out=out,
                        transition_capacity=tcap if gather else 0)
            if ev_pair:
                ev_pair[1].record(stream)
            if gather:     # counts now, the valid records once this launch's counts are on the host
                gather.start(i)
                gather.progress(i - 1)
            if tgather:
                tgather.start(out)
            launch_no[0] += 1

    for _ in range(warm // chunk):
        one()
    if gather:
        gather.finish()
    if tgather:
        tgather.wait()
    gathered0, dropped0 = (gather.gathered, gather.dropped()) if gather else (0, 0)
    tbytes0 = tgather.bytes_moved if tgather else 0
    n_launch = steps // chunk
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_launch)]

    def run():
        for i in range(n_launch):
            one(ev[i])
        if gather:
            gather.finish()
        if tgather:
            tgather.wait()
    elapsed = timed(dev, world, run)
    launch_ms = [a.elapsed_time(b) for a, b in ev]
    if args.launch_trace:
        print("launch_ms " + " ".join(f"{x:.4f}" for x in launch_ms), file=sys.stderr)
    kern_ms = float(np.median(launch_ms))
    st = env.get_state()
    rs = 4 if args.precision == 32 else 8
    alg = algorithmic_bytes_per_launch(n_env, chunk, rs, float(st["n_wpt"][1].double().mean().item()),
                                       float(st["n_wpt"][0].double().mean().item()), args.mode)
    env_steps = world * n_env * steps
    pmc = latest_pmc(args.precision, args.mode, n_env, chunk)
    rl = roofline(alg, kern_ms, pmc, kernel_name(env))
    rl["algorithmic_bytes_per_env_step"] = alg / (n_env * chunk)
    rl["launch_ms"] = stats_of(launch_ms)
    rl["kernel_ms_statistic"] = "median over the timed launches (HIP events on the launch stream)"
    if args.mode == "step":
        workload = (f"drop-in sit_step: one MultiShipRLEnv.step launch per env step for {n_env} envs "
                    f"({2 * n_env} ships), explicit IW actions, no auto-reset")
    elif world == 1:
        workload = "C3: 65 536 ships = 32 768 two-ship envs per GPU, random IW actions, auto-reset"
    else:
        workload = (f"C4: {2 * n_env * world} ships sharded over {world} GPUs, random IW actions, RCCL gather of "
                    f"the replay transitions to the learner")
    res = {
        "value": env_steps / elapsed, "steps": steps, "warmup": warm, "ms_per_step": elapsed * 1e3 / steps,
        "config": {"workload": workload, "envs_per_gpu": n_env, "ships_per_gpu": 2 * n_env,
                   "fused_steps_per_launch": chunk, "n_launch": n_launch, "mode": args.mode,
                   "parallelism": f"env-shard x{world}", "ship_steps_per_s": 2 * env_steps / elapsed,
                   "steps_requested": args.steps, "warmup_requested": args.warmup},
        "roofline": rl,
        "roofline_valu": roofline_valu(kern_ms, pmc, n_env, chunk) if args.mode == "rollout" else None,
    }
    if tgather is not None:
        res["config"]["rccl_trajectory_gather"] = {
            "to": "rank 0", "stride": args.trajectory_stride, "rows_per_launch_per_rank": tgather.rows,
            "fields": list(TrajectoryGather.FIELDS), "bytes_received_timed": tgather.bytes_moved - tbytes0}
    if gather is not None:
        stats = torch.tensor([gather.gathered - gathered0, gather.dropped() - dropped0], dtype=torch.float64,
                             device=dev)
        res["config"]["rccl_transition_gather"] = {
            "to": "rank 0 (learner)" + (" (N = 1: the learner's own records, no transfer)" if world == 1 else ""),
            "records_gathered": int(stats[0].item()),
            "records_dropped": int(stats[1].item()), "capacity_per_rank_launch": tcap,
            "bytes_per_record": 24 * rs, "pipelining": "count all-gather behind each launch; valid records "
                                                       "point-to-point once the next launch is enqueued"}
    return res


def bench_policy(args, rank, world, dev):
    """Config C5: the SAC-AST Gaussian policy (fp32 actor, 256x256 MLP) chooses the IWs, evaluated by
    the step kernel for its waiting envs at the end of each launch (--serve kernel), or between
    launches on the request queue (--serve queue: sit_policy_actor); envs may be split into `--groups`
    groups on separate HIP streams.  value = env-steps executed (device counter) / time.  At N > 1
    every group's replay transitions (all launches of a HIP graph append to one buffer) go to the
    learner (rank 0) over RCCL after each graph replay, pipelined behind the next replay."""
    from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario
    from sac_maritime_ast_amd.samplers import GaussianPolicy, OverlappedPolicySampler, PolicySampler
    from sac_maritime_ast_amd.shard import AsyncTransitionGather, shard_offset

    n_env, G, chunk = args.n_env, args.groups, args.chunk
    per = n_env // G
    per_graph = max(1, min(args.graph_launches, max(1, args.steps // chunk)))
    gathering = not args.no_gather
    # transitions of one graph replay per group: 1 per ~390 env-steps measured (C3), 1 per 96 here
    tcap = per * chunk * per_graph // 96 if gathering else 0
    torch.manual_seed(args.seed)
    policy = GaussianPolicy(hidden=(256, 256)).to(dev)
    samplers = []
    for g in range(G):
        off = shard_offset(rank, n_env) + g * per
        env = VecMultiShipRLEnv(scenario=make_scenario(per, cap=48, seed=args.seed, env_offset=off),
                                precision=args.precision, device=dev)
        env.reset()
        env.init_step()
        cap = None if args.serve == "kernel" else max(256, per // args.request_div)
        samplers.append(PolicySampler(env, policy, chunk=chunk, seed=args.seed, env_id_offset=off,
                                      request_capacity=cap, transition_capacity=tcap, serve=args.serve,
                                      fused_actor=not getattr(args, "torch_actor", False),
                                      actor_stream=getattr(args, "actor_stream", False) and args.serve == "queue"))
    runner = OverlappedPolicySampler(samplers) if G > 1 else None
    cur = torch.cuda.current_stream(dev)
    # the timed loop: HIP-graph replays of `per_graph` launches of every group
    (runner or samplers[0]).capture(per_graph)
    n_rep = max(2, args.steps // (chunk * per_graph))
    n_warm = max(1, args.warmup // (chunk * per_graph))
    gathers = [AsyncTransitionGather(tcap, 24, samplers[0].env.dtype, dev, world) for _ in range(G)] if gathering else []
    rep_no = [0]

    def replay():
        (runner or samplers[0]).replay()
        i = rep_no[0]
        for g, (sm, ga) in enumerate(zip(samplers, gathers)):
            rec, cnt = ga.buffers(i)
            rec.copy_(sm.out["transitions"])
            cnt.copy_(sm.out["transition_count"])
            ga.start(i)
            ga.progress(i - 1)
        rep_no[0] += 1
    for _ in range(n_warm):
        replay()
    for ga in gathers:
        ga.finish()
    torch.cuda.synchronize(dev)
    # kernel duration of the env launches in the steady state (after the warm-up): eager launches through the
    # sampler, HIP events on each group's stream around the env kernel (the timed replays are HIP graphs)
    n_ev = 16
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
          for _ in range(n_ev)]
    for i in range(n_ev):
        # the GPU kept busy while the host enqueues the launch (an eager launch otherwise starts after its start
        # event by the host's enqueue time: the PyTorch-actor launch's ~20 us of Python)
        torch.cuda._sleep(1_000_000)
        if runner:
            runner.launch(events=ev[i])
        else:
            samplers[0].launch(events=ev[i][0])
    torch.cuda.synchronize(dev)
    launch_ms = [a.elapsed_time(b) for row in ev for a, b in row]
    kern = kernel_name(samplers[0].env)
    g0 = [(ga.gathered, ga.dropped()) for ga in gathers]
    before = sum(int(sm.env_steps.item()) for sm in samplers)

    def run():
        for _ in range(n_rep):
            replay()
        for ga in gathers:
            ga.finish()
    elapsed = timed(dev, world, run)
    n_launch = n_rep * per_graph
    done_steps = sum(int(sm.env_steps.item()) for sm in samplers) - before
    tot = torch.tensor([done_steps], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(tot)
    env_steps = float(tot.item())
    kern_ms = float(np.median(launch_ms))
    rs = 4 if args.precision == 32 else 8
    alg = algorithmic_bytes_per_launch(per, chunk, rs, 3.0, 5.0, "rollout")
    pmc = latest_pmc(args.precision, "policy", per, chunk, args.serve)
    rl = roofline(alg, kern_ms, pmc, kern)
    rl["launch_ms"] = stats_of(launch_ms)
    rl["note"] = "per group launch (n_env / groups envs), groups run concurrently on separate streams"
    rl["kernel_ms_statistic"] = (f"median over {n_ev * G} eager launches after the warm-up (steady state; HIP events on "
                                 f"each group's stream)")
    cfg = {"workload": "C5: 65 536 ships driven by the SAC-AST Gaussian policy (256x256 MLP, fp32, "
                       "evaluated in HIP for the envs waiting at each sampling event) and the HIP env step"
                       if world == 1 else
                       f"C5 x{world}: {2 * n_env * world} policy-driven ships sharded over {world} GPUs",
           "actor": ("in the step kernel (sit_rollout_args.actor_weights)" if args.serve == "kernel" else
                     "sit_policy_actor (fused) on the request queue, capacity n/" + str(args.request_div))
                    if all(sm.fused for sm in samplers) else "PyTorch-ROCm",
           "envs_per_gpu": n_env, "ships_per_gpu": 2 * n_env, "fused_steps_per_launch": chunk,
           "mode": "policy", "stream_groups": G, "launches_per_hip_graph": per_graph,
           "actor_on_own_stream": samplers[0].actor_stream is not None,
           "parallelism": f"env-shard x{world}",
           "env_step_fraction": env_steps / (world * n_env * n_launch * chunk),
           "policy_evaluations": int(sum(int(sm.served.item()) for sm in samplers))}
    if samplers[0].fused:
        # the cost of re-packing the fused actor's weights after an optimizer step (refresh_weights: the
        # reference's SAC updates the policy between env steps, main_ast.py:350-362; here the natural
        # granularity is a launch, so this is the price per policy update), host wall time with sync
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(20):
            samplers[0].refresh_weights()
        torch.cuda.synchronize(dev)
        cfg["refresh_weights_us"] = (time.perf_counter() - t0) / 20 * 1e6
    if gathers:
        stats = torch.tensor([sum(ga.gathered for ga in gathers) - sum(x[0] for x in g0),
                              sum(ga.dropped() for ga in gathers) - sum(x[1] for x in g0)],
                             dtype=torch.float64, device=dev)
        cfg["rccl_transition_gather"] = {
            "to": "rank 0 (learner)", "records_gathered": int(stats[0].item()), "records_dropped": int(stats[1].item()),
            "capacity_per_group_replay": tcap, "pipelining": "per group: count all-gather behind each graph replay; "
                                                            "valid records point-to-point once the next replay is enqueued"}
    return {"value": env_steps / elapsed, "steps": n_launch * chunk, "warmup": n_warm * per_graph * chunk,
            "ms_per_step": elapsed * 1e3 / (n_launch * chunk), "config": cfg, "roofline": rl}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args))
    rank, world, dev = setup_dist(args)
    if args.dry_run:
        r = dry_run(args, rank, world, dev)
        if rank == 0:
            print(json.dumps(r), flush=True)
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    r = bench_policy(args, rank, world, dev) if args.mode == "policy" else bench_rollout(args, rank, world, dev)
    c5 = None
    if args.mode == "rollout" and not args.no_c5:
        # config C5 beside the headline C3/C4 line: policy mode, driver-timed in the same run
        a5 = argparse.Namespace(**vars(args))
        a5.mode, a5.chunk, a5.groups = "policy", args.c5_chunk, args.c5_groups
        a5.steps, a5.warmup = max(args.c5_steps, a5.chunk * 16 * 2), args.c5_warmup
        c5 = bench_policy(a5, rank, world, dev)
    extra = {}
    # (single-GPU runs only: the scaling runs time the headline and the C5 line; the secondary lines
    # would add two more sharded phases per N without adding a scaling measurement)
    if args.mode == "rollout" and not args.no_extra_lines and args.precision == 32 and world == 1:
        # secondary lines (not the headline): C3 in the reference's own float64 arithmetic, and C5 with the
        # actor forward in PyTorch-ROCm on the request queue, on a HIP stream of its own (north_star's C5
        # wording); one group of 64-step launches (tools/c5_torch_sweep.sh, profiles/r06_c5_torch_sweep.json)
        a64 = argparse.Namespace(**vars(args))
        a64.precision, a64.chunk, a64.steps, a64.warmup = 64, 10000, 30000, 40000
        r64 = bench_rollout(a64, rank, world, dev)
        extra["c3_f64"] = {"metric": "env-steps/sec, 65 536 ships per GPU, float64 (the reference's arithmetic)",
                           "value": r64["value"], "unit": "env-steps/s", "dtype": "f64", "steps": r64["steps"],
                           "warmup": r64["warmup"], "ms_per_step": r64["ms_per_step"], "config": r64["config"],
                           "roofline": r64["roofline"]}
        if not args.no_c5:
            at = argparse.Namespace(**vars(args))
            at.mode, at.chunk, at.groups, at.serve, at.torch_actor, at.actor_stream = "policy", 80, 1, "queue", True, True
            at.steps, at.warmup = 80 * 16 * 8, 80 * 16 * 12
            rt = bench_policy(at, rank, world, dev)
            extra["c5_torch_actor"] = {
                "metric": "env-steps/sec, 65 536 policy-driven ships per GPU (config C5), PyTorch-ROCm actor",
                "value": rt["value"], "unit": "env-steps/s", "steps": rt["steps"], "warmup": rt["warmup"],
                "ms_per_step": rt["ms_per_step"], "config": rt["config"], "roofline": rt["roofline"]}
    result = {"metric": METRIC, "value": r["value"], "unit": "env-steps/s", "n_gpus": world, "steps": r["steps"],
              "warmup": r["warmup"], "ms_per_step": r["ms_per_step"], "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "f32" if args.precision == 32 else "f64",
              "data": "synthetic (SURVEY §8(d) routes, island map of test_policy.py:189-194, Philox random IWs)",
              "config": r["config"], "roofline": r["roofline"]}
    if r.get("roofline_valu"):
        result["roofline_valu"] = r["roofline_valu"]
    if c5 is not None:
        result["c5"] = {"metric": "env-steps/sec, 65 536 policy-driven ships per GPU (config C5)", "value": c5["value"],
                        "unit": "env-steps/s", "steps": c5["steps"], "warmup": c5["warmup"],
                        "ms_per_step": c5["ms_per_step"], "config": c5["config"], "roofline": c5["roofline"]}
    result.update(extra)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, args.seed, args.cpu_baseline_workers)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
