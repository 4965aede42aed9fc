"""Host-side pieces of bench.py (no GPU): the algorithmic-bytes model and the CPU-baseline leg."""
import pytest

import bench


def test_algorithmic_bytes_per_env_step_rollout():
    # f32, K = 5000: 65 B of outputs per env-step plus the per-launch state/scenario/route traffic
    n_env, k = 32768, 5000
    b = bench.algorithmic_bytes_per_launch(n_env, k, 4, 3.0, 5.0, "rollout")
    per = b / (n_env * k)
    assert 65.0 < per < 65.2
    # longer launches amortise the state read/write: bytes per env-step fall towards 65
    b200 = bench.algorithmic_bytes_per_launch(n_env, 200, 4, 3.0, 5.0, "rollout") / (n_env * 200)
    assert b200 > per


def test_cpu_baseline_workers_report():
    r = bench.cpu_baseline(0.5, 25450, 3)     # 2 vectorised workers + the scalar loop, concurrently
    assert r["kind"] == "port" and r["unit"] == "env-steps/s"
    assert r["cores"] == 2 and r["value"] > 0 and r["per_core_value"] > 0
    assert "2 single-threaded processes" in r["sample"]
    sc = r["scalar_1core"]
    assert sc["cores"] == 1 and sc["value"] > 0
    if bench.latest_calibration() is not None:
        assert sc["reference_estimate"] == pytest.approx(sc["value"] * sc["calibration"]["ratio_reference_over_restatement"])


def _run_bench(*argv, env_extra=None, timeout=300):
    import json
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"), *argv],
                       capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_gpus_flag_starts_ranks_itself():
    """`bench.py --gpus 2` without torchrun's environment re-launches itself as 2 rank processes
    (torch.distributed.run, 127.0.0.1); rank 0 prints one JSON line with n_gpus = world size = 2
    after the pipelined transition gather moved every rank's records to the learner (gloo here,
    RCCL on the GPU node)."""
    rc, line, err = _run_bench("--gpus", "2", "--dry-run")
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["dry_run"]
    assert line["records_per_launch_ok"] is True and line["dropped"] == 0
    assert line["gathered"] == sum(3 + i + r for i in range(line["launches"]) for r in range(2))


def test_bench_rejects_gpus_world_size_mismatch():
    rc, line, err = _run_bench("--gpus", "4", "--dry-run", env_extra={"WORLD_SIZE": "2", "RANK": "0",
                                                                       "LOCAL_RANK": "0"})
    assert rc != 0 and line is None
    assert "WORLD_SIZE=2" in err


def test_launch_plan_whole_launches():
    import argparse
    a = argparse.Namespace(steps=20, warmup=5, min_launches=3, min_warmup_launches=8)
    assert bench.launch_plan(a, 5000) == (15000, 40000)
    a = argparse.Namespace(steps=20001, warmup=45000, min_launches=3, min_warmup_launches=8)
    assert bench.launch_plan(a, 5000) == (25000, 45000)
