"""Host-side pieces of bench.py (no GPU): the algorithmic-bytes model and the CPU-baseline leg."""
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
    r = bench.cpu_baseline(0.5, 25450, 2)
    assert r["kind"] == "port" and r["unit"] == "env-steps/s"
    assert r["cores"] == 2 and r["value"] > 0 and r["per_core_value"] > 0
    assert "2 single-threaded processes" in r["sample"]
