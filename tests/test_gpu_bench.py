"""bench.py's output contract, on the GPU: the one JSON line the driver reads (its keys, the
roofline and cpu_baseline objects), and that the timed region times the fits and nothing else
(every step's wall time equals the fit's own total)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_contract_c2():
    steps = 2
    proc = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--config", "c2",
                           "--steps", str(steps), "--warmup", "1", "--no-consensus-roofline"],
                          cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert proc.returncode == 0, proc.stderr[-2000:]
    lines = [ln for ln in proc.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, proc.stdout[-2000:]  # exactly one JSON line
    d = json.loads(lines[0])

    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] in ("weak", "strong")
    assert d["unit"] == "resample-clusterings/s" and "workload" in d["config"]

    # value = every clustering of the timed fits over the timed wall time
    H, (K0, K1) = d["config"]["H"], d["config"]["K_range"]
    clusterings = H * (K1 - K0 + 1)
    assert d["value"] == pytest.approx(clusterings / (d["ms_per_step"] * 1e-3), rel=1e-9)

    # the timed region is the fits: each step's wall time is its fit's own total
    assert len(d["step_ms"]) == steps == len(d["fit_total_ms"])
    for wall, fit in zip(d["step_ms"], d["fit_total_ms"]):
        assert abs(wall - fit) < 5.0, (d["step_ms"], d["fit_total_ms"])
    assert sum(d["step_ms"]) <= steps * d["ms_per_step"] + 1e-6

    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma") and r["unit"] in ("GB/s", "TFLOP/s")
    assert 0.0 < r["frac"] <= 1.0
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-9)
    # achieved = the kernel's credited flops per launch over its HIP-event launch time
    assert r["achieved"] == pytest.approx(r["flops_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e12, rel=1e-9)
    assert r["executed_flops_per_launch"] >= r["flops_per_launch"]  # padding slots only add work
    co = d["roofline_coassoc"]
    assert 0.0 < co["frac"] <= 1.0

    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["value"] > 0 and cb["kind"] in ("reference", "port") and cb["cores"] >= 1
