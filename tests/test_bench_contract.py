"""bench.py's output contract (the driver parses it): one JSON line from rank 0 carrying the
BASELINE.json metric, the timing fields, `roofline` and `cpu_baseline`.  A short run of the real
bench on the GPU (few steps, a 0.2 s CPU sample, no extra legs)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line():
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
           "--cpu-seconds", "0.2", "--no-configs", "--e2e-batches", "0", "--timing-launches", "4"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and "workload" in d["config"]
    roof = d["roofline"]
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s"
    assert 0 < roof["achieved"] and 0 < roof["frac"] <= 1.0
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference")
    # every rank checked a sample of its results against the host path (BASELINE multi-GPU runs)
    assert d["parity"] is True and len(d["ranks"]) == 1 and d["ranks"][0]["parity"] is True
    assert d["one_batch_per_launch"]["value"] > 0
