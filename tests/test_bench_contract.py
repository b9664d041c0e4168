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
           "--cpu-seconds", "0.2", "--no-configs", "--no-c4", "--e2e-batches", "0", "--timing-launches", "4"]
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
    assert d["devices_used"] == 1 and d["per_gpu_gibs"] == d["value"]
    r0 = d["ranks"][0]
    assert r0["value"] > 0 and r0["roofline"]["frac"] == roof["frac"] and "uuid" in r0 and "pci_bus_id" in r0
    assert "box" in d and "sclk" in d["box"]


@pytest.mark.gpu
def test_bench_c4_leg_one_gpu():
    """--gpus 1: the C4 leg scans the whole 8 GiB set on the one GPU (one strided launch per pass) and
    its digest matches the golden one; C2 stays the line's value"""
    r, lines = _bench([], timeout=300, c4=True)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["config"]["workload"].startswith("C2:")
    for alg in ("crc32c", "crc64nvme"):
        c4 = d["configs"][f"C4_{alg}"]
        assert c4["digest_match"] is True and c4["parity"] is True and c4["n_gpus"] == 1
        assert c4["ranks"][0]["buffers"] == 1 << 20 and 0 < c4["roofline"]["frac"] <= 1
        # burst, from-idle and sustained regimes
        rg = c4["regimes"]
        assert rg["burst_ms_per_pass"] > 0 and rg["from_idle_ms_per_pass"] > 0 and rg["preload_passes"] >= 1
        assert 0 < c4["ranks"][0]["burst_frac"] <= 1 and 0 < c4["roofline_burst"]["frac"] <= 1


def _bench(args, timeout=300, cpu=False, c4=False):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2", "--no-configs",
           "--e2e-batches", "0", "--timing-launches", "4", "--no-read-ceiling"]
    cmd += ["--cpu-seconds", "0.2"] if cpu else ["--no-cpu-baseline"]
    cmd += ["--c4-passes", "1"] if c4 else ["--no-c4"]
    cmd += args
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


@pytest.mark.gpu
def test_bench_two_ranks_gloo_rehearsal():
    """--gpus 2 without a launcher: two rank processes (here sharing the box's one GPU over gloo, the
    rehearsal of the 8-GPU rank path); rank 0 prints one line with both ranks' records, the C4 leg
    (the full 1M x 8 KiB set, buffer i on rank i mod 2, its gathered digest checked) and the CPU
    baseline timed on rank 0 in the same run"""
    r, lines = _bench(["--gpus", "2", "--dist-backend", "gloo"], timeout=420, cpu=True, c4=True)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["shared_devices"] is True
    assert [x["rank"] for x in d["ranks"]] == [0, 1]
    assert all(x["parity"] is True and x["value"] > 0 and 0 < x["frac"] <= 1 for x in d["ranks"])
    assert d["parity"] is True
    assert d["cpu_baseline"] is not None and d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["parity_with_gpu"]
    assert abs(d["per_gpu_gibs"] * 2 - d["value"]) < 0.05
    for alg in ("crc32c", "crc64nvme"):
        c4 = d["configs"][f"C4_{alg}"]
        assert c4["digest_match"] is True and c4["parity"] is True and c4["scaling"] == "strong"
        assert [x["rank"] for x in c4["ranks"]] == [0, 1] and all(0 < x["frac"] <= 1 for x in c4["ranks"])
        assert sum(x["buffers"] for x in c4["ranks"]) == 1 << 20
        assert c4["cpu_baseline"]["value"] > 0


@pytest.mark.gpu
def test_bench_rccl_refuses_more_ranks_than_gpus():
    import torch

    n = torch.cuda.device_count() + 1
    r, lines = _bench(["--gpus", str(n)], timeout=180)
    assert r.returncode == 2 and "no GPU of its own" in r.stderr and not lines


@pytest.mark.gpu
def test_bench_inproc_per_device_records():
    """--inproc: every device runs the full --steps (weak scaling) with its own roofline and parity"""
    r, lines = _bench(["--inproc", "--gpus", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["scaling"] == "weak" and d["devices_used"] == 1
    assert len(d["devices"]) == 1 and d["devices"][0]["parity"] is True and 0 < d["devices"][0]["frac"] <= 1
    assert d["roofline"]["bound"] == "hbm" and d["value"] > 0
