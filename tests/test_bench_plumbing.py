"""bench.py's rank plumbing (CPU, no GPU call): `--gpus N` without a launcher spawns N rank
processes; under torch.distributed.run `--gpus` must equal WORLD_SIZE; RCCL ranks each need their own
device, gloo ranks may share (the one-GPU rehearsal).  --plumbing-check DEVICES makes every rank print
its layout and exit before touching the GPU (BASELINE.json north_star: 1, 2, 4 and 8 GPUs)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
sys.path.insert(0, ROOT)


def _run(args, env=None, launcher=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    cmd = (launcher or [sys.executable]) + [BENCH] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=180, env=e)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, sorted(lines, key=lambda d: d["rank"]), r.stderr


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_spawns_n_ranks(n):
    rc, lines, err = _run(["--gpus", str(n), "--plumbing-check", "8"])
    assert rc == 0, err[-2000:]
    assert [d["rank"] for d in lines] == list(range(n))
    assert all(d["world"] == n for d in lines)
    assert [d["device_index"] for d in lines] == list(range(n))  # one GPU per rank
    assert not any(d["shared"] for d in lines)
    assert len({d["master"] for d in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")


def test_gpus_1_is_one_process():
    rc, lines, err = _run(["--plumbing-check", "8"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1 and lines[0]["world"] == 1 and lines[0]["device_index"] == 0


def test_rccl_refuses_ranks_without_a_gpu():
    rc, lines, err = _run(["--gpus", "2", "--plumbing-check", "1"])
    assert rc == 2 and "no GPU of its own" in err


def test_gloo_rehearsal_shares_the_device():
    rc, lines, err = _run(["--gpus", "2", "--plumbing-check", "1", "--dist-backend", "gloo"])
    assert rc == 0, err[-2000:]
    assert [d["device_index"] for d in lines] == [0, 0] and all(d["shared"] for d in lines)


def test_gpus_must_match_the_launchers_world():
    rc, _, err = _run(["--gpus", "3", "--plumbing-check", "8"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert rc == 2 and "WORLD_SIZE=2" in err


def test_under_torchrun():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    launcher = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(port)]
    rc, lines, err = _run(["--gpus", "2", "--plumbing-check", "8"], launcher=launcher)
    assert rc == 0, err[-2000:]
    assert [(d["rank"], d["world"], d["device_index"]) for d in lines] == [(0, 2, 0), (1, 2, 1)]


def test_rank_layout_and_device_count():
    import bench

    a = bench.parse(["--gpus", "4"])
    assert bench.rank_layout(a, {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}, 8) == (4, 3, 3, 3, False)
    with pytest.raises(SystemExit):
        bench.rank_layout(a, {"WORLD_SIZE": "2", "RANK": "0"}, 8)
    assert bench.distinct_devices([{"uuid": "a"}, {"uuid": "a"}]) == 1
    assert bench.distinct_devices([{"uuid": None, "pci_bus_id": 3}, {"uuid": None, "pci_bus_id": 4}]) == 2


def test_split_is_weak_scaling_per_rank():
    """every rank / device runs the full --steps (weak scaling): the launch split of K steps"""
    import bench

    assert bench.split(20, 32) == [0, 20]
    assert bench.split(20, 1) == list(range(21))
    assert bench.widest(200, 32) == 29
