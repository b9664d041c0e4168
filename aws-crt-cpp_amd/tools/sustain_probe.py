"""Time series of back-to-back scans of one shape after an idle hold: the duration of every launch, so
that a launch-length effect (drift inside one launch) and a power-management transient (launches
slowing down some milliseconds into a burst, then recovering) can be told apart.

    python aws-crt-cpp_amd/tools/sustain_probe.py [--shape c4full|c2_20|c5_20] [--alg crc64nvme]
                                                   [--launches 40] [--hold-ms 10] [--ceiling]

Prints one JSON line per run: per-launch ms (events between launches on one stream), and the mean of
launches in windows of the burst.
"""
import argparse
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402
import bench  # noqa: E402

PEAK = 8.0e12
SHAPES = {"c4full": (1 << 20, 8192, 1), "c2_20": (1024, 65536, 20), "c5_20": (8, 64 << 20, 20),
          "c5_1": (8, 64 << 20, 1), "c4": (131072, 8192, 1)}


class Metrics:
    """amdsmi gpu_metrics samples (read-only) of the device in use, on a thread, host-timestamped"""

    KEYS = ("current_gfxclk", "current_gfxclks", "current_socket_power", "average_socket_power", "current_uclk",
            "throttle_status", "indep_throttle_status", "temperature_hotspot", "ppt_residency_acc",
            "socket_thm_residency_acc", "firmware_timestamp")

    def __init__(self, bdf):
        import amdsmi
        self.m = amdsmi
        amdsmi.amdsmi_init()
        hs = amdsmi.amdsmi_get_processor_handles()
        self.h = next((h for h in hs if amdsmi.amdsmi_get_gpu_device_bdf(h).lower().endswith(bdf.lower())), None)
        if self.h is None:
            raise RuntimeError(f"no amdsmi handle for {bdf}")
        self.samples, self.run = [], False

    def one(self):
        d = self.m.amdsmi_get_gpu_metrics_info(self.h)
        return {k: d.get(k) for k in self.KEYS}

    def start(self):
        self.run, self.samples = True, []

        def loop():
            while self.run:
                t = time.perf_counter()
                try:
                    self.samples.append((t, self.one()))
                except Exception as e:  # noqa: BLE001
                    self.samples.append((t, {"error": str(e)}))
                time.sleep(0.0005)
        self.th = threading.Thread(target=loop, daemon=True)
        self.th.start()

    def stop(self):
        self.run = False
        self.th.join()
        return self.samples


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c4full")
    ap.add_argument("--algs", default="crc64nvme,crc32c")
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--hold-ms", type=float, default=10.0)
    ap.add_argument("--ceiling", action="store_true", help="also the read-ceiling kernel (diagnostic build)")
    ap.add_argument("--metrics", action="store_true", help="sample amdsmi gpu_metrics during the burst")
    a = ap.parse_args()
    eng.init()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    n, L, nb = SHAPES[a.shape]
    step = n * L
    data = torch.empty((nb + 1) * step, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5A)
    for j in range(nb + 1):
        data[j * step:(j + 1) * step].copy_(torch.randint(0, 256, (step,), dtype=torch.uint8, device=dev, generator=g))
    met = None
    if a.metrics:
        pr = torch.cuda.get_device_properties(0)
        bdf = f"{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        try:
            met = Metrics(bdf)
            print(json.dumps({"metrics_device": bdf, "idle_sample": met.one()}), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"metrics_error": repr(e), "bdf": bdf}), flush=True)
            met = None
    kinds = a.algs.split(",") + (["read_ceiling"] if a.ceiling else [])
    for kind in kinds:
        if kind == "read_ceiling":
            def go(i):
                eng.read_ceiling(data, nb * step, stream=st, base_offset=(i % 2) * step)
        else:
            outs = [torch.empty(n, dtype=torch.int64 if kind == "crc64nvme" else torch.int32, device=dev)
                    for _ in range(nb + 1)]

            def go(i, kind=kind, outs=outs):
                o = i % 2
                eng.checksum_batches(bench.ALG[kind], [(data.data_ptr() + ((o + j) % (nb + 1)) * step, None,
                                                        outs[(o + j) % (nb + 1)]) for j in range(nb)], L, L, n, stream=st)
        go(0)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.launches + 1)]
        if met:
            met.start()
            time.sleep(0.02)
        if a.hold_ms > 0:
            with torch.cuda.stream(st):
                torch.cuda._sleep(int(a.hold_ms * 2e6))
        ev[0].record(st)
        for i in range(a.launches):
            go(i)
            ev[i + 1].record(st)
        tb = None
        while not ev[0].query():
            pass
        tb = time.perf_counter()  # host time of the burst's start (within the query loop's latency)
        torch.cuda.synchronize()
        if met:
            time.sleep(0.02)
            smp = met.stop()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.launches)]
        w = max(1, a.launches // 8)
        windows = [round(sum(ms[i:i + w]) / len(ms[i:i + w]), 4) for i in range(0, a.launches, w)]
        t = 0.0
        starts = []
        for m in ms:
            starts.append(round(t, 3))
            t += m
        print(json.dumps({"shape": a.shape, "kind": kind, "bytes_per_launch": nb * step, "hold_ms": a.hold_ms,
                          "ms": [round(x, 4) for x in ms], "start_ms": starts,
                          "frac": [round(nb * step / (x * 1e-3) / PEAK, 3) for x in ms],
                          "window_launches": w, "window_mean_ms": windows}), flush=True)
        if met:
            print(json.dumps({"kind": kind, "metrics": [dict(v, t_ms=round((t - tb) * 1e3, 3)) for t, v in smp]}), flush=True)


if __name__ == "__main__":
    main()
