"""Per-wave timeline of crc32_stream_kernel (diagnostic library: aws_crt_amd_debug_scan_stamps) on the
headline's launches -- one C2 batch (1024 x 64 KiB) and the driver's 20-batch launch -- to see where
a launch's time goes beyond its bytes: the dispatch ramp (entry spread), the
table build + barrier, the wait for the first group, the waves' lives against the launch span, the
tail (exit percentiles) and the spread by XCD.  s_memrealtime ticks at 100 MHz (10 ns).

  python aws-crt-cpp_amd/tools/stamp_probe.py [reps]   -> one JSON line per launch shape
"""
import ctypes
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402

TICK_US = 0.01
W = 16  # words per wave (crc_kernels.hip kStampWords)


def pct(v, ps=(0, 10, 50, 90, 99, 100)):
    s = sorted(v)
    return [round(s[min(len(s) - 1, int(p / 100 * (len(s) - 1) + 0.5))], 2) for p in ps]


def hw_fields(hwid):
    """gfx9 HW_ID: wave [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]; XCC_ID in the high word"""
    return {"simd": (hwid >> 4) & 3, "cu": ((hwid >> 32) & 0xF, (hwid >> 13) & 7, (hwid >> 12) & 1, (hwid >> 8) & 0xF)}


def by_cu_order(rows, idx):
    """the two workgroups sharing a CU: the one entering first against the second (oldest-first issue
    would favour the first), and the spread over SIMDs"""
    cus = {}
    for r, i in zip(rows, idx):
        if r[6] == 0:
            continue
        f = hw_fields(r[5])
        cus.setdefault(f["cu"], {}).setdefault(i // 8, []).append(r)
    first, second = [], []
    nblocks = max(idx) // 8 + 1 if idx else 0
    low_first = 0
    for wgs in cus.values():
        if len(wgs) != 2:
            continue
        (ba, a), (bb, b) = sorted(wgs.items(), key=lambda kv: min(w[0] for w in kv[1]))
        low_first += ba < nblocks // 2 <= bb
        first += [(w[4] - w[0]) * TICK_US for w in a]
        second += [(w[4] - w[0]) * TICK_US for w in b]
    simd = {}
    for r in rows:
        if r[6]:
            simd.setdefault(hw_fields(r[5])["simd"], []).append((r[4] - r[0]) * TICK_US)
    out = {"cus_with_two_workgroups": sum(1 for w in cus.values() if len(w) == 2),
           "first_workgroup_in_lower_half_of_grid": low_first,
           "simd_mean_life_us": {k: round(statistics.mean(v), 2) for k, v in sorted(simd.items())}}
    if first:
        out["first_workgroup_life_us"] = pct(first)
        out["second_workgroup_life_us"] = pct(second)
    return out


def analyse(st, nw):
    idx = [i for i in range(nw) if st[i * W + 4] != 0]
    rows = [st[i * W:(i + 1) * W] for i in idx]
    t0 = min(r[0] for r in rows)
    us = lambda t: (t - t0) * TICK_US  # noqa: E731
    entry = [us(r[0]) for r in rows]
    ex = [us(r[4]) for r in rows]
    span = max(ex)
    work = [r for r in rows if r[6] > 0]
    tab = [(r[1] - r[0]) * TICK_US for r in rows]
    pro = {name: pct([(r[k] - r[0]) * TICK_US for r in work]) for name, k in
           (("kernel_args_in_us", 8), ("first_group_issued_us", 9), ("second_group_issued_us", 10),
            ("tables_stored_us", 11), ("barrier_passed_us", 1))}
    first = [(r[2] - r[1]) * TICK_US for r in work]
    life = [(r[4] - r[0]) * TICK_US for r in work]
    fin = [(r[4] - r[3]) * TICK_US for r in work]
    per_group = [((r[3] - r[2]) * TICK_US) / max(1, r[6] - 1) for r in work if r[6] > 1]
    xcc = {}
    for r, e, lf in zip(work, [us(r[4]) for r in work], life):
        x = (r[5] >> 32) & 0xF
        xcc.setdefault(x, []).append((e, lf))
    by_xcc = {x: {"waves": len(v), "mean_life_us": round(statistics.mean(l for _, l in v), 2),
                  "max_exit_us": round(max(e for e, _ in v), 2), "median_exit_us": round(statistics.median(e for e, _ in v), 2)}
              for x, v in sorted(xcc.items())}
    return {"waves": len(rows), "working_waves": len(work), "groups_per_wave": pct([r[6] for r in work], (0, 50, 100)),
            "span_us": round(span, 2), "entry_us": pct(entry), "tables_us": pct(tab), "prologue_from_entry": pro, "first_group_us": pct(first),
            "per_group_us": pct(per_group), "life_us": pct(life), "mean_life_frac": round(statistics.mean(life) / span, 4),
            "final_finish_us": pct(fin), "exit_us": pct(ex), "by_xcc": by_xcc, "by_cu": by_cu_order(rows, idx)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    D = eng.diag_lib()
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    D.aws_crt_amd_init()
    D.aws_crt_amd_debug_scan_stamps.argtypes = [vp]
    D.aws_crt_amd_plan_create.argtypes = [ctypes.c_int, ctypes.POINTER(eng._Batch), sz, sz, sz, sz, ctypes.POINTER(vp)]
    D.aws_crt_amd_plan_launch.argtypes = [vp, vp]
    D.aws_crt_amd_plan_destroy.argtypes = [vp]
    D.aws_crt_amd_profile_next_launch.argtypes = [vp, vp]
    D.aws_crt_amd_profile_elapsed_ms.argtypes = [vp, vp]
    D.aws_crt_amd_profile_elapsed_ms.restype = ctypes.c_float
    count, L, nb = 1024, 65536, 20
    step = count * L
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    data = torch.randint(0, 256, (nb * step,), dtype=torch.uint8, device="cuda", generator=g)
    outs = [torch.empty(count, dtype=torch.int32, device="cuda") for _ in range(nb)]
    nwmax = 256 * 2 * 8 * 2
    stamps = torch.zeros(nwmax * W, dtype=torch.int64, device="cuda")
    assert D.aws_crt_amd_debug_scan_stamps(vp(stamps.data_ptr())) == 0
    st = torch.cuda.current_stream()
    for nbatch in (1, nb):
        arr = (eng._Batch * nbatch)()
        for i in range(nbatch):
            arr[i].d_base, arr[i].d_seeds, arr[i].d_out = data.data_ptr() + i * step, None, outs[i].data_ptr()
        h = vp()
        assert D.aws_crt_amd_plan_create(1, arr, nbatch, L, L, count, ctypes.byref(h)) == 0
        res = []
        for r in range(reps + 1):
            stamps.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            e1.record(st)
            D.aws_crt_amd_profile_next_launch(vp(e0.cuda_event), vp(e1.cuda_event))
            assert D.aws_crt_amd_plan_launch(h, vp(st.cuda_stream)) == 0
            torch.cuda.synchronize()
            ms = D.aws_crt_amd_profile_elapsed_ms(vp(e0.cuda_event), vp(e1.cuda_event))
            if r == 0:
                continue  # first launch of the shape: warm-up
            a = analyse(stamps.cpu().tolist(), nwmax)
            a["kernel_us_events"] = round(ms * 1e3, 2)
            a["frac"] = round(nbatch * step / (ms * 1e-3) / 8e12, 4)
            res.append(a)
        D.aws_crt_amd_plan_destroy(h)
        best = sorted(res, key=lambda a: a["kernel_us_events"])[len(res) // 2]  # the median launch
        print(json.dumps({"shape": f"{nbatch} x C2 batch ({nbatch * step >> 20} MiB)",
                          "kernel_us_all": [a["kernel_us_events"] for a in res], "median_launch": best}), flush=True)
    assert D.aws_crt_amd_debug_scan_stamps(vp(0)) == 0
    # results still right with the stamps on (the first 64 buffers of batch 0 against the host path)
    hs = data[: 64 * L].cpu().numpy()
    want = eng.cpu_batch(eng.CRC32C, [hs.ctypes.data + i * L for i in range(64)], [L] * 64)
    assert eng.as_unsigned(outs[0])[:64] == want, "parity"
    print(json.dumps({"parity": True}))


if __name__ == "__main__":
    main()
