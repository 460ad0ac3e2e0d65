#!/usr/bin/env python3
"""Where the first launches' extra time comes from (VERDICT r01 "what's weak" #1).

Per-launch HIP-event times of the C2 kernel (1M x 4 KiB, the bench's headline launch) in four
situations, each 100 back-to-back launches:
  A  fresh process, fresh buffer (what `bench.py --warmup 5` times)
  B  the same buffer after the GPU idled 2 s            (cold GPU, warm buffer)
  C  a NEW 4-GiB buffer right after B                   (warm GPU, fresh buffer: page-table /
                                                          TLB first-touch would show here)
  D  the load-only kernel with the same loads (read_pattern4k 21) after 2 s idle
                                                         (no CRC work: clock / power vs memory)
and, if amd-smi answers, the GPU clocks sampled before and after.  Prints one JSON object.
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c, diag  # noqa: E402

NBLK = 1 << 20


def timed(fn, n=100):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b), 4) for a, b in ev]


class SysfsSampler:
    """Samples the GPUs' hwmon SCLK (freq1_input), power (power1_input / power1_average) and the
    active pp_dpm_sclk level every ~1 ms in a background thread (read-only sysfs), so a launch
    sequence can be lined up with the clock the power manager gave it."""

    def __init__(self):
        import glob
        import threading

        self.files = {}
        for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
            card = dev.split("/")[4]
            for hw in glob.glob(dev + "/hwmon/hwmon*"):
                for nm in ("freq1_input", "power1_input", "power1_average", "temp2_input"):
                    if os.path.exists(os.path.join(hw, nm)):
                        self.files[f"{card}:{nm}"] = os.path.join(hw, nm)
        self.samples = []
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        while not self._stop.is_set():
            row = {"t_ms": round((time.perf_counter() - t0) * 1e3, 2)}
            for k, p in self.files.items():
                try:
                    with open(p) as f:
                        row[k] = int(f.read().strip())
                except (OSError, ValueError):
                    pass
            self.samples.append(row)
            time.sleep(0.001)

    def __enter__(self):
        self._th.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        self._th.join()

    def busy_card(self):
        """The card whose SCLK moved the most (the one our kernels ran on)."""
        best, spread = None, -1
        for k in self.files:
            if k.endswith("freq1_input"):
                v = [r[k] for r in self.samples if k in r]
                if v and max(v) - min(v) > spread:
                    best, spread = k.split(":")[0], max(v) - min(v)
        return best

    def trace(self):
        c = self.busy_card()
        if c is None:
            return None
        keys = [k for k in self.files if k.startswith(c + ":")]
        return {"card": c, "rows": [[r["t_ms"]] + [r.get(k) for k in keys] for r in self.samples], "cols": ["t_ms"] + keys}


def clocks():
    try:
        r = subprocess.run(["amd-smi", "metric", "-g", "0", "-c", "--json"], capture_output=True, text=True, timeout=20)
        return r.stdout[-1500:] if r.returncode == 0 else None
    except Exception as e:  # noqa: BLE001 -- diagnostics only
        return repr(e)


def summary(t):
    t = np.array(t)
    return {"first10": t[:10].tolist(), "mean_0_10": round(float(t[:10].mean()), 4),
            "mean_10_40": round(float(t[10:40].mean()), 4), "mean_40_100": round(float(t[40:].mean()), 4),
            "min": round(float(t.min()), 4)}


def main():
    crc32c.init_device(0)
    res = {"clocks_before": clocks()}
    t0 = time.perf_counter()
    d1 = torch.empty(NBLK * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d1, 301)
    out = torch.empty(NBLK, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    res["alloc_fill_s"] = round(time.perf_counter() - t0, 3)
    res["A_fresh"] = summary(timed(lambda: crc32c.batch_fixed(d1, 4096, 4096, NBLK, out=out)))
    res["clocks_after_A"] = clocks()
    time.sleep(2.0)
    res["B_idle2s_same_buffer"] = summary(timed(lambda: crc32c.batch_fixed(d1, 4096, 4096, NBLK, out=out)))
    d2 = torch.empty(NBLK * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d2, 302)
    res["C_warm_gpu_new_buffer"] = summary(timed(lambda: crc32c.batch_fixed(d2, 4096, 4096, NBLK, out=out)))
    del d2
    o = torch.zeros(1, dtype=torch.int32, device="cuda")
    time.sleep(2.0)
    res["D_idle2s_load_only"] = summary(timed(lambda: diag.read_pattern4k(d1, NBLK, 21, o)))
    time.sleep(2.0)
    with SysfsSampler() as smp:
        time.sleep(0.02)
        tE = time.perf_counter()
        e_times = timed(lambda: crc32c.batch_fixed(d1, 4096, 4096, NBLK, out=out), 200)
        res["E_launches_end_ms"] = round((time.perf_counter() - tE) * 1e3, 2)
        time.sleep(0.02)
    res["E_idle2s_crc_again"] = summary(e_times)
    res["E_per_launch_ms"] = e_times
    res["E_sysfs"] = smp.trace()
    time.sleep(2.0)
    with SysfsSampler() as smp2:
        time.sleep(0.02)
        d_times = timed(lambda: diag.read_pattern4k(d1, NBLK, 21, o), 200)
        time.sleep(0.02)
    res["F_load_only_per_launch_ms"] = d_times
    res["F_sysfs"] = smp2.trace()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
