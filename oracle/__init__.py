"""oracle -- TEST INFRASTRUCTURE ONLY (the checker, never the thing measured or shipped).

ctypes bindings for
  * ``_build/liboracle.so``  -- the C restatement of the reference CRC32C
    (oracle/crc32c_oracle.c; cites /root/reference/src/util/crc32c.cc:25-32,585-625)
  * ``_ref/libpdbref.so``    -- the reference's own util/crc32c.cc compiled in place by
    oracle/build_ref.sh (only present where /root/reference was available at build time;
    the .so travels to the GPU box, the reference sources do not)
plus the numpy twin of the splitmix64 synthetic-data generator.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libpdbref.so")

BLK_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("init", "<u4")])  # == pdb_blk / oracle_blk

_u8p = ctypes.c_void_p


def build() -> None:
    """Compile the C restatement and, when the reference is present, the reference shim and
    the reference's db_bench (as-is and GPU-hooked; needs pebblesdb_amd's library built)."""
    subprocess.check_call([os.path.join(HERE, "build_oracle.sh")])
    subprocess.check_call([os.path.join(HERE, "build_ref.sh")])
    subprocess.check_call([os.path.join(HERE, "build_ref_dbbench.sh")])


def _bind(lib, prefix: str) -> None:
    lib_ext = getattr(lib, f"{prefix}_crc32c_extend")
    lib_ext.restype = ctypes.c_uint32
    lib_ext.argtypes = [ctypes.c_uint32, _u8p, ctypes.c_size_t]
    for nm in ("mask", "unmask"):
        f = getattr(lib, f"{prefix}_crc32c_{nm}")
        f.restype = ctypes.c_uint32
        f.argtypes = [ctypes.c_uint32]
    b = getattr(lib, f"{prefix}_crc32c_batch")
    b.restype = ctypes.c_int
    b.argtypes = [_u8p, _u8p, ctypes.c_size_t, ctypes.c_uint32, _u8p, ctypes.c_int]


class _CrcLib:
    def __init__(self, path: str, prefix: str):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.path = path
        self.prefix = prefix
        self.lib = ctypes.CDLL(path)
        _bind(self.lib, prefix)
        self._extend = getattr(self.lib, f"{prefix}_crc32c_extend")
        self._mask = getattr(self.lib, f"{prefix}_crc32c_mask")
        self._unmask = getattr(self.lib, f"{prefix}_crc32c_unmask")
        self._batch = getattr(self.lib, f"{prefix}_crc32c_batch")

    def extend(self, init: int, data) -> int:
        buf = _as_u8(data)
        return int(self._extend(init & 0xFFFFFFFF, buf.ctypes.data, buf.size))

    def value(self, data) -> int:
        return self.extend(0, data)

    def mask(self, c: int) -> int:
        return int(self._mask(c & 0xFFFFFFFF))

    def unmask(self, c: int) -> int:
        return int(self._unmask(c & 0xFFFFFFFF))

    def batch(self, base: np.ndarray, blk: np.ndarray, flags: int = 0, nthreads: int = 1) -> np.ndarray:
        base = _as_u8(base)
        blk = np.ascontiguousarray(blk, dtype=BLK_DTYPE)
        out = np.zeros(len(blk), dtype=np.uint32)
        rc = self._batch(base.ctypes.data, blk.ctypes.data, len(blk), flags, out.ctypes.data, nthreads)
        if rc != 0:
            raise RuntimeError(f"{self.prefix} batch rc={rc}")
        return out


class Oracle(_CrcLib):
    """The C restatement (always available: built from repo sources)."""

    def __init__(self, path: str = ORACLE_SO):
        super().__init__(path, "oracle")
        self._bitwise = self.lib.oracle_crc32c_extend_bitwise
        self._bitwise.restype = ctypes.c_uint32
        self._bitwise.argtypes = [ctypes.c_uint32, _u8p, ctypes.c_size_t]
        self._fill = self.lib.oracle_fill_splitmix
        self._fill.restype = None
        self._fill.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]

    def extend_bitwise(self, init: int, data) -> int:
        buf = _as_u8(data)
        return int(self._bitwise(init & 0xFFFFFFFF, buf.ctypes.data, buf.size))

    def fill(self, nbytes: int, seed: int, byte_offset: int = 0) -> np.ndarray:
        out = np.empty(nbytes, dtype=np.uint8)
        self._fill(out.ctypes.data, nbytes, seed & 0xFFFFFFFFFFFFFFFF, byte_offset)
        return out


class Reference(_CrcLib):
    """The reference's own util/crc32c.cc, compiled in place (oracle/_ref)."""

    def __init__(self, path: str = REF_SO):
        super().__init__(path, "ref")
        self._dbb = getattr(self.lib, "ref_crc32c_dbbench_loop", None)
        if self._dbb is not None:
            self._dbb.restype = ctypes.c_double
            self._dbb.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]

    def dbbench_crc32c(self, total: int = 500 << 20) -> tuple[float, int]:
        """db_bench's `crc32c` loop (db/db_bench.cc:1112-1129) in C: (MiB/s, last crc)."""
        if self._dbb is None:
            raise RuntimeError("oracle/_ref/libpdbref.so predates ref_crc32c_dbbench_loop; rebuild")
        c = ctypes.c_uint32(0)
        secs = self._dbb(total, ctypes.byref(c))
        return total / secs / (1 << 20), int(c.value)


def timed_batch(crc, base, blk, nthreads: int, seconds: float = 1.0, cpus=None) -> dict:
    """Host CPU throughput of `crc` (an Oracle or Reference) over the sample (base, blk): nthreads
    threads, each hashing its own contiguous slice of the blocks over and over until `seconds`
    have passed, started together on a barrier (no thread creation inside the timed window).
    ctypes drops the GIL for the duration of each call, so the threads run in parallel; a call
    hashes a whole slice (>= MiBs), so the Python loop costs nothing measurable.  cpus: pin thread t
    to cpus[t % len(cpus)] (NUMA-node runs).  Returns {"GiB/s", "threads", "seconds", "bytes"}."""
    base = _as_u8(base)
    blk = np.ascontiguousarray(blk, dtype=BLK_DTYPE)
    nthreads = max(1, min(int(nthreads), len(blk)))
    lens = blk["len"].astype(np.int64)
    cuts = [len(blk) * t // nthreads for t in range(nthreads + 1)]
    slice_bytes = [int(lens[cuts[t] : cuts[t + 1]].sum()) for t in range(nthreads)]
    reps = [0] * nthreads
    stop = threading.Event()
    start = threading.Barrier(nthreads + 1)

    def work(t):
        if cpus:
            try:
                os.sched_setaffinity(0, {cpus[t % len(cpus)]})
            except OSError:
                pass
        part = blk[cuts[t] : cuts[t + 1]]
        start.wait()
        while not stop.is_set():
            crc.batch(base, part, nthreads=1)
            reps[t] += 1

    th = [threading.Thread(target=work, args=(t,), daemon=True) for t in range(nthreads)]
    for x in th:
        x.start()
    start.wait()
    t0 = time.perf_counter()
    time.sleep(seconds)
    stop.set()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    total = sum(r * b for r, b in zip(reps, slice_bytes))
    return {"GiB/s": total / dt / (1 << 30), "threads": nthreads, "seconds": dt, "bytes": total}


def host_cpus() -> dict:
    """The host's CPU picture: logical CPUs, the ones this process may run on, a cgroup CPU quota
    if one is set, and the CPUs of every NUMA node."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": None, "numa": {}}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                info["cgroup_cpu_quota"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    node_dir = "/sys/devices/system/node"
    try:
        for d in sorted(os.listdir(node_dir)):
            if d.startswith("node") and d[4:].isdigit():
                with open(os.path.join(node_dir, d, "cpulist")) as f:
                    cpus = []
                    for part in f.read().strip().split(","):
                        if part:
                            a, _, b = part.partition("-")
                            cpus.extend(range(int(a), int(b or a) + 1))
                allowed = os.sched_getaffinity(0)
                info["numa"][d] = [c for c in cpus if c in allowed]
    except OSError:
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    info["cpu_model"] = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return info


def reference_available() -> bool:
    return os.path.exists(REF_SO)


def _as_u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    a = np.ascontiguousarray(data)
    if a.dtype != np.uint8:
        a = a.view(np.uint8).reshape(-1)
    return a.reshape(-1)


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix_bytes(nbytes: int, seed: int, byte_offset: int = 0) -> np.ndarray:
    """numpy twin of oracle_fill_splitmix / the device fill kernel."""
    if nbytes == 0:
        return np.zeros(0, dtype=np.uint8)
    w0 = byte_offset >> 3
    w1 = (byte_offset + nbytes + 7) >> 3
    with np.errstate(over="ignore"):
        i = np.arange(w0, w1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    s = byte_offset - (w0 << 3)
    return b[s : s + nbytes].copy()
