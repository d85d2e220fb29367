"""Host-link rate against the NUMA node the process runs on (diagnostic).
bench.py's host extras ran slower than the same calls in a small fresh
process (one-shot 39 vs 47 GiB/s, pipelined 35-48 vs 74-77): this prints
the NUMA layout, the GPU's node, and the one-shot / pipelined host rates
with the process bound to each node's CPUs (allowed ones only) before its
pinned buffers are allocated and touched."""
import ctypes as C
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += range(int(a), int(b) + 1)
        elif part:
            out.append(int(part))
    return out


def main():
    nodes = {}
    for d in sorted(Path("/sys/devices/system/node").glob("node[0-9]*")):
        nodes[int(d.name[4:])] = cpulist((d / "cpulist").read_text())
    allowed = sorted(os.sched_getaffinity(0))
    print("nodes:", {n: (len(c), c[0], c[-1]) for n, c in nodes.items()}, "allowed:", len(allowed), allowed[:4], "...")
    from rs16._lib import hip_runtime  # noqa: E402
    hip = hip_runtime()
    bus = C.create_string_buffer(64)
    hip.hipDeviceGetPCIBusId(bus, 64, 0)
    bdf = bus.value.decode().lower()
    p = Path("/sys/bus/pci/devices") / bdf / "numa_node"
    print("gpu", bdf, "numa_node", p.read_text().strip() if p.exists() else "?")
    which = int(sys.argv[1])
    cpus = [c for c in nodes.get(which, []) if c in allowed]
    if not cpus:
        print("node", which, "has no allowed cpus")
        return
    os.sched_setaffinity(0, cpus)
    import numpy as np
    import rs16
    from rs16.device import PinnedArray
    k = m = 32768
    S = 1024
    nb = 8
    GIB = 2.0 ** 30
    eng = rs16.Engine(0)
    ho, hr = PinnedArray(eng, nb * k * S), PinnedArray(eng, nb * m * S)
    ho.array[:] = 7
    hr.array[:] = 0
    for rep in range(4):
        t = time.perf_counter()
        rs16.encode_host(k, m, S, ho.ptr, hr.ptr, engine=eng)
        t1 = time.perf_counter() - t
        t = time.perf_counter()
        rs16.encode_host_batch(k, m, S, nb, ho.ptr, k * S, hr.ptr, m * S, engine=eng)
        t2 = time.perf_counter() - t
    print(f"node {which} ({len(cpus)} cpus): one-shot encode {(k + m) * S / t1 / GIB:.1f} GiB/s, "
          f"pipelined x{nb} {nb * (k + m) * S / t2 / GIB:.1f} GiB/s", flush=True)


if __name__ == "__main__":
    main()
