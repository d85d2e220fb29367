"""Workloads for the PMC traffic passes beyond the bench step (run under
rocprofv3 --pmc by scripts/gpu_profile.sh): the general decode at the
reference bench's 1 % loss (32768:32768 x 1 KiB: DEC_FIRST / DEC_MID /
tile_last_kernel), and the column codec at 1000:1000 x 1 KiB (configs[1] /
[2]: encode, 100 %-loss decode, and the 1 %-loss general decode).  Each
workload runs `reps` times; its kernels are distinct, so the per-kernel
means of the counters belong to one workload each."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
import numpy as np  # noqa: E402

import rs16  # noqa: E402
from rs16.device import DeviceArray  # noqa: E402
from rs16.util import generate_original  # noqa: E402


def case(eng, k, m, S, lost, reps):
    o = generate_original(k, S, 1)
    d_o, d_r = DeviceArray.from_numpy(eng, o), DeviceArray(eng, m * S)
    rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
    of = np.ones(k, np.uint8)
    of[k - lost:] = 0
    rf = np.zeros(m, np.uint8)
    rf[m - k:] = 1 if lost == k else 0
    if lost < k:
        rf[:lost] = 1
    held = o.copy()
    held[k - lost:] = 0
    x = DeviceArray.from_numpy(eng, held)
    a, b = DeviceArray.from_numpy(eng, of), DeviceArray.from_numpy(eng, rf)
    for _ in range(reps):
        if lost == 0:
            rs16.encode_device(k, m, S, d_o.ptr, d_r.ptr, engine=eng)
        else:
            rs16.decode_device(k, m, S, x.ptr, a.ptr, d_r.ptr, b.ptr, int(of.sum()), int(rf.sum()), engine=eng)
    eng.synchronize()
    if lost:
        assert np.array_equal(x.download(shape=(k, S)), o)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    eng = rs16.Engine(0)
    case(eng, 32768, 32768, 1024, 327, reps)  # 1 % general decode
    case(eng, 1000, 1000, 1024, 0, reps)      # configs[1]
    case(eng, 1000, 1000, 1024, 1000, reps)   # configs[2]
    case(eng, 1000, 1000, 1024, 10, reps)     # 1 % general decode, column form
    print("PMC_EXTRA_DONE")


if __name__ == "__main__":
    main()
