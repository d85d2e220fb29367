"""Debug: general decode with a given loss list, split vs LDS derivative."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "reed-solomon-16_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np
import rs16
from rs16.util import generate_original
from test_gpu_device_path import dev_encode, dev_decode

eng = rs16.Engine(0)
cases = [(4096, 4096, 64, [64 * kk - 4096]) for kk in (64, 71, 120, 127, 119, 112, 95)]
cases += [(2000, 2000, 64, [64 * kk - 2048]) for kk in (32, 35, 59, 60, 63)]
for k, m, sb, lost in cases:
    original = generate_original(k, sb, 13)
    recovery = dev_encode(eng, original, m)
    om = np.ones(k, bool); om[lost] = False
    rm = np.zeros(m, bool); rm[:len(lost)] = True
    for fd in (0, rs16.DIAG_FD_LDS):
        old = rs16.set_diagnostics(fd)
        out = dev_decode(eng, original, recovery, om, rm)
        rs16.set_diagnostics(old)
        bad = np.flatnonzero((out != original).any(axis=1))
        print(k, m, sb, lost[:3], len(lost), "fd_lds" if fd else "split", "bad rows:", bad[:10], len(bad),
              "bad cols:", np.flatnonzero((out != original).any(axis=0))[:8], flush=True)
