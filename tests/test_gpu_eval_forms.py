"""Both forms of the decode's eval_poly on block-aligned geometries: the
one-kernel form (eval_fused_kernel, the default there) runs in this process
through every aligned decode of the suite; here the two-kernel form
(fwht_lo_flags_kernel + fwht_hi_mulw_kernel, rs16.DIAG_EVAL_TWO_KERNEL) runs the same
decodes in a subprocess.  Both must restore every lost original bit-exactly
(100 % loss = half-transform decode; tail / scattered losses = general decode
with lost-range pruning)."""
import json
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]

SCRIPT = textwrap.dedent("""
    import sys
    sys.path[:0] = [{pkg!r}, {tests!r}]
    import numpy as np
    import rs16
    from rs16.device import DeviceArray
    from rs16.util import generate_original
    rs16.set_diagnostics({flags})
    eng = rs16.default_engine()
    out = []
    for k, m, sb in ((32768, 32768, 64), (4096, 4096, 128), (61440, 4096, 64)):
        orig = generate_original(k, sb, 7)
        d_o, d_r = DeviceArray.from_numpy(eng, orig), DeviceArray(eng, m * sb)
        rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
        for pattern in ("all", "tail", "scatter"):
            om = np.ones(k, bool)
            if pattern == "all":
                om[:min(k, m)] = False
            elif pattern == "tail":
                om[k - max(1, min(k, m) // 100):] = False
            else:
                om[::max(2, k // (m // 2))] = False
            lost = int((~om).sum())
            rm = np.zeros(m, bool)
            rm[:lost] = True
            holes = orig.copy()
            holes[~om] = 0x5A
            d_x = DeviceArray.from_numpy(eng, holes)
            d_of = DeviceArray.from_numpy(eng, om.astype(np.uint8))
            d_rf = DeviceArray.from_numpy(eng, rm.astype(np.uint8))
            rs16.decode_device(k, m, sb, d_x.ptr, d_of.ptr, d_r.ptr, d_rf.ptr, int(om.sum()), lost, engine=eng)
            out.append([k, m, pattern, bool(np.array_equal(d_x.download(shape=(k, sb)), orig))])
    print("RESULT", __import__("json").dumps(out))
""")


@pytest.mark.parametrize("fused", ["0", "1"])
def test_eval_forms_restore(fused):
    flags = 0 if fused == "1" else 2  # rs16.DIAG_EVAL_TWO_KERNEL
    code = SCRIPT.format(pkg=str(ROOT / "reed-solomon-16_amd"), tests=str(ROOT / "tests"), flags=flags)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    for k, m, pattern, ok in json.loads(line[7:]):
        assert ok, (k, m, pattern)


def test_unaligned_flag_arrays():
    # received-flag arrays at odd device addresses: eval_fused_ok refuses the
    # one-kernel form (16-byte loads) and the two-kernel form runs instead
    import numpy as np
    import rs16
    from rs16.device import DeviceArray
    from rs16.util import generate_original

    eng = rs16.default_engine()
    k = m = 4096
    sb = 128
    orig = generate_original(k, sb, 3)
    d_o, d_r = DeviceArray.from_numpy(eng, orig), DeviceArray(eng, m * sb)
    rs16.encode_device(k, m, sb, d_o.ptr, d_r.ptr, engine=eng)
    for lost_n in (k, 40):
        om = np.ones(k, bool)
        om[k - lost_n:] = False
        rm = np.zeros(m, bool)
        rm[:lost_n] = True
        fo = np.concatenate([[7], om.astype(np.uint8)]).astype(np.uint8)  # flags start at byte 1
        fr = np.concatenate([[7], rm.astype(np.uint8)]).astype(np.uint8)
        d_fo, d_fr = DeviceArray.from_numpy(eng, fo), DeviceArray.from_numpy(eng, fr)
        holes = orig.copy()
        holes[~om] = 0
        d_x = DeviceArray.from_numpy(eng, holes)
        rs16.decode_device(k, m, sb, d_x.ptr, d_fo.ptr + 1, d_r.ptr, d_fr.ptr + 1, int(om.sum()), lost_n, engine=eng)
        assert np.array_equal(d_x.download(shape=(k, sb)), orig), lost_n
