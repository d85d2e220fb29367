"""The passes' 64-bit lane-offset address path (PassArgs::voff32 = 0: row
offsets that do not fit 32 bits, i.e. shards of >= 1 MiB at 65536 rows) is
forced with rs16.set_diagnostics(DIAG_FORCE_VOFF64) in a subprocess and checked bit for bit
against the oracle: encode (3 passes), general decode at partial loss and the
half-transform decode at 100 % original loss, both rates."""
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
    import oracle_bind as O
    import rs16
    from rs16.util import generate_original
    rs16.set_diagnostics(rs16.DIAG_FORCE_VOFF64)
    out = []
    for rate, k, m in (("high", 4096, 4096), ("low", 1000, 3000), ("default", 2000, 2048)):
        sb = 128
        orig = generate_original(k, sb, 5)
        enc = rs16.RateEncoder(k, m, sb, rate)
        for o in orig:
            enc.add_original_shard(o)
        with enc.encode() as r:
            rec = list(r.recovery_iter())
        want = O.encode(k, m, orig, rate=rate)
        ok_enc = b"".join(rec) == want.tobytes()
        res = []
        for lost in (range(k), range(0, k, 3)):      # 100 % and 1/3 of the originals lost
            lost = set(lost)
            dec = rs16.RateDecoder(k, m, sb, rate)
            for i in range(k):
                if i not in lost:
                    dec.add_original_shard(i, orig[i])
            for j in range(min(m, len(lost))):
                dec.add_recovery_shard(j, rec[j])
            with dec.decode() as d:
                got = dict(d.restored_original_iter())
            res.append(set(got) == lost and all(got[i] == orig[i].tobytes() for i in lost))
        out.append([rate, ok_enc] + res)
    print("RESULT", __import__("json").dumps(out))
""")


def test_forced_64bit_lane_offsets():
    code = SCRIPT.format(pkg=str(ROOT / "reed-solomon-16_amd"), tests=str(ROOT / "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    for rate, *oks in json.loads(line[7:]):
        assert all(oks), (rate, oks)
