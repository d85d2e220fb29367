"""The multi-rank JSON line of bench.py, on CPU.

`bench.py --gpus 2 --cpu-stub` goes through the driver's launch form
(torch.distributed.run, one process per rank, gloo control plane) and the
same barrier / max-over-ranks / per-rank helpers as the GPU run, around a
numpy stand-in step.  The line must name every rank -- host, local rank,
device, its own time per step -- and the configs[4] per-rank codec times, so
that a straggler in the first 8-GPU run can be identified."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def run_stub(gpus):
    env = dict(os.environ)
    for v in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    res = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), "--cpu-stub", "--steps", "6",
                          "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env, cwd=str(ROOT))
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, res.stdout  # one JSON line, from rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_line_names_every_rank(gpus):
    out = run_stub(gpus)
    assert out["stub"] is True and out["n_gpus"] == gpus
    ranks = out["ranks"]
    assert [r["rank"] for r in ranks] == list(range(gpus))
    for r in ranks:
        for key in ("hostname", "local_rank", "device", "pid", "ms_per_step", "gib_s"):
            assert key in r, key
        assert r["ms_per_step"] > 0 and r["gib_s"] > 0
    assert sorted(r["local_rank"] for r in ranks) == list(range(gpus))
    # the metric's time is the slowest rank's
    assert out["ms_per_step"] == pytest.approx(max(r["ms_per_step"] for r in ranks), rel=1e-3)
    codec = out["extra"]["configs4_rccl"]["codec_ms_per_rank"]
    assert len(codec) == gpus and all(t > 0 for t in codec)
