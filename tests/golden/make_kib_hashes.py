"""Generate tests/golden/kib_hashes.json with the CPU oracle.

The reference holds no golden vector for 1024-byte shards at the BASELINE
configurations (its large vectors use 64-byte shards).  Once the oracle
reproduces every reference vector (tests/test_oracle_golden.py), it produces
these: SHA-256 of the concatenated recovery shards of
reed_solomon_16::encode(k, m, generate_shards(k, 1024, seed 0)) -- the
benchmark input of benches/benchmarks.rs:21-28 -- for the BASELINE configs.
"""
import hashlib
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parents[1] / "reed-solomon-16_amd"))

import oracle_bind as O  # noqa: E402
from rs16.util import generate_original  # noqa: E402

CONFIGS = [(100, 100), (1000, 1000), (32768, 32768)]


def main():
    cases = []
    for k, m in CONFIGS:
        rec = O.encode(k, m, generate_original(k, 1024, 0))
        cases.append({"k": k, "m": m, "shard_bytes": 1024, "seed": 0,
                      "recovery_sha256": hashlib.sha256(rec.tobytes()).hexdigest()})
        print(cases[-1])
    (HERE / "kib_hashes.json").write_text(json.dumps({"generator": "oracle NoSimd (tests/golden/make_kib_hashes.py)",
                                                      "cases": cases}, indent=1))


if __name__ == "__main__":
    main()
