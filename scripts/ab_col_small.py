"""Same-box A/B of two builds of the column codec: runs this script's `arm`
mode in a child process per library (RS16_LIB), alternating, and prints the
host-timed call rates of the radix-2 column forms (probe_col2.run / run_1pct).

usage: python scripts/ab_col_small.py LIB_A LIB_B [ROUNDS]"""
import json
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent


def arm():
    sys.path.insert(0, str(HERE))
    import probe_col2 as pc
    import rs16
    eng = rs16.Engine(0)
    out = {}
    for k, m in ((1000, 1000), (512, 512), (100, 100)):
        r = pc.run(eng, k, m, 1024, 0)
        out[f"{k}:{m}"] = {"exact": r["exact"], "enc": r["encode"]["host_us"], "dec": r["decode"]["host_us"],
                           "enc_k": r["encode"]["kernel_us"], "dec_k": r["decode"]["kernel_us"]}
    for k, m in ((1000, 1000), (100, 1000)):
        out[f"{k}:{m} 1%"] = pc.run_1pct(eng, k, m, 1024, 0)
    if os.environ.get("AB_WIDE"):
        # multi-chunk encodes (colm_kernel / chunked col2_kernel) and the
        # 1 %-loss decode at 32768:32768 (tile_last_kernel)
        for k, m in ((100, 1000), (1000, 100), (3000, 1000)):
            r = pc.run(eng, k, m, 1024, 0)
            out[f"{k}:{m}"] = {"exact": r["exact"], "enc": r["encode"]["host_us"]}
        out["32768:32768 1%"] = pc.run_1pct(eng, 32768, 32768, 1024, 0)
    print(json.dumps(out), flush=True)


def main():
    if sys.argv[1] == "arm":
        arm()
        return
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    for i in range(rounds):
        for lib in libs:
            env = dict(os.environ, RS16_LIB=lib)
            res = subprocess.run([sys.executable, __file__, "arm"], env=env, capture_output=True, text=True, timeout=240)
            if res.returncode != 0:
                print(res.stderr[-2000:], flush=True)
                sys.exit(res.returncode)
            print(f"round {i} {Path(lib).name} {res.stdout.strip()}", flush=True)


if __name__ == "__main__":
    main()
