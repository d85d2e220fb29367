"""profiles/pmc_traffic.json from a scripts/gpu_profile.sh run: HBM bytes
per launch of every kernel from its FETCH_SIZE / WRITE_SIZE passes
(MI355X_MICROARCH.md's rocprofv3 recipe: separate --pmc passes; on gfx950
FETCH_SIZE counts half of the streamed read bytes, so bytes = (2 FETCH_SIZE +
WRITE_SIZE) KiB), next to the algorithmic bytes of the launch.
usage: pmc_traffic.py <prof dir> <tag>"""
import collections
import csv
import json
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import short  # noqa: E402

MB1K = 1024
# pmc passes of gpu_profile.sh: 1 / 2 = the bench step (32768:32768 x 1 KiB,
# encode + 100 %-loss decode), 5 / 6 = scripts/pmc_extra.py
WORK = {
    "bench": "32768:32768:1024",
    "extra": {"DEC_FIRST/T8": "32768:32768:1024 1% loss", "DEC_MID/T8": "32768:32768:1024 1% loss",
              "rs16::tile_last_kernel": "32768:32768:1024 1% loss",
              "rs16::mid_direct_kernel": "32768:32768:1024 1% loss",
              "col2_kernel<L10,ENC>": "1000:1000:1024 encode",
              "col2_kernel<L10,DEC_EVAL>": "1000:1000:1024 100% loss",
              "col2_kernel<L11,DEC_GEN>": "1000:1000:1024 1% loss"},
}
# the bench step's kernels under the program names bench.py's profile uses
# (the half decode runs DEC_FIRST at T = 7 and ENC_MID at T = 8)
BENCH_NAMES = {"ENC_FIRST+DEC_HALF_FIRST/T7": ["ENC_FIRST", "DEC_HALF_FIRST"],
               "ENC_MID+DEC_HALF_MID/T8": ["ENC_MID", "DEC_HALF_MID"],
               "ENC_LAST+DEC_HALF_LAST/T7": ["ENC_LAST", "DEC_HALF_LAST"], "DEC_HALF_FIRST/T7": ["DEC_HALF_FIRST"],
               "DEC_HALF_LAST/T7": ["DEC_HALF_LAST"], "rs16::eval_fused_kernel": ["EVAL_POLY"]}


def mean_counter(path, counter):
    acc, ids = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        acc[k] += float(r["Counter_Value"])
        ids[k].add(r["Dispatch_Id"])
    return {k: acc[k] / len(ids[k]) for k in acc}


def main():
    d, tag = Path(sys.argv[1]), sys.argv[2]
    out = {}
    for fp, wp, extra in ((1, 2, False), (5, 6, True)):
        f = mean_counter(d / f"pmc{fp}" / "run_counter_collection.csv", "FETCH_SIZE")
        w = mean_counter(d / f"pmc{wp}" / "run_counter_collection.csv", "WRITE_SIZE")
        for k in f:
            if "rocclr" in k or not k:
                continue
            if extra and k not in WORK["extra"]:
                continue  # (the extra run's bench-shaped passes are the bench's)
            wl = WORK["extra"][k] if extra else WORK["bench"]
            # bench.py looks the dominant kernel up as "<program>:<k>:<m>:<S>"
            names = BENCH_NAMES.get(k, [k]) if not extra else [k]
            rec = {"fetch_size_kib": round(f[k], 1), "write_size_kib": round(w.get(k, 0.0), 1),
                   "hbm_bytes_per_launch": int((2 * f[k] + w.get(k, 0.0)) * MB1K),
                   "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = 1/2 of streamed read bytes)",
                   "workload": wl, "collected": tag}
            for nm in names:
                out[f"{nm}:{wl}"] = dict(rec, kernel=k)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
