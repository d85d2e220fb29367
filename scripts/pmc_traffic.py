"""rocprofv3 --pmc CSVs (a FETCH_SIZE pass and a WRITE_SIZE pass of the same
bench command) -> profiles/pmc_traffic.json: HBM-side bytes per launch of each
pass program, keyed "<PROG>:<k>:<m>:<S>" as bench.py reads it.

Units and gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md §HBM,
cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE
reports 1/2 of the bytes of a coalesced streaming read on gfx950, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Counters are summed over
XCD/SE instances per dispatch, then averaged over dispatches.

usage: pmc_traffic.py K M S OUT.json FETCH_DIR WRITE_DIR
"""
import collections
import csv
import glob
import json
import re
import sys

PROGS = ["GEN_FFT", "GEN_IFFT", "ENC_FIRST", "ENC_MID", "ENC_LAST", "ENC_SINGLE", "DEC_FIRST", "DEC_MID", "DEC_LAST",
         "DEC_SINGLE", "DEC_HALF_LAST", "DEC_HALF_SINGLE"]
# The half-transform decode of the 32768:32768 bench reuses two kernels under
# its own profiling names: pass_kernel<ENC_MID, 8> (same bytes as the
# encode's) and pass_kernel<DEC_FIRST, 7> (the full decode's DEC_FIRST is T = 8).
ALIASES = {(3, 8): ["ENC_MID", "DEC_HALF_MID"], (6, 7): ["DEC_HALF_FIRST"]}


def per_launch(d, counter):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"pass_kernel<(\d+), (\d+)>", r["Kernel_Name"])
            if not m:
                continue
            key = (int(m.group(1)), int(m.group(2)))
            for name in ALIASES.get(key, [PROGS[key[0]]]):
                acc[name][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {p: sum(v.values()) / len(v) for p, v in acc.items() if v}


def main():
    k, m, s, out, fdir, wdir = sys.argv[1:7]
    fetch, write = per_launch(fdir, "FETCH_SIZE"), per_launch(wdir, "WRITE_SIZE")
    res = {}
    try:
        res = json.load(open(out))
    except (OSError, ValueError):
        pass
    for p in sorted(set(fetch) & set(write)):
        res[f"{p}:{k}:{m}:{s}"] = {
            "fetch_size_kib": round(fetch[p], 1), "write_size_kib": round(write[p], 1),
            "hbm_bytes_per_launch": round((2 * fetch[p] + write[p]) * 1024),
            "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = 1/2 of streamed read bytes)"}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for key, v in res.items():
        print(key, v["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
