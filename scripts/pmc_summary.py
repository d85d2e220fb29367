"""Summarize rocprofv3 --pmc counter_collection CSVs: per kernel, mean of each
counter over dispatches (counters summed over XCD/SE instances per dispatch)."""
import csv, sys, glob, collections, re
def short(n):
    m = re.search(r"pass_kernel<(\d+), (\d+)>", n)
    progs = ["GEN_FFT","GEN_IFFT","ENC_FIRST","ENC_MID","ENC_LAST","ENC_SINGLE","DEC_FIRST","DEC_MID","DEC_LAST",
             "DEC_SINGLE","DEC_HALF_LAST","DEC_HALF_SINGLE"]
    # the half-transform decode runs ENC_MID (T8) as DEC_HALF_MID, and with
    # identity multipliers (the bench step) ENC_FIRST / ENC_LAST
    # (T7) as DEC_HALF_FIRST / DEC_HALF_LAST: those rows average both uses;
    # the evaluated half decode runs DEC_FIRST (T7) as DEC_HALF_FIRST
    alias = {("ENC_MID", "8"): "ENC_MID+DEC_HALF_MID", ("ENC_FIRST", "7"): "ENC_FIRST+DEC_HALF_FIRST",
             ("ENC_LAST", "7"): "ENC_LAST+DEC_HALF_LAST", ("DEC_FIRST", "7"): "DEC_HALF_FIRST"}
    if m:
        name = progs[int(m.group(1))]
        return f"{alias.get((name, m.group(2)), name)}/T{m.group(2)}"
    n = n.replace("(anonymous namespace)::", "")
    m = re.search(r"(col2?_kernel)<(\d+), (\d+)>", n)
    if m:  # the column codec (rs16_col.hip): L, mode (ColMode)
        return f"{m.group(1)}<L{m.group(2)},{['ENC', 'DEC_EWORK', 'DEC_EVAL', 'DEC_GEN'][int(m.group(3))]}>"
    return n.split("(")[0].replace("void rs16::","")[:28]
def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(set))
    dur = collections.defaultdict(list)
    for f in sys.argv[1:]:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"]); c = r["Counter_Name"]
            acc[k][c] += float(r["Counter_Value"]); cnt[k][c].add(r["Dispatch_Id"])
            dur[k].append((r["Dispatch_Id"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k in acc:
        d = dict(dur[k]); us = sum(d.values()) / len(d) / 1e3
        vals = {c: acc[k][c] / len(cnt[k][c]) for c in acc[k]}
        print(f"{k:16s} {us:8.1f}us " + " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))


if __name__ == "__main__":
    main()
