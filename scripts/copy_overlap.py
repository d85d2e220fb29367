"""Overlap of host->device and device->host copies in a rocprofv3
--memory-copy-trace CSV (run_memory_copy_trace.csv): per stream the copy
intervals, the time both directions were in flight, and each direction's
busy time and rate.  Usage: copy_overlap.py TRACE.csv [min_bytes_ignored]"""
import csv
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if b > a:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


rows = list(csv.DictReader(open(sys.argv[1])))
h2d = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if r["Direction"].endswith("HOST_TO_DEVICE")]
d2h = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if r["Direction"].endswith("DEVICE_TO_HOST")]
streams = sorted({r["Stream_Id"] for r in rows})
uh, ud = union(h2d), union(d2h)
bh, bd = sum(b - a for a, b in uh), sum(b - a for a, b in ud)
both = inter(uh, ud)
span = max(b for _, b in h2d + d2h) - min(a for a, _ in h2d + d2h)
print(f"copies: {len(h2d)} H2D, {len(d2h)} D2H on streams {streams}; span {span / 1e6:.2f} ms")
print(f"busy: H2D {bh / 1e6:.2f} ms, D2H {bd / 1e6:.2f} ms, both in flight {both / 1e6:.2f} ms "
      f"({both / max(1, min(bh, bd)):.0%} of the shorter direction)")
