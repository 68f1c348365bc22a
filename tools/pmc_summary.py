#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory: kernel-trace stats plus mean PMC counters per kernel,
with the derived per-launch HBM traffic (gfx950: FETCH_SIZE reports half of 16-B streaming reads, so it
is doubled; FETCH_SIZE / WRITE_SIZE are in KiB) -- MI355X_MICROARCH.md's HBM/rocprofv3 recipe.

    python tools/pmc_summary.py gpurun_out/prof_<tag> [LAST] > profiles/<name>.txt

Only the LAST dispatches of each kernel are averaged (default 6 = bench.py --warmup 1 --steps 5): the
earlier ones are the bench's set-up launches (packing, checks) of other sizes.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, last=6):
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    print("# rocprofv3 summary of %s" % d)
    traces = glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True)
    if traces:
        durs = defaultdict(list)
        with open(traces[0]) as f:
            for row in csv.DictReader(f):
                if "hhuff" in row["Kernel_Name"]:
                    durs[row["Kernel_Name"]].append((int(row["Dispatch_Id"]),
                                                     int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
        print("## kernel trace: mean duration of the last %d dispatches (the bench steps)" % last)
        for k, v in sorted(durs.items()):
            v.sort()
            t = [x for _, x in v[-last:]]
            print("  %-70s last=%d mean_ns=%.0f" % (k[:70], len(t), sum(t) / len(t)))
    if stats:
        print("## kernel trace (--kernel-trace --stats, all dispatches)")
        with open(stats[0]) as f:
            for row in csv.DictReader(f):
                if "hhuff" in row["Name"]:
                    print("  %-70s calls=%-4s avg_ns=%-12s min_ns=%-10s max_ns=%s" % (
                        row["Name"][:70], row["Calls"], row["AverageNs"], row["MinNs"], row["MaxNs"]))
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", row.get("Kernel-Name", ""))
                if "hhuff" not in k:
                    continue
                disp = row.get("Dispatch_Id", row.get("Correlation_Id", ""))
                vals[k][row["Counter_Name"]].append((disp, float(row["Counter_Value"])))
    print("## PMC (mean per dispatch; counters summed over dimensions per dispatch)")
    for k in sorted(vals):
        print("  " + k)
        for c in sorted(vals[k]):
            per = defaultdict(float)
            for disp, v in vals[k][c]:
                per[int(disp)] += v
            keep = sorted(per)[-last:]
            m = sum(per[x] for x in keep) / max(len(keep), 1)
            print("     %-24s dispatches=%-4d mean(last %d)=%.6g" % (c, len(per), len(keep), m))
        fetch = vals[k].get("FETCH_SIZE")
        write = vals[k].get("WRITE_SIZE")
        if fetch and write:
            pf, pw = defaultdict(float), defaultdict(float)
            for disp, v in fetch:
                pf[int(disp)] += v
            for disp, v in write:
                pw[int(disp)] += v
            kf, kw = sorted(pf)[-last:], sorted(pw)[-last:]
            mf = sum(pf[x] for x in kf) / len(kf)
            mw = sum(pw[x] for x in kw) / len(kw)
            print("     => HBM traffic per launch = 2 x FETCH + WRITE = %.4g GB" % ((2 * mf + mw) * 1024 / 1e9))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 6)
