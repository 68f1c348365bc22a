#!/usr/bin/env python3
"""Per-kernel duration summary of rocprofv3 --kernel-trace databases (the default .db output).

    python tools/prof_db.py DIR [substring]   # name, calls, mean/min us for kernels matching substring
"""
import glob
import os
import sqlite3
import sys


def main(d, pat="hhuff"):
    for f in sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)):
        c = sqlite3.connect(f)
        print(f)
        q = ("select name, count(*), avg(end - start) / 1000.0, min(end - start) / 1000.0 from kernels "
             "where name like ? group by name order by 3 desc")
        for name, n, avg, mn in c.execute(q, ("%" + pat + "%",)):
            print("  %-70s %5d  mean %9.2f us  min %9.2f us" % (name[:70], n, avg, mn))


if __name__ == "__main__":
    main(*sys.argv[1:])
