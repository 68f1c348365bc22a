"""print per-kernel mean counter values of rocprofv3 csv dirs: python tools/pmc_show.py DIR..."""
import csv, os, sys
for d in sys.argv[1:]:
    vals = {}
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    if "hhuff" not in r["Kernel_Name"] or "edge" in r["Kernel_Name"]:
                        continue
                    k = r["Kernel_Name"].split("(")[0][-60:]
                    vals.setdefault(k, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                    vals[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, cs in vals.items():
        print(d, k)
        for c, per in sorted(cs.items()):
            v = list(per.values())[-2:]
            print("   %-28s %14.0f" % (c, sum(v) / len(v)))
