"""tools/pmc_summary.py OUTDIR -- fold the rocprofv3 --pmc passes of tools/pmc_inst.sh / tools/pmc_zstd.sh into
per-dispatch averages per kernel."""
import csv, glob, os, sys, collections
out = sys.argv[1]
avg = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    s = collections.defaultdict(float)
    d = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name", "?").split("(")[0], r["Counter_Name"])
        s[k] += float(r["Counter_Value"])
        d[k].add(r.get("Dispatch_Id"))
    for (kern, name), v in s.items():
        avg[kern][name] = v / max(1, len(d[(kern, name)]))
for k, c in avg.items():
    print(k)
    for n in sorted(c):
        print(f"  {n:24s} {c[n]:.6g}")
