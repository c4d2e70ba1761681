"""tools/traffic_summary.py OUTDIR -- fold the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh into
OUTDIR/traffic.json: per kernel, bytes per dispatch (counters are in KiB, summed over the dispatch's
XCDs/channels by rocprofv3).  Raw counter values: the guide's x2 FETCH correction applies to 16-B-per-lane
streaming reads only; these kernels read with dword loads and dword LDS-DMA (uncalibrated widths)."""
import csv, glob, json, os, sys, collections
out = sys.argv[1]
res = collections.defaultdict(dict)
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    s = collections.defaultdict(float)
    d = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name", "?").split("(")[0], r["Counter_Name"])
        s[k] += float(r["Counter_Value"])
        d[k].add(r.get("Dispatch_Id"))
    for (kern, name), v in s.items():
        if kern.startswith("lzh_"):
            res[kern][name + "_bytes_per_dispatch"] = v / max(1, len(d[(kern, name)])) * 1024.0
# the machine code measured: the code hash of each kernel in the library the passes loaded (bench.py reports a
# profile's traffic only while the loaded library's kernel has the same hash)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lzbench_amd import kernel_hash
lib = os.environ.get("LZH_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lzbench_amd", "liblzbench_hip.so")
hashes = kernel_hash.kernel_hashes(lib)
for k, v in res.items():
    v["kernel_hash"] = hashes.get(k)
    v["traffic_bytes_per_dispatch"] = v.get("FETCH_SIZE_bytes_per_dispatch", 0.0) + v.get("WRITE_SIZE_bytes_per_dispatch", 0.0)
wkey = sys.argv[2] if len(sys.argv) > 2 else "lz4/1/64/text/1073741824"   # bench.py's workload key
json.dump({"workload": "tools/prof_kernels.py " + wkey, "workload_key": wkey, "kernels": res}, open(os.path.join(out, "traffic.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
