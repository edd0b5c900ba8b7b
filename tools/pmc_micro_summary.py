"""Per-dispatch average of rocprofv3 PMC counters (gpurun_out/pmcm_*/) per micro-benchmark kernel."""
import collections
import csv
import glob
import re
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "pmcm_"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"gpurun_out/{pat}*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
        name = re.sub(r"^void ", "", name)
        agg[name][r["Counter_Name"]].append((r.get("Dispatch_Id"), float(r["Counter_Value"])))
for k, d in agg.items():
    if "fill" in k:
        continue
    print(k)
    for c, vals in sorted(d.items()):
        per = collections.defaultdict(float)
        for disp, v in vals:
            per[disp] += v
        xs = list(per.values())
        print(f"   {c:28s} {sum(xs) / len(xs):16.0f}  (x{len(xs)})")
