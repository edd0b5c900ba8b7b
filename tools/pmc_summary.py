"""Sum rocprofv3 PMC CSVs (gpurun_out/pmc_*/run_counter_collection.csv, or the directory given) per kernel family."""
import collections
import csv
import glob
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
pat = (sys.argv[1].rstrip("/") + "/**/*counter_collection.csv") if len(sys.argv) > 1 else \
    "gpurun_out/pmc_*/run_counter_collection.csv"
for f in sorted(glob.glob(pat, recursive=True)):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(walk_kernel<\w+>|onesweep_kernel<\d|prep_kernel|key_hist|u32_hist|hist_scan|filter_\w+_kernel|pass0_kernel|downsweep_wc_kernel<\d|stack4_kernel|order_kernel)",
                      r["Kernel_Name"])
        if m:
            agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
            agg[m.group(1)]["rows:" + r["Counter_Name"]] += 1
for k, d in agg.items():
    print(k)
    waves = d.get("SQ_WAVES", 0)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:16.0f}" + (f"   {v / waves:10.1f}/wave" if waves and c.startswith("SQ_INSTS") else ""))
