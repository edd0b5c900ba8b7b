"""SQ / SQC counter table of one kernel from tools/sq_nfa.sh's passes (gpurun_out/<prefix>_<i>/): totals, per wave and
the derived shares the round notes quote (waiting, issuing, VALU / SALU / VMEM / LDS instructions per wave, icache).

usage: python3 tools/sq_summary.py <prefix> <title> [command]   (markdown on stdout)"""
import collections
import csv
import glob
import os
import sys


def load(prefix):
    agg = collections.defaultdict(float)
    meta = {}
    for f in sorted(glob.glob(os.path.join("gpurun_out", prefix + "_*", "**", "*counter_collection.csv"),
                              recursive=True)):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            meta.setdefault("kernel", r["Kernel_Name"])
            for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size",
                      "Scratch_Size"):
                meta.setdefault(k, r[k])
    return agg, meta


def main():
    prefix, title = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else ""
    agg, meta = load(prefix)
    if not agg:
        sys.exit(f"no counter CSVs under gpurun_out/{prefix}_*")
    w = agg.get("SQ_WAVES") or 1.0
    cyc = agg.get("SQ_WAVE_CYCLES") or 1.0
    print(f"# SQ counters — {title}\n")
    if cmd:
        print(f"Passes: `{cmd}` (one `rocprofv3 --pmc` pass per counter group, one step each).\n")
    print("Kernel `{}`: grid {}, workgroup {}, {} VGPRs (+{} AGPRs), {} SGPRs, LDS {} B, scratch {} B.\n".format(
        meta.get("kernel", "?"), meta.get("Grid_Size"), meta.get("Workgroup_Size"), meta.get("VGPR_Count"),
        meta.get("Accum_VGPR_Count"), meta.get("SGPR_Count"), meta.get("LDS_Block_Size"), meta.get("Scratch_Size")))
    print("| counter | total | per wave |\n|---|---|---|")
    for k, v in sorted(agg.items()):
        print(f"| `{k}` | {v:.4g} | {v / w:.4g} |")
    print("\n| derived | value |\n|---|---|")
    rows = [("waiting share of wave-cycles (SQ_WAIT_ANY / SQ_WAVE_CYCLES)", agg.get("SQ_WAIT_ANY", 0) / cyc),
            ("issuing share of wave-cycles (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES)", agg.get("SQ_ACTIVE_INST_ANY", 0) / cyc)]
    if "SQ_INSTS_VMEM" in agg:
        rows.append(("VALU instructions per VMEM instruction", agg.get("SQ_INSTS_VALU", 0) / max(agg["SQ_INSTS_VMEM"], 1)))
    if "SQ_WAIT_INST_LDS" in agg:
        rows.append(("LDS waits share of waiting", agg["SQ_WAIT_INST_LDS"] / max(agg.get("SQ_WAIT_ANY", 1), 1)))
    if "SQC_ICACHE_REQ" in agg:
        rows.append(("instruction-cache miss rate", agg.get("SQC_ICACHE_MISSES", 0) / max(agg["SQC_ICACHE_REQ"], 1)))
    for name, v in rows:
        print(f"| {name} | {v:.3f} |")


if __name__ == "__main__":
    main()
