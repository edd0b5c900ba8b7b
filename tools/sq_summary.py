"""Condense a tools/sq_stack.sh run (gpurun_out/sq_<i>/run_counter_collection.csv, one kernel, one step) into a
committed table: profiles/<tag>.md with the raw SQ counters and the ratios DESIGN.md quotes (share of wave-cycles
waiting, LDS bank-conflict share of LDS cycles, wave-instructions per event).
Usage: python tools/sq_summary.py <tag> <events per launch> [note]"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, events = sys.argv[1], float(sys.argv[2])
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    agg = collections.defaultdict(float)
    kernels = set()
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "sq_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            kernels.add(r["Kernel_Name"])
    if not agg:
        sys.exit("no gpurun_out/sq_*/run_counter_collection.csv")

    def ratio(a, b):
        return agg[a] / agg[b] if agg.get(b) else float("nan")

    lines = [f"# SQ counters — {tag}", "",
             "Command: `tools/sq_stack.sh` (two `rocprofv3 --pmc` passes of 8 SQ counters each, "
             "`--kernel-include-regex`, one bench step; no trace domains). " + note, "",
             "Kernel(s): " + ", ".join(f"`{k}`" for k in sorted(kernels)), "",
             "| counter | value | per event |", "|---|---|---|"]
    for c, v in sorted(agg.items()):
        lines.append(f"| {c} | {v:.0f} | {v / events:.3f} |")
    lines += ["", "| ratio | value |", "|---|---|",
              f"| wave-cycles waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES) | {ratio('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'):.3f} |",
              f"| wave-cycles issuing (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES) | "
              f"{ratio('SQ_ACTIVE_INST_ANY', 'SQ_WAVE_CYCLES'):.3f} |",
              f"| LDS bank conflicts (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) | "
              f"{ratio('SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE'):.3f} |",
              f"| VALU wave-instructions per event | {agg['SQ_INSTS_VALU'] / events:.2f} |",
              f"| SALU wave-instructions per event | {agg['SQ_INSTS_SALU'] / events:.2f} |",
              f"| LDS wave-instructions per event | {agg['SQ_INSTS_LDS'] / events:.2f} |",
              f"| VMEM wave-instructions per event | {agg['SQ_INSTS_VMEM'] / events:.3f} |", ""]
    out = os.path.join(ROOT, "profiles", tag + ".md")
    open(out, "w").write("\n".join(lines))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
