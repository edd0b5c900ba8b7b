"""Condense a tools/round_profile.sh run (gpurun_out/) into a committed profile summary:
per-kernel rocprofv3 --stats (calls, average duration) and, per launch, FETCH_SIZE x2 (gfx950 wide-read
correction, MI355X_MICROARCH.md HBM section) and WRITE_SIZE from separate PMC passes, next to the algorithmic
bytes bench.py prices each kernel at. Usage: python tools/summarize_profile.py <tag> [events]"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import alg_bytes  # noqa: E402

OUT = "gpurun_out"
FAMILIES = [("walk_kernel<true", "walk"), ("walk_kernel<false", "walk"),
            ("downsweep_kernel<0", "key_pass0"), ("downsweep_kernel<1", "key_pass"),
            ("downsweep_kernel<2", "j_pass*"), ("upsweep_kernel<sm::(anonymous namespace)::KeyColDigits", "key_up"),
            ("upsweep_kernel<sm::(anonymous namespace)::RecDigits", "key_up"),
            ("upsweep_kernel<sm::(anonymous namespace)::PairDigits", "j_up"), ("c1_mask_kernel", "c1_mask"),
            ("prep_kernel", "prep"), ("scan_chunks_kernel", "scan"), ("digit_base_kernel", "scan")]


def family(name):
    for pat, lab in FAMILIES:
        if pat in name:
            return lab
    return None


def short(name):
    n = re.sub(r"sm::\(anonymous namespace\)::", "", name).replace("void ", "")
    return n.split("(")[0][:90]


def main():
    tag = sys.argv[1]
    bench = None
    for l in open(os.path.join(OUT, "bench_full.log")):
        if l.startswith("{"):
            bench = json.loads(l)
    n = bench["config"]["events"]
    m = bench["config"]["matches"]
    lines = [f"# rocprofv3 summary — {tag}", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --steps 3 --warmup 1` "
             f"(config 4: N = {n}, K = {bench['config']['keys']}, M = {m} matches), MI355X.",
             "PMC: separate `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs of `bench.py --no-cpu --steps 1 "
             "--warmup 0` (one launch per kernel). FETCH_SIZE is doubled (gfx950 reports half the bytes of wide "
             "streaming reads), WRITE_SIZE as reported (KB x 1024).", "",
             "| kernel | calls | avg ms (rocprof) | avg ms (bench HIP events) | alg GB/launch | HBM read GB | "
             "HBM write GB | alg GB/s |",
             "|---|---|---|---|---|---|---|---|"]
    pmc = {}
    for kind in ("fetch", "write"):
        p = os.path.join(OUT, f"pmc_{kind}", "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            fam = family(r["Kernel_Name"])
            if fam:
                key = (short(r["Kernel_Name"]), r["Counter_Name"])
                pmc[key] = pmc.get(key, 0.0) + float(r["Counter_Value"])
    brk = bench["roofline"]["breakdown"]
    for r in csv.DictReader(open(os.path.join(OUT, "prof_stats", "run_kernel_stats.csv"))):
        fam = family(r["Name"])
        if not fam:
            continue
        nm = short(r["Name"])
        avg = float(r["AverageNs"]) / 1e6
        labs = ["j_pass", "j_pass_last"] if fam == "j_pass*" else [fam]
        ev = "/".join(f"{brk[l]['avg_ms']:.3f}" for l in labs if l in brk)
        alg = alg_bytes(labs[0], n, m) / 1e9 if labs[0] in brk or labs[0] in ("scan",) else 0
        fetch = pmc.get((nm, "FETCH_SIZE"))
        write = pmc.get((nm, "WRITE_SIZE"))
        calls1 = {"key_up": 2, "j_up": 2, "scan": 5, "j_pass*": 3}.get(fam, 1)  # launches in the 1-step PMC run
        rd = f"{2 * fetch * 1024 / calls1 / 1e9:.2f}" if fetch else "-"
        wr = f"{write * 1024 / calls1 / 1e9:.2f}" if write else "-"
        lines.append(f"| `{nm}` | {r['Calls']} | {avg:.3f} | {ev} | {alg:.2f} | {rd} | {wr} | "
                     f"{alg / (avg * 1e-3) if avg else 0:.0f} |")
    lines += ["", "bench line:", "", "```", json.dumps(bench), "```"]
    path = os.path.join("profiles", f"{tag}.md")
    open(path, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
