"""Condense a tools/round_profile.sh run (gpurun_out/) into committed profile files:

  profiles/<tag>.md            per-kernel rocprofv3 --stats (calls, average duration), the bench's own HIP-event
                               average for the same kernel, and per launch the HBM bytes from the PMC passes
  profiles/pmc_config<C>.json  per bench kernel label: HBM read / write bytes per launch (bench.py reports the
                               dominant kernel's sum as roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE come from separate rocprofv3 --pmc
runs; FETCH_SIZE is doubled (gfx950 tallies 128-B requests of wide streaming reads at 64 B), WRITE_SIZE is taken as
reported; both are KB (x 1024). Usage: [PROF_DIR=<sub>] python tools/summarize_profile.py <tag> [config]"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import alg_bytes  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out", os.environ.get("PROF_DIR", "."))
# kernel-name fragment -> bench label (first match wins)
FAMILIES = [("walk_kernel<", "walk"), ("jt_count_kernel", "j_count"), ("jt_place_kernel", "j_tile"), ("pass0_kernel", "key_pass0"), ("downsweep_wc_kernel<0", "key_pass0"), ("downsweep_kernel<0", "key_pass0"),
            ("downsweep_wc_kernel<1", "key_pass"), ("downsweep_kernel<1", "key_pass"),
            ("downsweep_wc_kernel<2", "j_pass*"), ("downsweep_kernel<2", "j_pass*"),
            ("upsweep_kernel<sm::(anonymous namespace)::KeyColDigits", "key_up"),
            ("upsweep_kernel<sm::(anonymous namespace)::RecDigits", "key_up"),
            ("upsweep_kernel<sm::(anonymous namespace)::PairDigits", "j_up"), ("prep_kernel", "prep"),
            ("scan_chunks_kernel", "scan"), ("digit_base_kernel", "scan"),
            ("stack_kernel", "stack"), ("stack4_kernel", "stack"), ("order_kernel", "order"), ("order2_kernel", "order"), ("stage_base_kernel", "stack_prep"),
            ("carry_in_kernel", "stack_prep"), ("merge_main_kernel", "carry_merge"),
            ("merge_carried_kernel", "carry_merge"),
            ("filter_count", "filter_count"), ("filter_write", "filter_write"), ("filter_block_scan", "filter_scan"),
            ("nfa_kernel", "nfa"), ("sm_nfa_jit", "nfa"), ("lane_events_lds_kernel", "nfa_setup"), ("lane_events16_kernel", "nfa_setup"),
            ("event_index_kernel", "event_index"), ("ts_tile_max_kernel", "event_index"),
            ("tile_prefix_max_kernel", "event_index"), ("advance_points_kernel", "event_index"), ("advance_rank_kernel", "event_index"),
            ("select_records_kernel", "nfa_select"), ("select_mask_kernel", "nfa_select"), ("key_lookup_kernel", "nfa_group"),
            ("rs_upsweep", "nfa_group"), ("rs_downsweep", "nfa_group"),
            ("all_new_csr_kernel", "nfa_group"), ("lane_events_kernel", "nfa_setup"),
            ("lane_index_kernel", "nfa_setup")]


# the closed-form pipelines (configs 3 / 4) use the radix sort only to order the carried partials
CARRY_FAMILIES = [("rs_downsweep", "carry_out"), ("rs_upsweep", "carry_out"), ("carry_rows_kernel", "carry_out"),
                  ("gather_u64_kernel", "carry_out"), ("gather_rows_kernel", "carry_out")]


def family(name, config=4):
    for pat, lab in (CARRY_FAMILIES if config in (3, 4) else []) + FAMILIES:
        if pat in name:
            return lab
    return None


def short(name):
    n = re.sub(r"sm::\(anonymous namespace\)::", "", name).replace("void ", "")
    return n.split("(")[0][:90]


def csv_in(sub, suffix):
    hits = sorted(glob.glob(os.path.join(OUT, sub, "**", f"*{suffix}"), recursive=True))
    return hits[0] if hits else None


def main():
    tag = sys.argv[1]
    config = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    bench = None
    for l in open(os.path.join(OUT, "bench_full.log")):
        if l.startswith("{"):
            bench = json.loads(l)
    n = bench["config"]["events"]
    m = bench["config"]["matches"]
    brk = bench["roofline"]["breakdown"]
    # PMC passes: one step, no warmup -> calls_per_step launches per label
    pmc = {}
    for kind in ("fetch", "write"):
        p = csv_in(f"pmc_{kind}", "counter_collection.csv")
        if not p:
            continue
        for r in csv.DictReader(open(p)):
            nm = short(r["Kernel_Name"])
            key = (nm, r["Counter_Name"])
            pmc[key] = pmc.get(key, 0.0) + float(r["Counter_Value"])
    lines = [f"# rocprofv3 summary — {tag}", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --config {config} --no-cpu --steps 3 "
             f"--warmup 1` (N = {n}, M = {m} matches), MI355X.",
             f"PMC: separate `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs of `bench.py --config {config} "
             "--no-cpu --steps 1 --warmup 0`. FETCH_SIZE is doubled (gfx950 reports half the bytes of wide streaming "
             "reads), WRITE_SIZE as reported (KB x 1024). Bytes per launch.", "",
             "| kernel | label | calls | avg ms (rocprof) | avg ms (bench HIP events) | alg GB/launch | HBM read GB | "
             "HBM write GB | alg GB/s |",
             "|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    stats = csv_in("prof_stats", "kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        fam = family(r["Name"], config)
        if not fam:
            continue
        nm = short(r["Name"])
        avg = float(r["AverageNs"]) / 1e6
        labs = ["j_pass", "j_pass_last"] if fam == "j_pass*" else [fam]
        labs = [l for l in labs if l in brk]
        ev = "/".join(f"{brk[l]['avg_ms']:.3f}" for l in labs)
        alg = alg_bytes(labs[0], n, m, config) / 1e9 if labs else 0.0
        calls1 = max(1, round(sum(brk[l]["calls_per_step"] for l in labs))) if labs else 1
        fetch = pmc.get((nm, "FETCH_SIZE"))
        write = pmc.get((nm, "WRITE_SIZE"))
        rd = 2 * fetch * 1024 / calls1 if fetch is not None else None
        wr = write * 1024 / calls1 if write is not None else None
        for l in labs:
            t = traffic.setdefault(l, {"read_bytes": 0.0, "write_bytes": 0.0, "kernels": []})
            t["read_bytes"] += rd or 0.0
            t["write_bytes"] += wr or 0.0
            t["kernels"].append(nm)
        lines.append(f"| `{nm}` | {fam} | {r['Calls']} | {avg:.3f} | {ev or '-'} | {alg:.2f} | "
                     f"{rd / 1e9 if rd is not None else float('nan'):.2f} | "
                     f"{wr / 1e9 if wr is not None else float('nan'):.2f} | "
                     f"{alg / (avg * 1e-3) if avg else 0:.0f} |")
    # the embedded bench line carries THIS profile's PMC bytes (the bench ran before the PMC passes existed, so its
    # own traffic fields came from the previous summary or were null): one source for the table and the line
    roof = bench["roofline"]
    dom = roof.get("kernel")
    if dom in traffic:
        roof["traffic"] = traffic[dom]["read_bytes"] + traffic[dom]["write_bytes"]
        roof["traffic_source"] = f"this profile's PMC passes ({tag})"
        tot = 0.0
        for lab, b in brk.items():
            if lab in traffic:
                tot += (traffic[lab]["read_bytes"] + traffic[lab]["write_bytes"]) * b["calls_per_step"]
        roof["traffic_step"] = tot
        roof["traffic_step_ratio"] = tot / roof["alg_bytes_per_launch"]
    lines += ["", f"library build `{bench['config'].get('build_id')}`, variant `{bench['config'].get('variant')}`",
              "", "bench line (roofline traffic fields from the PMC passes above):", "", "```", json.dumps(bench),
              "```"]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    open(os.path.join(ROOT, "profiles", f"{tag}.md"), "w").write("\n".join(lines) + "\n")
    variant = bench["config"].get("variant", "literal")
    doc = {"config": config, "events": n, "matches": m, "tag": tag, "build_id": bench["config"].get("build_id"),
           "variant": variant,
           "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 wide-read correction) and --pmc WRITE_SIZE, separate "
                     "passes, 1 step; bytes per launch",
           "labels": {k: {"read_bytes": v["read_bytes"], "write_bytes": v["write_bytes"],
                          "hbm_bytes": v["read_bytes"] + v["write_bytes"], "kernels": v["kernels"]}
                      for k, v in traffic.items()}}
    name = f"pmc_config{config}" + ("" if variant == "literal" else f"_{variant}") + ".json"
    json.dump(doc, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
