"""Pretty-print the per-kernel breakdown of a bench.py JSON line read from stdin / a file."""
import json
import sys

for l in (open(sys.argv[1]) if len(sys.argv) > 1 else sys.stdin):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"value {d['value']:.4g} ev/s  {d['ms_per_step']:.2f} ms/step  step_frac {d['config']['step_hbm_fraction']:.3f}")
        r = d["roofline"] or {}
        for k, v in r.get("breakdown", {}).items():
            print(f"  {k:12s} {v['avg_ms']:8.3f} ms x{v['calls_per_step']:.0f} {v['gbps']:8.0f} GB/s")
    elif l.strip():
        print(l.rstrip())
