"""print the headline line of a bench run in brief: python tools/bench_brief.py <bench line json>"""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(f"value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.5f}  roof {r.get('bound')} "
      f"frac {r.get('frac'):.4f} launch {r.get('avg_launch_us'):.3f} us  cpu {d['cpu_baseline'] and d['cpu_baseline']['value']}")
for k, v in d.get("lines", {}).items():
    print(" ", k, json.dumps(v)[:300])
print("errors", d.get("secondary_errors"), "run_s", d.get("run_s"))
