"""Print value and per-kernel launch times of bench lines (A/B tables): ab_summary2.py files..."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("rooflines", {})
    print(f"{f.split('/')[-1]:22s} {d['value']:8.1f}  " + "  ".join(
        f"{k.split()[0][6:]} {v['avg_launch_ms']:.4f}ms {v['achieved_tflops']:.0f}TF" for k, v in r.items()))
