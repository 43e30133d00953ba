"""Print one line per bench JSON of an A/B run: value, ms/step, kernel launch times, lite stats."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:          # noqa: BLE001
        print(f, "unreadable", e)
        continue
    ro = d.get("rooflines", {})
    ks = " ".join(f"{k.split()[0]}={v['avg_launch_ms']:.3f}x{v['launches']}" for k, v in ro.items())
    lp = d.get("lite_pass") or {}
    print(f"{f.split('/')[-1][:-5]:28s} {d['value']:7.1f} obj/s {d['ms_per_step']:7.2f} ms  {ks}  "
          f"refine {lp.get('refine_fraction')} audit {lp.get('audit_fraction')} viol {lp.get('audit_violations')} "
          f"redo {lp.get('redo_objects')} err {lp.get('max_observed_lite_error')}")
