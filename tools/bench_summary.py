"""Print the key fields of the last bench.py JSON line found in a log (GPU-run scripts)."""
import json
import sys

lines = [x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")]
if not lines:
    print("no bench line")
    sys.exit(0)
d = json.loads(lines[-1])
r = d["roofline"]
print("ms_per_step %.3f single %.3f kernel_ms %.3f frac %.4f frac_step %.4f traffic %s" % (
    d["ms_per_step"], d.get("single_query_ms", 0), r["kernel_ms"], r["frac"], r["frac_per_step"], r.get("traffic")))
print(json.dumps({k: [round(v[0], 2), round(v[1], 3)] for k, v in r.get("kernels_per_step", {}).items()}))
