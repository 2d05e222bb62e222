"""Print the bench line's key numbers (headline, roofline, the extras' stage figures) from a bench.json file."""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print("headline", d["value"], "kernel_ms", r.get("kernel_ms"), "frac", r.get("frac"), "traffic", r.get("traffic"),
      "uniform", (r.get("uniform") or {}).get("kernel_ms"))
e = d.get("extras") or {}
for k in ("cfg3_esim_forward", "cfg2_dssm_forward", "cfg2_dssm_train_step", "feature_pipe"):
    v = e.get(k)
    print(k, json.dumps(v)[:700] if v else v)
c = d.get("cfg4_sharded") or {}
print("cfg4", c.get("ms_per_step"), json.dumps(c.get("simulated_p8"))[:700])
