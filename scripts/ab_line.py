"""One-line summary of a bench.py JSON line (last line of a log) for A/B runs: usage ab_line.py LOG TAG"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
out = {"tag": sys.argv[2], "value": round(d["value"] / 1e6, 2), "ms": round(d["ms_per_step"], 3)}
f = d.get("forward") or {}
for k in ("ms", "k4_fwd_ms_per_layer", "hbm_frac_k4", "hbm_frac_model"):
    if f.get(k) is not None:
        out["fwd_" + k] = round(f[k], 4)
r = d.get("roofline") or {}
for k in ("kernel_ms", "frac", "frac_survey", "fwd_kernel_ms"):
    if r.get(k) is not None:
        out["roof_" + k] = round(r[k], 4)
x = d.get("egnn_f32_exact")
if x:
    out["exact"] = round(x["value"] / 1e6, 2)
for w in ("mace", "gvp", "tfn"):
    if isinstance(d.get(w), dict):
        out[w] = round(d[w]["value"] / 1e6, 4)
print(json.dumps(out))
