"""Per-stream busy time of one training step in a rocprofv3 kernel trace (the last step whose
backward contains the marker kernel): python scripts/trace_streams.py <kernel_trace.csv>
<fwd marker prefix> <bwd marker prefix> <layers>."""
import collections
import csv
import sys

sys.path.insert(0, "scripts")
from prof_summary import short  # noqa: E402

path, fwd_m, bwd_m, L = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
rows = list(csv.DictReader(open(path)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = short(r["Kernel_Name"])[:60]
rows.sort(key=lambda r: r["s"])
bw = [r for r in rows if r["k"].startswith(bwd_m)]
last_b = bw[-L]
fw = [r for r in rows if r["k"].startswith(fwd_m) and r["s"] < last_b["s"]]
a = fw[-L]["s"]
ad = [r for r in rows if "multi_tensor_apply" in r["Kernel_Name"] and r["s"] > bw[-1]["s"]]
b = max(r["e"] for r in ad) if ad else bw[-1]["e"]
step = [r for r in rows if a <= r["s"] < b]
streams = collections.Counter(r["Stream_Id"] for r in step)
print(f"step window {(b - a) / 1e6:.2f} ms")
for sid in streams:
    ks = [r for r in step if r["Stream_Id"] == sid]
    c = collections.defaultdict(float)
    for r in ks:
        c[r["k"][:56]] += (r["e"] - r["s"]) / 1e6
    print(f"== stream {sid}: {len(ks)} kernels, busy {sum(c.values()):.2f} ms")
    for k, v in sorted(c.items(), key=lambda x: -x[1])[:int(__import__("os").environ.get("TOPN","16"))]:
        print(f"   {v:7.2f} {k}")
iv = sorted((r["s"], r["e"]) for r in step)
u, (cs, ce) = 0, iv[0]
for s, e in iv[1:]:
    if s > ce:
        u += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f"union busy {u / 1e6:.2f} ms")
