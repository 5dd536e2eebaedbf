"""Timeline of one training step from a rocprofv3 --kernel-trace CSV (dev tool): kernels of the
last complete step between two markers, per-queue gaps, and GPU-idle time (union of busy
intervals over all queues).  usage: trace_step.py trace.csv [marker_substring] [--list]"""
import csv
import re
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "gather_rows_kernel"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
step = rows[a:b]


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("at::native::", "")
    n = n.replace("gmp::", "")
    n = re.sub(r"\(.*", "", n)
    if n.startswith("Cijk"):
        n = "GEMM " + n.split("_MT")[1].split("_")[0]
    return n[:58]


t0 = int(step[0]["Start_Timestamp"])
t1 = int(rows[b]["Start_Timestamp"])
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
busy, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"step span {(t1 - t0) / 1e3:.1f} us, GPU busy (union) {busy / 1e3:.1f} us, idle "
      f"{(t1 - t0 - busy) / 1e3:.1f} us, kernels {len(step)}")
agg = {}
for r in step:
    k = short(r["Kernel_Name"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    c, t = agg.get(k, (0, 0.0))
    agg[k] = (c + 1, t + d)
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:30]:
    print(f"{t:9.1f} us {c:4d}x {k}")
if "--list" in sys.argv:
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])}")
