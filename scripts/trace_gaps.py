"""Timeline of one training step from a rocprofv3 kernel trace (dev tool): kernels in start
order with gaps and per-stream busy time, for the step between the last two occurrences of a
marker kernel.  usage: trace_gaps.py kernel_trace.csv [marker-substring] [max-lines] [markers-per-step]"""
import csv
import sys

t = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "gather_rows"
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
per = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # marker occurrences per step
t.sort(key=lambda x: int(x["Start_Timestamp"]))
starts = [i for i, x in enumerate(t) if marker in x["Kernel_Name"]]
i0, i1 = starts[-1 - 2 * per], starts[-1 - per]
seg = t[i0:i1]
T0 = int(seg[0]["Start_Timestamp"])
qkey = "Queue_Id" if "Queue_Id" in seg[0] else ("Stream_Id" if "Stream_Id" in seg[0] else None)
busy, last_end = {}, {}
for n, x in enumerate(seg):
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    q = x.get(qkey, "?") if qkey else "?"
    gap = s - last_end.get(q, s)
    busy[q] = busy.get(q, 0) + e - s
    last_end[q] = max(last_end.get(q, 0), e)
    if n < lim:
        print(f"{(s - T0) / 1e3:8.1f} q{q:>3} +{gap / 1e3:6.1f} {(e - s) / 1e3:7.1f}  {x['Kernel_Name'][:80]}")
span = max(last_end.values()) - T0
print(f"span {span / 1e3:.1f} us; busy per queue: " +
      ", ".join(f"q{q} {b / 1e3:.1f}" for q, b in busy.items()))
