"""Per-stream timeline of one training step from a rocprofv3 kernel trace (stats_kernel_trace.csv):
step = the span between the first launches of a marker kernel in consecutive steps (marker: a
kernel name prefix launched `per_step` times per step); per stream: busy time, idle gaps and
the kernels with the most time; gaps > 5 us listed with the kernels around them.
    python3 scripts/trace_timeline.py <trace.csv> [marker] [per_step] [step_idx]"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, "scripts")
from prof_summary import short  # noqa: E402


def main(path, marker="egnn_fwd_kernel", per_step=4, step_idx=-2, top=12):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["k"] = short(r["Kernel_Name"])
    rows.sort(key=lambda r: r["s"])
    mk = [r for r in rows if r["k"].startswith(marker)][::per_step]
    a, b = mk[step_idx]["s"], mk[step_idx + 1]["s"]
    step = [r for r in rows if a <= r["s"] < b]
    print(f"step wall {(b - a) / 1e3:.1f} us, {len(step)} kernels")
    by = defaultdict(list)
    for r in step:
        by[r["Stream_Id"]].append(r)
    for sid, ks in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy = sum(r["e"] - r["s"] for r in ks)
        tot = defaultdict(float)
        for r in ks:
            tot[r["k"]] += (r["e"] - r["s"]) / 1e3
        print(f"stream {sid}: {len(ks)} kernels, busy {busy / 1e3:.1f} us")
        for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
            print(f"    {v:8.1f} us  {k}")
        gaps = []
        for p, q in zip(ks, ks[1:]):
            if q["s"] - p["e"] > 5000:
                gaps.append(((q["s"] - p["e"]) / 1e3, p["k"], q["k"]))
        idle = sum(g for g, _, _ in gaps)
        print(f"    gaps > 5 us: {len(gaps)}, {idle:.1f} us")
        for g in sorted(gaps, reverse=True)[:8]:
            print(f"      {g[0]:7.1f} us  after {g[1]}  before {g[2]}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *(int(x) for x in sys.argv[3:5]))
