"""Stream overlap in a rocprofv3 kernel trace: per stream, kernel time; and for kernels whose name
starts with PREFIX, how much of their time overlaps kernels of other streams.
    python3 scripts/trace_overlap.py <kernel_trace.csv> [prefix]"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, "scripts")
from prof_summary import short  # noqa: E402


def main(path, prefix="tp_node_outer"):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["k"] = short(r["Kernel_Name"])
    by = defaultdict(list)
    for r in rows:
        by[r["Stream_Id"]].append(r)
    for sid, ks in by.items():
        print(f"stream {sid}: {len(ks)} kernels, {sum(r['e'] - r['s'] for r in ks) / 1e6:.1f} ms")
    tgt = [r for r in rows if r["k"].startswith(prefix)]
    tot = ov = 0
    for r in tgt:
        others = [(q["s"], q["e"]) for q in rows if q["Stream_Id"] != r["Stream_Id"]
                  and q["e"] > r["s"] and q["s"] < r["e"]]
        # union of the overlapping intervals clipped to r
        iv = sorted((max(a, r["s"]), min(b, r["e"])) for a, b in others)
        u, cur = 0, None
        for a, b in iv:
            if cur is None or a > cur[1]:
                if cur:
                    u += cur[1] - cur[0]
                cur = [a, b]
            else:
                cur[1] = max(cur[1], b)
        if cur:
            u += cur[1] - cur[0]
        tot += r["e"] - r["s"]
        ov += u
    print(f"{prefix}: {len(tgt)} launches, {tot / 1e6:.1f} ms, overlapped with other streams "
          f"{ov / 1e6:.1f} ms ({ov / max(tot, 1):.0%})")
    if tgt:
        r = tgt[len(tgt) // 2]
        print("streams of the target kernel:", sorted({q["Stream_Id"] for q in tgt}))


if __name__ == "__main__":
    main(*sys.argv[1:])
