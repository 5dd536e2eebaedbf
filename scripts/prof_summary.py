"""Summarise a gpurun_out/prof_<workload>/ rocprofv3 directory (scripts/gpu_profile.sh) into
profiles/<round>_<workload>_kernels.md + .json: per kernel calls, average duration and share
(--kernel-trace --stats pass) and per-dispatch HBM traffic from the separate FETCH_SIZE and
WRITE_SIZE passes.  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts
half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.  Counter
values are KB (rocprofv3 derived metric units)."""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "").replace("gmp::", "").replace("at::native::", "")
    if n.startswith("Cijk_"):
        n = "rocBLAS/Tensile " + n.split("_MT")[1].split("_")[0] if "_MT" in n else "Tensile GEMM"
    return n[:70]


def load_counters(path, counter):
    per = defaultdict(list)
    if not os.path.exists(path):
        return per
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main(src, workload, tag, steps=None):
    stats = os.path.join(src, "stats_kernel_stats.csv")
    rows = []
    with open(stats) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    fetch = load_counters(os.path.join(src, "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = load_counters(os.path.join(src, "write_counter_collection.csv"), "WRITE_SIZE")
    out = []
    for r in rows:
        name = r["Name"]
        fb = fetch.get(name)
        wb = write.get(name)
        out.append({
            "kernel": short(name), "full_name": name, "calls": int(r["Calls"]),
            "avg_us": float(r["AverageNs"]) / 1e3, "total_ms": float(r["TotalDurationNs"]) / 1e6,
            "pct": float(r["Percentage"]),
            "hbm_read_bytes_per_launch": (2.0 * sum(fb) / len(fb)) if fb else None,
            "hbm_write_bytes_per_launch": (sum(wb) / len(wb)) if wb else None,
        })
    os.makedirs("profiles", exist_ok=True)
    base = os.path.join("profiles", f"{tag}_{workload}_kernels")
    with open(base + ".json", "w") as f:
        json.dump({"workload": workload, "source": "rocprofv3 --kernel-trace --stats; "
                   "--pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE in separate passes",
                   # training steps the traced run executed (warm-up + timed): calls / steps =
                   # launches per step (bench.py reads per-step kernel time and HBM bytes)
                   "steps_in_trace": steps, "kernels": out}, f, indent=1)
    with open(base + ".md", "w") as f:
        f.write(f"# rocprofv3 kernel summary — {workload} ({tag})\n\n")
        if steps:
            tot = sum(o["total_ms"] for o in out) / steps
            f.write(f"{steps} training steps in the trace; kernel time {tot:.1f} ms per step")
            if all(o["hbm_read_bytes_per_launch"] is not None for o in out):
                hbm = sum(o["calls"] * (o["hbm_read_bytes_per_launch"] +
                                        o["hbm_write_bytes_per_launch"]) for o in out) / steps
                f.write(f"; HBM traffic (PMC) {hbm / 1e9:.1f} GB per step")
            f.write(".\n\n")
        f.write("| kernel | calls | avg µs | % time | HBM read MB/launch | HBM write MB/launch |\n")
        f.write("|---|---|---|---|---|---|\n")
        for o in out[:40]:
            rd = "" if o["hbm_read_bytes_per_launch"] is None else \
                f"{o['hbm_read_bytes_per_launch'] / 1e6:.1f}"
            wr = "" if o["hbm_write_bytes_per_launch"] is None else \
                f"{o['hbm_write_bytes_per_launch'] / 1e6:.1f}"
            f.write(f"| `{o['kernel']}` | {o['calls']} | {o['avg_us']:.1f} | {o['pct']:.2f} | "
                    f"{rd} | {wr} |\n")
    print(base)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "r01",
         int(sys.argv[4]) if len(sys.argv) > 4 else None)
