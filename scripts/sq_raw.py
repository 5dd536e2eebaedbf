"""Per-kernel totals of every counter in a rocprofv3 counter_collection.csv (markdown), with each
SQ_WAIT_* / SQ_ACTIVE_* / SQ_*_CYCLES column also as a fraction of SQ_WAVE_CYCLES when present.
    python3 scripts/sq_raw.py <counter_collection.csv> [kernel-substring]"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, "scripts")
from prof_summary import short  # noqa: E402

tot = defaultdict(lambda: defaultdict(float))
order, names = [], []
for r in csv.DictReader(open(sys.argv[1])):
    k = short(r["Kernel_Name"])
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    if k not in tot:
        order.append(k)
    if r["Counter_Name"] not in names:
        names.append(r["Counter_Name"])
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
print("| kernel | " + " | ".join(names) + " |")
print("|---" * (len(names) + 1) + "|")
for k in order:
    c, wc = tot[k], tot[k].get("SQ_WAVE_CYCLES")
    cells = []
    for n in names:
        v = c.get(n, 0.0)
        cells.append(f"{v:.3g}" + (f" ({v / wc:.2f})" if wc and n != "SQ_WAVE_CYCLES" and
                                    ("CYCLES" in n or "WAIT" in n or "ACTIVE" in n) else ""))
    print(f"| `{k}` | " + " | ".join(cells) + " |")
