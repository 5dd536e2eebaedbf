"""Markdown table of SQ counters per kernel from a rocprofv3 --pmc counter_collection.csv
(SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY
SQ_BUSY_CYCLES SQ_WAVE_CYCLES; scripts/gpu_pmc_tpgemm.sh), totals over each kernel's dispatches.
    python3 scripts/sq_table.py <counter_collection.csv>"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, "scripts")
from prof_summary import short  # noqa: E402


def main(path):
    tot = defaultdict(lambda: defaultdict(float))
    order = []
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k not in tot:
            order.append(k)
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    print("| kernel | MFMA instrs | VALU instrs | VALU / MFMA | LDS instrs | LDS bank-conflict / "
          "LDS-active cycles | issue-stall / wave cycles | waitcnt+barrier / wave cycles |")
    print("|---|---|---|---|---|---|---|---|")
    for k in order:
        c = tot[k]
        mf, va = c.get("SQ_INSTS_MFMA", 0.0), c.get("SQ_INSTS_VALU", 0.0)
        lds_act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        wave = c.get("SQ_WAVE_CYCLES", 0.0)
        wany = c.get("SQ_WAIT_ANY")
        print(f"| `{k}` | {mf:.3g} | {va:.3g} | {va / mf if mf else float('nan'):.2f} | "
              f"{c.get('SQ_INSTS_LDS', 0.0):.3g} | "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds_act if lds_act else 0.0:.2f} | "
              f"{c.get('SQ_WAIT_INST_ANY', 0.0) / wave if wave else 0.0:.2f} | "
              f"{'-' if wany is None or not wave else f'{wany / wave:.2f}'} |")

if __name__ == "__main__":
    main(*sys.argv[1:])
