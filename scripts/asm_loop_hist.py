"""Instruction histogram of a kernel's hottest loop in a hipcc -S listing (dev tool).
usage: asm_loop_hist.py file.s kernel_substring [top]"""
import re
import sys
from collections import Counter

path, key = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end]
# split into basic blocks; a loop = its header block + every block tagged "Header=BB<n>"
blocks, cur = [], None
for l in body:
    m = re.match(r"^\.LBB(\d+_\d+):(.*)$", l)
    if m:
        cur = [m.group(1), m.group(2), []]
        blocks.append(cur)
    elif cur is not None and l.startswith("\t") and not l.strip().startswith(";"):
        cur[2].append(l.split()[0])
best = None
for lab, comment, _ in blocks:
    if "Loop Header" not in comment:
        continue
    ins = [x for b in blocks if b[0] == lab or f"Header=BB{lab}" in b[1] for x in b[2]]
    n_mfma = sum(1 for x in ins if "mfma" in x)
    if best is None or n_mfma > best[0]:
        best = (n_mfma, lab, ins)
n_mfma, lab, ins = best
c = Counter(re.sub(r"_(e32|e64|dpp|sdwa)$", "", x) for x in ins if not x.startswith(".") and "ASM" not in x)
vgpr = re.search(r"\.name:\s+\S*" + re.escape(key) + r"[\s\S]*?\.vgpr_count:\s+(\d+)[\s\S]*?\.vgpr_spill_count:\s+(\d+)",
                 "\n".join(lines))
print(f"{key}: loop {lab}: {len(ins)} instructions, {n_mfma} mfma"
      + (f", vgpr {vgpr.group(1)} spill {vgpr.group(2)}" if vgpr else ""))
print("  " + "  ".join(f"{k}:{v}" for k, v in c.most_common(top)))
