"""Instruction mix of one kernel's loops in a hipcc -S listing (dev tool).

usage: python scripts/isa_stats.py file.s KERNEL_SUBSTRING
Prints, for each basic block that is the target of a backward branch (a loop head) up to the
branch, the counts of MFMA / VALU / LDS / VMEM / SALU / waitcnt instructions.
"""
import re
import sys
from collections import Counter

path, want = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = None
for i, l in enumerate(lines):
    if l and l.split()[0].endswith(":") and want in l.split()[0]:
        start = i
        break
if start is None:
    sys.exit("kernel not found")
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = [l.strip() for l in lines[start:end]]
labels = {l[:-1]: i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:$", l)}


def cls(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_exp") or op.startswith("v_log") or op.startswith("v_rcp"):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


for i, l in enumerate(body):
    m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        j = labels[m.group(2)]
        c = Counter(cls(x) for x in body[j:i + 1] if x and not x.startswith((".", ";")) and not x.endswith(":"))
        vops = Counter(x.split()[0] for x in body[j:i + 1] if x.startswith("v_") and not x.startswith("v_mfma"))
        print(f"loop {m.group(2)} lines {j}-{i}: " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
        print("   top VALU:", ", ".join(f"{k}:{v}" for k, v in vops.most_common(14)))
