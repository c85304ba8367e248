"""Basic blocks of one kernel in a hipcc -S listing: label, instruction counts by class, branch targets.
usage: python tools/isa_blocks.py <listing.s> <kernel-symbol-substring>"""
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
key = sys.argv[2]
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l and l.rstrip().endswith(key + ":") or (l.startswith("_Z") and key in l.split(":")[0]))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
blocks, cur = [], {"label": "entry", "v": 0, "s": 0, "m": 0, "o": 0, "br": [], "ins": []}
for l in lines[start + 1:end]:
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        if re.match(r"^\.LBB\S+:", t):
            blocks.append(cur)
            cur = {"label": t.split(":")[0], "v": 0, "s": 0, "m": 0, "o": 0, "br": [], "ins": []}
        continue
    op = t.split()[0]
    cur["ins"].append(t.split(";")[0].strip())
    if op.startswith("v_"):
        cur["v"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"):
        cur["br"].append((op, t.split()[1] if len(t.split()) > 1 else ""))
        cur["s"] += 1
    elif op.startswith("s_"):
        cur["s"] += 1
    elif op.startswith(("global_", "buffer_", "ds_", "flat_", "scratch_")):
        cur["m"] += 1
    else:
        cur["o"] += 1
blocks.append(cur)
tv = sum(b["v"] for b in blocks)
ts = sum(b["s"] for b in blocks)
print("%d blocks, %d VALU, %d SALU (static)" % (len(blocks), tv, ts))
for b in blocks:
    print("%-14s V%4d S%4d M%3d  -> %s" % (b["label"], b["v"], b["s"], b["m"], " ".join("%s %s" % x for x in b["br"])))
    if "-v" in sys.argv:
        for i in b["ins"]:
            print("      " + i)
