"""Debug: per-basic-block instruction counts of one kernel in the device
assembly (python -m pvnet_amd.build asm output).  usage: asm_blocks.py NAME-SUBSTRING"""
import sys

s = open("pvnet_amd/csrc/pvvote.gfx950.s").read().split("\n")
key = sys.argv[1]
start = next(i for i, l in enumerate(s) if l.startswith("_Z") and key in l and l.split(":")[0].endswith("E"))
blocks, cur = [], ["entry", 0, 0, 0, 0, []]
for l in s[start + 1:]:
    t = l.split(";")[0].strip()
    if t.startswith(".Lfunc_end"):
        break
    if not t or (t.startswith(".") and not t.endswith(":")):
        continue
    if t.endswith(":"):
        blocks.append(cur)
        cur = [t[:-1], 0, 0, 0, 0, []]
        continue
    op = t.split()[0]
    cur[1] += 1
    cur[2] += op.startswith("v_")
    cur[3] += op.startswith(("ds_", "global_", "buffer_", "flat_"))
    if op.startswith(("s_cbranch", "s_branch")):
        cur[5].append(t.split()[-1])
blocks.append(cur)
names = [b[0] for b in blocks]
tot = 0
for k, b in enumerate(blocks):
    tot += b[1]
    back = [x for x in b[5] if x in names and names.index(x) <= k]
    print(f"{b[0]:14s} n={b[1]:4d} valu={b[2]:4d} mem={b[3]:3d} cum={tot:5d}" + (f"  LOOP->{back}" if back else ""))
