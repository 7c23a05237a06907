"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (tuning aid).
usage: isa_blocks.py kernels.s KERNEL [min_instrs]"""
import re
import sys

src, kern = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(kern + ":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur, order = {}, "entry", ["entry"]
blocks[cur] = []
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        cur = m.group(1)
        order.append(cur)
        blocks[cur] = []
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    blocks[cur].append(t.split()[0])
pos = {b: i for i, b in enumerate(order)}
def cls(op):
    for p, n in (("v_readlane", "readlane"), ("v_writelane", "writelane"), ("v_", "valu"), ("s_load", "smem"),
                 ("s_buffer_load", "smem"), ("s_waitcnt", "wait"), ("s_cbranch", "branch"), ("s_branch", "branch"),
                 ("s_", "salu"), ("global_load", "vmem"), ("buffer_load", "vmem"), ("global_store", "vst"),
                 ("buffer_store", "vst"), ("ds_", "lds"), ("flat_", "flat"), ("scratch_", "scratch")):
        if op.startswith(p):
            return n
    return "other"
tot = {}
for b in order:
    mix = {}
    for op in blocks[b]:
        k = cls(op)
        mix[k] = mix.get(k, 0) + 1
        tot[k] = tot.get(k, 0) + 1
    back = [l for l in blocks[b] if False]
    if len(blocks[b]) >= mn:
        print(b, len(blocks[b]), mix)
print("TOTAL", sum(tot.values()), tot)
# loops: branches to a label at or before the current block
for i, l in enumerate(lines[start + 1:end]):
    m = re.match(r"\s*s_c?branch\w*\s+(\.LBB\w+)", l)
    if m:
        pass
cur = "entry"
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        cur = m.group(1)
    m = re.match(r"\s*s_c?branch\w*\s+(\.LBB\w+)", l)
    if m and m.group(1) in pos and pos[m.group(1)] <= pos[cur]:
        body = order[pos[m.group(1)]:pos[cur] + 1]
        print("LOOP", m.group(1), "->", cur, "blocks", len(body), "instrs", sum(len(blocks[x]) for x in body))
