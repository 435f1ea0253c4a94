"""Instruction mix per basic block of one kernel in a hipcc -S output.
  python tools/asm_blocks.py build/obj/ipp_pipe.s <substring of the mangled name>"""
import re
import sys

s = open(sys.argv[1]).read()
names = [n for n in re.findall(r"^(_Z\w+):", s, re.M) if sys.argv[2] in n]
name = names[0]
start = s.index(name + ":")
end = s.index(".Lfunc_end", start)
blocks, cur = [], [name[-20:], []]
for l in s[start:end].splitlines():
    m = re.match(r"^(\.LBB\w+|_Z\w+):", l)
    if m:
        blocks.append(cur)
        cur = [m.group(1), []]
        continue
    t = l.strip()
    if t and not t.startswith((".", ";", "//")):
        cur[1].append(t)
blocks.append(cur)
for lab, ins in blocks:
    if not ins:
        continue
    kinds = {}
    for i in ins:
        op = i.split()[0]
        k = ("v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_")
             else "g" if op.startswith(("global_", "buffer_", "flat_")) else "o")
        kinds[k] = kinds.get(k, 0) + 1
    br = [i for i in ins if i.startswith(("s_cbranch", "s_branch"))]
    print(f"{lab:12s} {len(ins):4d} {kinds} {br[-1] if br else ''}")
