"""Static check of the H pass's hand-waited gathers.

k_pipe_hpass2 issues its source gathers as inline-asm buffer_load_dword and
waits for them with an inline-asm s_waitcnt that names the four registers of
its set (ipp_pipe.hip asm_gather / asm_wait).  The compiler does not know
those registers are in flight: if it read, copied or spilled one between its
load and that wait, the copy would carry stale bytes.

For every k_pipe_hpass2 instantiation this builds the control-flow graph of
the emitted ISA and runs a forward may-analysis of in-flight gather
registers (a gather adds its destination, the wait that names a register
removes it; union at joins).  It reports every other instruction that names
an in-flight register, and any scratch use or private segment (spills).

  python tools/asm_hazard.py file.s     (exit 1 on a finding)
"""
from __future__ import annotations

import re
import sys
from typing import Dict, List, Set, Tuple

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")
Reg = Tuple[str, int]


def regs(text: str) -> Set[Reg]:
    out: Set[Reg] = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            out.update((m.group(3), i) for i in range(int(m.group(4)), int(m.group(5)) + 1))
    return out


def kernels(asm: str, pattern: str) -> Dict[str, List[str]]:
    res = {}
    for m in re.finditer(r"^(_Z\S*%s\S*):" % pattern, asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        res[m.group(1)] = asm[m.end():end].split("\n")
    return res


def items(lines: List[str]):
    """(kind, payload): ('label', name) | ('gather', dst regs) | ('wait', regs) |
    ('asm', text) | ('ins', text)."""
    out = []
    i, n = 0, len(lines)
    while i < n:
        raw = lines[i].strip()
        if raw.startswith(";;#ASMSTART"):
            j = i + 1
            block = []
            while j < n and not lines[j].strip().startswith(";;#ASMEND"):
                block.append(lines[j].strip())
                j += 1
            text = "\n".join(block)
            if "buffer_load_dword" in text:
                out.append(("gather", regs(text.split("buffer_load_dword", 1)[1].split(",")[0])))
            elif "gather wait" in text:
                out.append(("wait", regs(text.split("gather wait", 1)[1].split("\n")[0])))
            else:
                out.append(("asm", text))
            i = j + 1
            continue
        code = raw.split(";")[0].strip()
        if code.endswith(":") and not code.startswith("."):
            out.append(("label", code[:-1]))
        elif code.startswith(".LBB") and code.endswith(":"):
            out.append(("label", code[:-1]))
        elif code and not code.startswith("."):
            out.append(("ins", code))
        elif code.startswith(".LBB"):
            out.append(("label", code.rstrip(":")))
        i += 1
    return out


def cfg(its):
    """Split into basic blocks; successors by label."""
    blocks, cur = [], []
    for it in its:
        if it[0] == "label" and cur:
            blocks.append(cur)
            cur = []
        cur.append(it)
        if it[0] == "ins" and (it[1].startswith("s_branch") or it[1].startswith("s_cbranch")
                               or it[1].startswith("s_endpgm") or it[1].startswith("s_setpc")):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    label_of = {}
    for bi, b in enumerate(blocks):
        if b[0][0] == "label":
            label_of[b[0][1]] = bi
    succ = []
    for bi, b in enumerate(blocks):
        last = b[-1]
        s = []
        if last[0] == "ins" and last[1].startswith("s_branch"):
            s.append(label_of[last[1].split()[1]])
        elif last[0] == "ins" and last[1].startswith("s_cbranch"):
            s.append(label_of[last[1].split()[1]])
            if bi + 1 < len(blocks):
                s.append(bi + 1)
        elif last[0] == "ins" and (last[1].startswith("s_endpgm") or last[1].startswith("s_setpc")):
            pass
        elif bi + 1 < len(blocks):
            s.append(bi + 1)
        succ.append(s)
    return blocks, succ


def check_kernel(lines: List[str]) -> List[str]:
    blocks, succ = cfg(items(lines))
    n = len(blocks)
    inn: List[Set[Reg]] = [set() for _ in range(n)]
    out: List[Set[Reg]] = [set() for _ in range(n)]
    changed = True
    while changed:
        changed = False
        for bi in range(n):
            live = set(inn[bi])
            for kind, pay in blocks[bi]:
                if kind == "gather":
                    live |= pay
                elif kind == "wait":
                    live -= pay
            if live != out[bi]:
                out[bi] = live
                changed = True
                for s in succ[bi]:
                    if not live <= inn[s]:
                        inn[s] |= live
    problems = []
    for bi in range(n):
        live = set(inn[bi])
        for kind, pay in blocks[bi]:
            if kind == "gather":
                # (a gather into a register another path left in flight is
                # not itself a read: the in-order returns leave the newer
                # value, and the static paths are correlated — a live issue
                # always reaches its wait)
                live |= pay
            elif kind == "wait":
                live -= pay
            elif kind in ("ins", "asm"):
                if "scratch_" in pay:
                    problems.append(f"scratch access: {pay}")
                hit = regs(pay) & live
                if hit:
                    problems.append(f"in-flight gather register {sorted(hit)} touched: {pay}")
    return problems


def main(path: str, pattern: str = "k_pipe_hpass2") -> int:
    asm = open(path).read()
    ks = kernels(asm, pattern)
    bad = 0
    for name, lines in ks.items():
        meta = re.search(r"\.amdhsa_kernel %s(.*?)\.end_amdhsa_kernel" % re.escape(name), asm, re.S)
        priv = int(re.search(r"\.amdhsa_private_segment_fixed_size\s+(\d+)", meta.group(1)).group(1)) if meta else 0
        probs = check_kernel(lines)
        # A private segment matters when the kernel touches it (the scratch
        # accesses check_kernel reports, or buffer accesses through the
        # scratch resource); the backend can leave a frame reserved for SGPR
        # spill slots that all went to VGPR lanes, which nothing reads.
        if priv and any(re.search(r"\bbuffer_\w+\b.*\bs\[0:3\]", l) for l in lines):
            probs.append(f"private segment {priv} B accessed through the scratch resource")
        elif priv:
            print(f"{name}: note: private segment {priv} B reserved, never accessed")
        if probs:
            bad += 1
            print(name)
            for p in probs[:8]:
                print("   ", p)
    print(f"{len(ks)} kernels checked, {bad} with findings")
    return 1 if bad or not ks else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
