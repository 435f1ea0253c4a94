"""Register / LDS / spill summary of every kernel in a `make asm` .s file
(the amdhsa.kernels metadata): python tools/kernel_res.py build/obj/ipp_pipe.s [filter]"""
import re
import subprocess
import sys


def kernels(path):
    txt = open(path).read()
    meta = txt[txt.index("amdhsa.kernels:"):]
    for blk in re.split(r"\n  - ", meta)[1:]:
        f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
        yield f


def body(asm: str, name: str) -> str:
    """The emitted ISA of kernel `name` (its label to its .Lfunc_end)."""
    a = asm.index("\n" + name + ":")
    return asm[a:asm.index(".Lfunc_end", a)]


def main():
    path = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = list(kernels(path))
    names = [r.get("name", "?") for r in rows]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    for r, d in zip(rows, dem):
        d = re.sub(r"\(anonymous namespace\)::", "", d)
        d = d.split("(")[0]
        if flt and flt not in d:
            continue
        if r.get("vgpr_count") is None:
            continue
        print(f"{d:60s} vgpr {r.get('vgpr_count'):>4} agpr {r.get('agpr_count', '0'):>3} sgpr {r.get('sgpr_count'):>4} "
              f"vspill {r.get('vgpr_spill_count'):>3} sspill {r.get('sgpr_spill_count'):>3} "
              f"lds {r.get('group_segment_fixed_size'):>6} scratch {r.get('private_segment_fixed_size')}")


if __name__ == "__main__":
    main()
