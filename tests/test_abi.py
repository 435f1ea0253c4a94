"""C-ABI boundary checks (CPU): the library loads, exports every entry point
include/ipp.h declares, and the ctypes/NumPy struct mirrors match the C
layouts exactly (offsets computed by the C compiler)."""
import re
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

from image_processor_pipeline_amd import _native as N

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "ipp.h"


def declared_functions():
    src = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(ipp_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_symbol():
    lib = N.load()
    names = declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) <= set(N.SIGNATURES), set(names) - set(N.SIGNATURES)
    assert b"gfx950" in lib.ipp_version()


STRUCTS = {
    "ipp_gather_desc": N.GATHER_DESC,
    "ipp_copy_desc": N.COPY_DESC,
    "ipp_hsv_range": N.HSV_RANGE,
    "ipp_hsv_params": N.HSV_PARAMS,
    "ipp_image_desc": N.IMAGE_DESC,
    "ipp_resample_desc": N.RESAMPLE_DESC,
    "ipp_paste_desc": N.PASTE_DESC,
    "ipp_pipe_desc": N.PIPE_DESC,
    "ipp_ccl_work": N.CCL_WORK,
    "ipp_affine_desc": N.AFFINE_DESC,
    "ipp_enhance_desc": N.ENHANCE_DESC,
    "ipp_pipe_plan_cfg": N.PIPE_PLAN_CFG,
    "ipp_pipe_item": N.PIPE_ITEM,
    "ipp_tap_axis": N.TAP_AXIS,
}


def test_struct_layouts_match_c_compiler():
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, dt in STRUCTS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in dt.names:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as td:
        c = Path(td) / "l.c"
        c.write_text("\n".join(lines))
        exe = Path(td) / "l"
        subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(c)], check=True)
        out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for ln in out:
        if ln:
            s, f, v = ln.split()
            got[(s, f)] = int(v)
    for cname, dt in STRUCTS.items():
        assert got[(cname, "size")] == dt.itemsize, cname
        for f in dt.names:
            assert got[(cname, f)] == dt.fields[f][1], (cname, f)


def test_hsv_tables_in_source_match_cvround():
    src = (ROOT / "image_processor_pipeline_amd" / "csrc" / "ipp_hsv.h").read_text()
    def table(name):
        body = re.search(name + r"\[256\] = \{(.*?)\};", src, re.S).group(1)
        return np.array([int(v) for v in body.replace("\n", " ").split(",") if v.strip()])
    from oracle.ops import SDIV_TABLE, HDIV_TABLE_180
    assert np.array_equal(table("kSdiv"), SDIV_TABLE)
    assert np.array_equal(table("kHdiv180"), HDIV_TABLE_180)


def test_product_library_reads_no_environment():
    """Diagnostic kernel switches exist only in -DIPP_DIAG builds: the product
    libipp.so does not even import getenv, so no environment variable can
    select a different (wrong-output) kernel."""
    import shutil
    import subprocess
    from image_processor_pipeline_amd import _native as N
    nm = shutil.which("nm") or "/usr/bin/nm"
    out = subprocess.run([nm, "-D", "--undefined-only", str(N.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert "getenv" not in out and "secure_getenv" not in out


def test_header_constants_match_the_python_mirror():
    """#define constants the host code mirrors (plan totals, copy group)."""
    src = HEADER.read_text()
    consts = dict(re.findall(r"#define (IPP_[A-Z0-9_]+) (-?\d+)", src))
    assert int(consts["IPP_PLAN_TOTALS"]) == N.IPP_PLAN_TOTALS
    assert int(consts["IPP_PIPE_COPY_GROUP"]) == N.IPP_PIPE_COPY_GROUP
    assert int(consts["IPP_PIPE_MAX_OV_W"]) == N.IPP_PIPE_MAX_OV_W
    for name, slot in N.PT.items():
        assert int(consts["IPP_PT_" + name.upper()]) == slot, name
