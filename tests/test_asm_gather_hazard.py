"""Static guard of the H pass's hand-waited gathers (gather
waits).  k_pipe_hpass2 issues its source gathers by inline asm and waits for
them by hand; a compiler copy, read or spill of a gather register before the
wait that names it would carry stale bytes.  tools/asm_hazard.py checks the
emitted ISA of every instantiation (control-flow-aware); this test runs it on
the build's ipp_pipe.s and on a mutation of the source that drops the
end-of-phase-2 waits (the round-2 structure: the next chunk's sets stayed in
flight across the loop's back edge, where the compiler copies them)."""
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "image_processor_pipeline_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"
sys.path.insert(0, str(ROOT))
from tools import asm_hazard  # noqa: E402

needs_hipcc = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


def _compile(src: Path, out: Path, inc: Path):
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT / 'include'}",
                    f"-I{inc}", "-S", "--cuda-device-only", str(src), "-o", str(out)],
                   check=True, capture_output=True)


def _asm_of_build(tmp_path) -> Path:
    s = ROOT / "build" / "obj" / "ipp_pipe.s"
    deps = [CSRC / "ipp_pipe.hip"] + list(CSRC.glob("*.h")) + [ROOT / "include" / "ipp.h"]
    if s.exists() and s.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return s
    out = tmp_path / "ipp_pipe.s"
    _compile(CSRC / "ipp_pipe.hip", out, CSRC)
    return out


@needs_hipcc
def test_hpass_gathers_never_touched_in_flight(tmp_path, capsys):
    path = _asm_of_build(tmp_path)
    for pattern, least in (("k_pipe_hpass2", 24),):
        rc = asm_hazard.main(str(path), pattern)
        out = capsys.readouterr().out
        n = int(re.search(r"(\d+) kernels checked", out).group(1))
        assert n >= least, out     # every NR / zones / channels instantiation
        assert rc == 0, out        # no in-flight register touched, no scratch


@needs_hipcc
def test_checker_flags_waits_left_to_the_back_edge(tmp_path, capsys):
    src = (CSRC / "ipp_pipe.hip").read_text()
    waits = ("        asm_wait(RA.p, RA.live ? 4 * RB.live : -1);\n"
             "        asm_wait(RB.p, RB.live ? 0 : -1);\n        if (!more) break;")
    assert waits in src
    mutated = src.replace(waits, "        if (!more) break;")
    d = tmp_path / "mut"
    d.mkdir()
    for h in CSRC.glob("*.h"):
        shutil.copy(h, d)
    (d / "ipp_pipe.hip").write_text(mutated)
    _compile(d / "ipp_pipe.hip", d / "ipp_pipe.s", d)
    rc = asm_hazard.main(str(d / "ipp_pipe.s"))
    out = capsys.readouterr().out
    assert rc == 1 and "in-flight gather register" in out, out
