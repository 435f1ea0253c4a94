"""Module-level stub plugins for the pipeline API tests (picklable for the
process-pool branch).  They follow the plugin contract of the reference's
pipeline.py:35-39 and touch only files."""
from pathlib import Path


def copy_upper(path: Path, output_dirs, suffix: str = ""):
    out = Path(output_dirs[0]) / f"{path.stem}{suffix}{path.suffix}"
    out.write_text(path.read_text().upper())
    return out


def pair_concat(a: Path, b: Path, output_dirs):
    out = Path(output_dirs[0]) / f"{a.stem}+{b.stem}.txt"
    out.write_text(a.read_text() + "|" + b.read_text())
    return [out]


def fail_on_odd(path: Path, output_dirs):
    if int(path.stem[-1]) % 2:
        raise RuntimeError(f"odd {path.name}")
    out = Path(output_dirs[0]) / path.name
    out.write_text("ok")
    return out


def returns_none(path: Path, output_dirs):
    return None


def returns_str(path: Path, output_dirs):
    return str(path)


def sample_args(path: Path, do_blur: bool, do_rgb: bool, output_dirs):
    out = Path(output_dirs[0]) / f"{path.stem}_{int(do_blur)}{int(do_rgb)}.txt"
    out.write_text("x")
    return out


def _batched(chunk, output_dirs, threads=1, suffix=""):
    res = []
    for (p,) in chunk:
        if p.stem.endswith("3"):
            res.append(ValueError("bad three"))
        else:
            res.append(copy_upper(p, output_dirs, suffix))
    return res


def batch_upper(path: Path, output_dirs, suffix: str = ""):
    return copy_upper(path, output_dirs, suffix)


batch_upper.batch = _batched
