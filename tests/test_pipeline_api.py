"""ProcessingStep / ProcessingPipeline behaviour (CPU, stub plugins):
pairing modes, chaining, logs/JSON, error accounting, worker clamping and
the batched-call hook.  Mirrors the reference pipeline.py:12-584."""
import json
import os
import random
from pathlib import Path

import pytest

import plugins_stub as P
from image_processor_pipeline_amd.pipeline import MODES, PathJSONEncoder, ProcessingPipeline, ProcessingStep


def _inputs(d: Path, n: int, prefix: str = "f"):
    d.mkdir(parents=True, exist_ok=True)
    for i in range(n):
        (d / f"{prefix}{i}.txt").write_text(f"{prefix}{i}")
    return d


def test_modes_and_validation(tmp_path):
    assert MODES == ('one_input', 'zip', 'modulo', 'sample', 'custom')
    with pytest.raises(ValueError):
        ProcessingStep("s", P.copy_upper, input_dirs=tmp_path)           # no output dirs
    with pytest.raises(ValueError):
        ProcessingStep("s", P.copy_upper, tmp_path, tmp_path / "o", pairing_method="bogus")
    with pytest.raises(ValueError):
        ProcessingStep("s", P.copy_upper, tmp_path, tmp_path / "o", pairing_method="custom")
    with pytest.raises(ValueError):
        ProcessingStep("s", P.copy_upper, [tmp_path, 3], tmp_path / "o")
    s = ProcessingStep("s", P.copy_upper, "in", "out", root_dir=tmp_path)
    assert s.input_paths == [tmp_path / "in"] and s.output_paths == [tmp_path / "out"]
    assert "Étape 's'" in str(s)


def test_one_input_sequential_logs_json(tmp_path):
    src = _inputs(tmp_path / "in", 4)
    s = ProcessingStep("up", P.copy_upper, src, tmp_path / "out" / "a", save_log=True, options={"suffix": "_u"})
    s.run()
    outs = sorted((tmp_path / "out" / "a").iterdir())
    assert [o.name for o in outs] == [f"f{i}_u.txt" for i in range(4)]
    assert outs[0].read_text() == "F0"
    assert [l["status"] for l in s.process_logs] == ["Success"] * 4
    log = json.loads((tmp_path / "out" / "up.json").read_text())
    assert log[0]["inputs"] == [str(src / "f0.txt")] and log[0]["outputs"] == [str(outs[0])]


def test_error_accounting_sequential_and_parallel(tmp_path, capsys):
    src = _inputs(tmp_path / "in", 6)
    for workers in (1, 2):
        s = ProcessingStep("odd", P.fail_on_odd, src, tmp_path / f"o{workers}", workers=workers)
        s.run()
        st = sorted(l["status"] for l in s.process_logs)
        assert st == ["Error"] * 3 + ["Success"] * 3, workers
        out = capsys.readouterr().out
        assert "3 éléments traités avec succès" in out and "3 erreur(s)" in out


def test_no_output_and_type_error(tmp_path):
    src = _inputs(tmp_path / "in", 2)
    s = ProcessingStep("none", P.returns_none, src, tmp_path / "o")
    s.run()
    assert {l["status"] for l in s.process_logs} == {"no_output"}
    s = ProcessingStep("str", P.returns_str, src, tmp_path / "o2")
    with pytest.warns(UserWarning):
        s.run()
    assert {l["status"] for l in s.process_logs} == {"Type Error"}


def test_zip_modulo_sample_custom(tmp_path):
    a = _inputs(tmp_path / "a", 5, "a")
    b = _inputs(tmp_path / "b", 2, "b")
    s = ProcessingStep("zip", P.pair_concat, [a, b], tmp_path / "z", pairing_method="zip")
    s.run()
    assert len(s.process_logs) == 2
    random.seed(7)
    s = ProcessingStep("mod", P.pair_concat, [a, b], tmp_path / "m", pairing_method="modulo")
    s.run()
    random.seed(7)
    bl = sorted((b).iterdir())
    random.shuffle(bl)
    exp = [f"a{i}+{bl[i % 2].stem}.txt" for i in range(5)]
    assert [Path(l["outputs"][0]).name for l in s.process_logs] == exp
    random.seed(3)
    s = ProcessingStep("smp", P.sample_args, a, tmp_path / "s", pairing_method="sample")
    s.run()
    random.seed(3)
    files = sorted(a.iterdir())
    blur = set(random.sample(files, 1))
    rgb = set(random.sample(files, 1))
    exp = [f"{f.stem}_{int(f in blur)}{int(f in rgb)}.txt" for f in files]
    assert [Path(l["outputs"][0]).name for l in s.process_logs] == exp
    s = ProcessingStep("cus", P.pair_concat, [a, b], tmp_path / "c", pairing_method="custom",
                       pairing_function=lambda lists: [(lists[0][0], lists[1][1])])
    s.run()
    assert [Path(l["outputs"][0]).name for l in s.process_logs] == ["a0+b1.txt"]


def test_sample_k_and_missing_inputs(tmp_path, capsys):
    a = _inputs(tmp_path / "a", 6)
    random.seed(1)
    s = ProcessingStep("k", P.copy_upper, a, tmp_path / "o", sample_k=3)
    s.run()
    assert len(s.process_logs) == 3
    s = ProcessingStep("missing", P.copy_upper, tmp_path / "nope", tmp_path / "o2")
    s.run()
    assert "Condition préalable non remplie" in capsys.readouterr().out and s.process_logs == []


def test_pipeline_chaining_and_run(tmp_path):
    src = _inputs(tmp_path / "in", 3)
    pipe = ProcessingPipeline(root_dir=tmp_path)
    with pytest.raises(ValueError):
        pipe.add_step(ProcessingStep("x", P.copy_upper, output_dirs="o"))
    pipe.add_step(ProcessingStep("s1", P.copy_upper, "in", "o1", options={"suffix": "_1"}))
    pipe.add_step(ProcessingStep("s3", P.copy_upper, output_dirs="o3", options={"suffix": "_3"}))
    pipe.add_step(ProcessingStep("s2", P.copy_upper, output_dirs="o2", options={"suffix": "_2"}), position=1)
    assert [s.name for s in pipe.steps] == ["s1", "s2", "s3"]
    assert pipe.steps[1].input_paths == [tmp_path / "o1"] and pipe.steps[2].input_paths == [tmp_path / "o2"]
    with pytest.raises(IndexError):
        pipe.add_step(ProcessingStep("s0", P.copy_upper, output_dirs="o0"), position=0)
    with pytest.raises(IndexError):
        pipe.run(from_step_index=5)
    pipe.run()
    assert sorted(p.name for p in (tmp_path / "o3").iterdir()) == [f"f{i}_1_2_3.txt" for i in range(3)]
    assert (tmp_path / "o3" / "f0_1_2_3.txt").read_text() == "F0"


def test_workers_clamped():
    with pytest.warns(UserWarning):
        s = ProcessingStep("w", P.copy_upper, "i", "o", workers=10 ** 6)
    assert s.parallels_workers == os.cpu_count()
    assert ProcessingStep("w", P.copy_upper, "i", "o", workers=-1).parallels_workers == os.cpu_count()


def test_batch_hook(tmp_path):
    src = _inputs(tmp_path / "in", 7)
    s = ProcessingStep("b", P.batch_upper, src, tmp_path / "o", batch_size=3, options={"suffix": "_b"})
    s.run()
    st = [l["status"] for l in s.process_logs]
    assert st == ["Success"] * 3 + ["Error"] + ["Success"] * 3
    assert s.process_logs[3]["error_message"].endswith("bad three")
    assert len(list((tmp_path / "o").iterdir())) == 6


def test_json_encoder():
    assert json.loads(json.dumps({"p": Path("/a/b"), "t": (1, 2)}, cls=PathJSONEncoder)) == {"p": "/a/b", "t": [1, 2]}
