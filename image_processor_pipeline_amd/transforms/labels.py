"""change_label_class — reference transforms/labels.py:7-65 (YOLO label side
channel of the dataset chain).

Text work on the host, as in the reference: every non-empty line
``cls x y w h`` gets ``cls`` mapped through ``cls_mapping`` (unmapped ids
unchanged), written to ``output_dirs[0] / input_path.name``; on any error the
message is printed, the partial output removed and None returned.
The reference's own known-answer self-check (labels.py:67-128) passes a
``class_id_mapping=`` keyword the function does not take;
here, as there, such a keyword lands in ``**options`` and is ignored.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Dict, List, Optional


def change_label_class(input_path: Path,
                       output_dirs: List[Path],
                       cls_mapping: Optional[Dict[int, int]] = None,
                       **options: Any) -> Optional[Path]:
    cls_mapping = {0: 0} if cls_mapping is None else cls_mapping
    output_dir = Path(output_dirs[0])
    output_path = output_dir / Path(input_path).name
    try:
        with Path(input_path).open("r", encoding="utf-8") as fin, output_path.open("w", encoding="utf-8") as fout:
            for line in fin:
                parts = line.strip().split()
                if not parts:
                    continue
                cur = int(parts[0])
                parts[0] = str(cls_mapping.get(cur, cur))
                fout.write(" ".join(parts) + "\n")
        return output_path
    except Exception as e:
        print(f"Problème : {e}")
        if output_path.exists():
            output_path.unlink()
        return None
