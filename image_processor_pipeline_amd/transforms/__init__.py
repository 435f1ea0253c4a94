"""The reference's transform plugins (transforms/*.py), same module and
function names and signatures, pixel work on the MI355X through libipp.so.

Each callable follows the plugin contract of pipeline.py:35-39:
``fn(*input_paths, output_dirs, **options) -> Path | List[Path] | None``.
Calls that need the same random draws as the reference use Python's global
``random`` module in the reference's order.
"""
