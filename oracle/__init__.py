"""CPU ORACLE — test infrastructure only.

This package restates, on the CPU, the pixel arithmetic that the reference
(Tezahc/image_processor_pipeline, mounted read-only at /root/reference) runs on
its hot path through its third-party C libraries (Pillow 12.2.0 for
rotate/getbbox/resize/paste/convert, OpenCV for flip/cvtColor/inRange/
threshold/connectedComponentsWithStats).  Every function cites the reference
call site (file:line) and the library routine it restates.

Rules:
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import anything under ``oracle/``, and only as the
    checker / the reported CPU baseline — never as the product path.
  * Parity status: Pillow-backed ops are PINNED against golden vectors generated
    from Pillow 12.2.0 through the reference's own ``rotations.py`` /
    ``overlays.py`` (``tools/make_goldens.py`` → ``tests/golden/``).  OpenCV
    ops (HSV conversion, inRange, connected components) are restated from
    OpenCV 4.x's published algorithm: "parity unpinned" (OpenCV is absent
    from this image); the CC *partition* is cross-checked against SciPy.
"""
