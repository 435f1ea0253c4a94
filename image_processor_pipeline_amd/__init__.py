"""image_processor_pipeline_amd — MI355X-native hot path of
Tezahc/image_processor_pipeline.

Layers:
  * ``pipeline``    — ProcessingStep / ProcessingPipeline (the compose API of
                      the reference's pipeline.py, plus a batched device mode).
  * ``transforms``  — the reference's plugin callables, same names/signatures.
  * ``device``      — tensor-level ops over the HIP C-ABI (libipp.so).
  * ``fused``       — the batched 5-stage pipe (configs 3/4).
  * ``geometry``    — host planning that reproduces Pillow/OpenCV host math.
  * ``_native``     — ctypes binding of include/ipp.h.
"""
__version__ = "0.1.0"
