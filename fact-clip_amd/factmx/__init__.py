"""factmx: MI355X-native FACT / FACT_CLIP forward+backward.

Drop-in for fact_clip.models.{basic,blocks,loss} (same class names, constructor
signatures, state_dict keys and config keys); compute runs on hand-written
HIP kernels for gfx950 behind the C ABI in include/factmx.h.
"""
__version__ = "0.1.0"
