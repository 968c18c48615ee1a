"""MI355X-native adapter-alignment engine for Porechop_ABI.

The hot path of hritikbharucha/Custom_Porechop_ABI -- every read window x every adapter at the
read ends, plus the middle-adapter scan -- runs as hand-written HIP kernels for gfx950 behind a
C ABI (include/pcabi.h, libpcabi.so). The Python modules mirror the reference's interfaces for
that path: cpp_function_wrappers.adapter_alignment, nanopore_read.NanoporeRead /
align_adapter, and the phase drivers of porechop_abi.py (now batched).
"""
__version__ = '0.1.0'
