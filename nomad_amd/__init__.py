"""MI355X-native placement engine for Nomad's scheduler hot path.

The product is nomad_amd/libnomadpe.so (HIP kernels for gfx950 + the C ABI of
include/nomad_pe.h). This package holds its host-side mirror of the reference
`scheduler.Stack` interface (stack.py), the flattening of Nomad structs into the
ABI tables (encode.py, structs.py) and seeded synthetic clusters (synth.py).
"""
__all__ = ["abi", "structs", "encode", "stack", "synth"]
