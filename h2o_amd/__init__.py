"""h2o_amd -- MI355X-native HPACK/QPACK Huffman codec (hhuff).

The product is the C-ABI library h2o_amd/libhhuff.so (HIP kernels for gfx950 + host shim, declared in
include/hhuff.h).  This package is the thin host-side mirror used by tests and bench.py:
  h2o_amd.codec   ctypes bindings of the C-ABI (per-string h2o signatures + device batch API)
  h2o_amd.dist    multi-GPU sharding of a batch (one process per GPU, torch.distributed)
  h2o_amd.synth   seeded synthetic batches for the benchmark configurations
  h2o_amd.tables  generated RFC 7541 code table (tools/gen_tables.py)
"""
__all__ = ["codec", "dist", "synth", "tables"]
