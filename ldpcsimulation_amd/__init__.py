"""ldpcsimulation_amd -- MI355X-native LDPC min-sum BER/FER Monte-Carlo simulator.

Hot path (ereiss123/LDPCsimulation C_implementations/src/decodeMinSum.cpp):
flooding min-sum / normalized / offset min-sum decoding of BPSK/AWGN frames,
as hand-written HIP kernels for gfx950 behind the C ABI in include/ldpc_hip.h.

Submodules:
  native  -- ctypes binding of libldpc_hip.so (no CPU fallback)
  codes   -- alist I/O and the 802.11n QC code generator
  sim     -- SNR-point driver: stop rule, sharded frame index space, collectives
"""
from . import codes  # noqa: F401  (pure Python, no GPU needed)

__all__ = ["codes", "native", "sim"]
