"""vame -- MI355X-native affine motion estimation (VVC, VTM-12.0 gradient search).

Python view of the C ABI in include/vame.h (libvame.so, HIP kernels for gfx950).
Device memory, streams and multi-GPU plumbing come from PyTorch-ROCm; the
compute is entirely in the HIP kernels.  There is no CPU fallback: importing
`vame.engine` without a built libvame.so, or calling it without a HIP device,
raises.
"""
from .hostlogic import lambda_for_poc, poc_qp, ref_list  # noqa: F401

__all__ = ["lambda_for_poc", "poc_qp", "ref_list"]
