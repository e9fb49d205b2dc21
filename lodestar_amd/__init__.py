"""lodestar_amd — MI355X-native batch BLS12-381 signature-set verifier for Lodestar.

The product is libblsgpu.so (HIP kernels for gfx950 + C-ABI, include/blsgpu.h).
``lodestar_amd.native`` binds it with ctypes; ``lodestar_amd.verifier`` mirrors
the reference's IBlsVerifier (BlsGpuVerifier).  Nothing here imports oracle/.
"""
__all__ = ["native", "verifier", "build"]
