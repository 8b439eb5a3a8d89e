"""Compute ops: HIP kernels for gfx950 with PyTorch CPU reference paths."""
