"""transplat_amd — MI355X-native (gfx950) TranSplat inference hot path.

Mirrors the reference's `src/model` encoder -> gaussian-adapter -> decoder operator API; the
window attention, depth-candidate correlation and Gaussian rasterizer run as hand-written HIP
kernels behind the C-ABI in include/transplat_hip.h.
"""
__version__ = "0.1.0"
