"""MI355X-native (gfx950) StableAvatar inference hot path: Wan-2.1 1.3B audio-driven DiT denoise
loop + 3-D causal VAE decode, as hand-written HIP kernels behind a C ABI
(include/stableavatar_hip.h), with drop-in Python modules mirroring the reference interfaces."""
__version__ = "0.1.0"
