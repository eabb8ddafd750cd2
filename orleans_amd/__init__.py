"""orleans_amd -- MI355X-native batched grain-dispatch engine for Orleans.

The product is libgraindispatch.so (C ABI, include/graindispatch.h, gfx950 HIP
kernels).  `graindispatch` binds it with ctypes; `sharded` runs the multi-GPU
exchange over torch.distributed (RCCL on GPU, gloo in CPU tests).
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libgraindispatch.so")
