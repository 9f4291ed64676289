"""HIP kernel bindings (ctypes) and weight packing for the gfx950 kernels in csrc/kernels."""
