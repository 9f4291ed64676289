#!/usr/bin/env python3
"""Per-CU operand load throughput: LDS-DMA vs VGPR loads vs both (scripts/probes/load_path_probe.hip).
    python scripts/load_path_probe.py --build   (CPU host)
    python scripts/load_path_probe.py           (GPU: one JSON line per (mode, depth))"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_load_probe.so")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                               os.path.join(ROOT, "scripts", "probes", "load_path_probe.hip"), "-o", SO])
        print("built", SO)
        return
    import torch
    L = ctypes.CDLL(SO)
    L.run_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                            ctypes.c_void_p]
    src = torch.randint(0, 255, (1 << 20,), dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    grid, iters = 256, 2000
    for mode, name in ((0, "ldsdma"), (1, "vgpr"), (2, "half_each")):
        for depth in (8, 16):
            st = torch.cuda.current_stream().cuda_stream
            for _ in range(2):
                assert L.run_probe(mode, depth, src.data_ptr(), grid, 50, sink.data_ptr(), st) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert L.run_probe(mode, depth, src.data_ptr(), grid, iters, sink.data_ptr(), st) == 0
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3
            per_cu = 8 * depth * 1024 * iters / us / 1e3  # GB/s per workgroup (= per CU)
            print(json.dumps({"mode": name, "depth": depth, "us": round(us, 1), "GBps_per_CU": round(per_cu, 1),
                              "chip_TBps": round(per_cu * grid / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
