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
                            ctypes.c_longlong, ctypes.c_void_p]
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    grid = 256
    # source: 1 MiB re-read by everyone (L2), 128 MiB streamed (Infinity Cache), 4 GiB streamed (HBM)
    for where, span in (("L2", 0), ("MALL", 128 << 20), ("HBM", 4 << 30)):
        src = torch.randint(0, 255, (max(span, 1 << 20),), dtype=torch.uint8, device="cuda")
        base_iters = 2000 if span == 0 else max(1, span // (2048 * 1024 * 16)) * 8
        for mode, name in ((0, "ldsdma"), (1, "vgpr"), (2, "half_each")):
            for depth in (8, 16, 32):
                iters = base_iters * 8 // depth  # the same bytes per wave at every depth
                if mode == 2 and depth == 32:
                    continue
                st = torch.cuda.current_stream().cuda_stream
                for _ in range(2):
                    assert L.run_probe(mode, depth, src.data_ptr(), grid, iters, sink.data_ptr(), span, st) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert L.run_probe(mode, depth, src.data_ptr(), grid, iters, sink.data_ptr(), span, st) == 0
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3
                per_cu = 8 * depth * 1024 * iters / us / 1e3  # GB/s per workgroup (= per CU)
                print(json.dumps({"source": where, "mode": name, "depth": depth, "us": round(us, 1),
                                  "GBps_per_CU": round(per_cu, 1), "chip_TBps": round(per_cu * grid / 1e3, 2)}),
                      flush=True)
        del src
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
