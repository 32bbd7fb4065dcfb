"""Drives scripts/valu_bench.hip: VALU wave-instructions per clock per SIMD, per opcode.
    python scripts/valu_bench.py build | run     (clock from rocprofv3 GRBM_GUI_ACTIVE when profiled)"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "scripts", "_build", "libvalu_bench.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    os.path.join(ROOT, "scripts", "valu_bench.hip"), "-o", SO], check=True)


def run():
    import torch
    lib = C.CDLL(SO)
    lib.valu_bench_run.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(ncu * 1024, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    iters = 2048
    for op, name in enumerate(("v_xor_b32", "v_bitop3_b32", "v_perm_b32", "v_alignbit_b32", "v_xor_b32_dpp")):
        ts = []
        for rep in range(4):
            ev[0].record()
            assert lib.valu_bench_run(op, iters, ncu, 1024, out.data_ptr(), s) == 0
            ev[1].record()
            torch.cuda.synchronize()
            if rep:
                ts.append(ev[0].elapsed_time(ev[1]))
        ms = sorted(ts)[1]
        inst_per_simd = iters * 64 * 8 * 4  # 16 waves / 4 SIMDs = 4 waves per SIMD
        print(f"{name:16s} {ms:7.3f} ms  {inst_per_simd / (ms * 1e-3) / 1e9:.3f} G wave-instr/s per SIMD "
              f"(= {inst_per_simd / (ms * 1e-3) / 2.4e9:.2f} per clk at 2.4 GHz)", flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
