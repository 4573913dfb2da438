#!/usr/bin/env python3
"""VALU issue-rate probe (diag kinds 8-11): wave-instructions per SIMD per
cycle for v_add3_u32 / v_alignbit_b32 / v_add_u32 / v_fma_f32 at full
occupancy, with the in-kernel clock from s_memtime / s_memrealtime (100 MHz)."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
D.md5diag_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                          ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
waves = 256 * 32          # 32 waves per CU
iters = 20000
waves = int(sys.argv[1]) if len(sys.argv) > 1 else waves
buf = torch.zeros(64 * waves * 4 + 2 * waves * 8, dtype=torch.uint8, device="cuda")
res = {}
NAMES = ["v_add3_u32(v,v,v)", "v_alignbit_b32(imm)", "v_add_u32_e32", "v_fma_f32", "v_add_u32_e64",
         "v_add_u32_e32+literal", "v_bitop3_b32", "v_add3_u32(v,v,s)", "v_xor_b32_e32", "v_mov_b32",
         "v_bfi_b32", "v_lshl_add_u32", "v_lshl_add_u64", "v_alignbit_b32(s)", "v_xad_u32",
         "v_perm_b32", "v_add_u32_sdwa", "v_and_b32_e32", "v_lshlrev_b32_e32", "v_pk_add_u16"]
waves = int(sys.argv[1]) if len(sys.argv) > 1 else waves
for kind, name in [(100 + i, n) for i, n in enumerate(NAMES)]:
    for rep in range(3):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        assert D.md5diag_run(kind, None, waves, iters, 0, buf.data_ptr(), s.cuda_stream) == 0
        e1.record(s)
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    clk = buf[64 * waves * 4:].view(torch.int64).view(-1, 2).cpu()
    ticks, real = clk[:, 0].double(), clk[:, 1].double()
    ghz = float((ticks / real).median()) * 0.1
    inst = waves * iters * 8
    per_simd_cycle = inst / (1024 * ms * 1e-3 * ghz * 1e9)
    res[name] = {"ms": round(ms, 3), "clock_ghz": round(ghz, 3),
                 "wave_inst_per_simd_cycle": round(per_simd_cycle, 4),
                 "cycles_per_wave_inst": round(1 / per_simd_cycle, 3)}
print(json.dumps(res))
