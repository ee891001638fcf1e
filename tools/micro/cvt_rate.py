"""Issue cost of e4m3 -> bf16 conversions (tools/micro/cvt_rate.hip): cycles per loop iteration of 8 independent
chains, each a conversion + an integer multiply-add (mode 2: the chain without the conversion)."""
import ctypes, os, sys
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "cvt_rate.so"))
inp = torch.randint(0, 2**31, (64 * 8,), dtype=torch.int64).to(torch.int32).cuda()
out = torch.zeros(64, dtype=torch.int32).cuda()
clk = torch.zeros(256, dtype=torch.int64).cuda()
iters = 4096
for mode, name in ((2, "base"), (0, "cvt_scalef32_pk_bf16_fp8"), (1, "cvt_pk_f32_fp8+perm")):
    for _ in range(2):
        assert lib.run(mode, ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()), iters,
                       ctypes.c_void_p(clk.data_ptr()), 256) == 0
    c = clk.cpu().double().median().item() / iters
    print(f"{name}: {c:.1f} cycles per iteration (8 conversions)", flush=True)
