"""torch's GPU conversions the reference meets with device="cuda" (awq.py:329/367 float -> int32
tensor_q on the device; awq.py:211 zero point clamp): NaN / inf / out-of-range float -> int32 on
the GPU and on the CPU, and clamp(-0.0) in the zero-point expression.  Diagnostics only."""
import torch
v = torch.tensor([float("nan"), -float("nan"), float("inf"), -float("inf"), 3e9, -3e9, -0.0, 2.5], dtype=torch.float32)
for dev in ("cpu", "cuda"):
    t = torch.zeros(8, dtype=torch.int32, device=dev)
    t[:] = v.to(dev)
    print(dev, "setitem f32->i32", t.cpu().tolist(), "to(int32)", v.to(dev).to(torch.int32).cpu().tolist())
    for dt in (torch.bfloat16, torch.float16, torch.float64):
        t[:] = v.to(dt).to(dev)
        print(dev, dt, "setitem", t.cpu().tolist())
    g = torch.tensor([0.1, 0.5, 1.0], device=dev)
    s = (g.max() - g.min()) / 15
    zp = (0 - g.min() / s).round().clamp(0, 15)
    print(dev, "zp bits", zp.view(torch.int32).item(), "scale", s.item())
