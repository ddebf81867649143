import torch
for dev in ("cpu", "cuda"):
    for dt in (torch.bfloat16, torch.float16, torch.float32, torch.float64):
        v = torch.tensor([-0.0, 0.0, -0.0, -0.3, -1e-30], dtype=dt, device=dev)
        a = torch.clamp(v, 0, 15)
        b = torch.clamp(torch.round(v), 0, 15)
        c = torch.clamp(v, -8, 7)
        sb = lambda t: [str(float(u)) for u in t.cpu()]
        print(dev, dt, sb(a), sb(b), sb(c), sb(torch.clamp(v.repeat(8), 0, 15)[:3]))
