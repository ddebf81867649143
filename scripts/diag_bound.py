"""Diagnose RTN-bound violations of the fast kernel on a large tensor (GPU)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "awq-converter_amd")]
import torch
from awq_quantizer.quantization import AWQQuantizer
from oracle import awq_oracle as orc

shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "14336x4096").split("x"))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
x = (torch.randn(*shape, generator=g, device=dev) * 0.02).to(torch.bfloat16)
q = AWQQuantizer(bits=4, symmetric=False, device="cuda", logger_level="ERROR")
pk = q.quantize_packed(x)
dq = q.dequantize_packed(pk)
s = pk["scales"].float().repeat_interleave(128, dim=1)
ratio = ((dq - x.float()).abs() / s)
print("max err/s", ratio.max().item(), "count>0.6", int((ratio > 0.6).sum()))
bad = (ratio > 0.6).nonzero()[:5]
rows = sorted(set(bad[:, 0].tolist()))[:4] + [0, shape[0] - 1]
for r in rows:
    xr = x[r:r + 1].cpu()
    ref = orc.quantize(xr, bits=4, group_size=128, symmetric=False)
    okq = torch.equal(pk["qweight"][r:r + 1].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0))
    oks = torch.equal(pk["scales"][r:r + 1].cpu(), ref["scales"])
    okz = torch.equal(pk["qzeros"][r:r + 1].cpu(), orc.pack_rows(ref["zero_points"], 4, 0))
    print("row", r, "qweight ok", okq, "scales ok", oks, "qzeros ok", okz)
for r, k in bad.tolist()[:3]:
    gi = k // 128
    xs = x[r, gi * 128:(gi + 1) * 128].float()
    print("r", r, "k", k, "x", x[r, k].item(), "dq", dq[r, k].item(), "s", s[r, k].item(),
          "grp min/max", xs.min().item(), xs.max().item())
# full tensor vs oracle (C oracle ~ 1-2 s per 50M elements)
ref = orc.quantize(x.cpu(), bits=4, group_size=128, symmetric=False)
print("full qweight equal:", torch.equal(pk["qweight"].cpu(), orc.pack_rows(ref["tensor_q"], 4, 0)))
print("full scales equal:", torch.equal(pk["scales"].cpu(), ref["scales"]))
print("full qzeros equal:", torch.equal(pk["qzeros"].cpu(), orc.pack_rows(ref["zero_points"], 4, 0)))
dqo = orc.dequantize(ref)
r2 = ((dqo - x.float().cpu()).abs() / s.cpu())
print("oracle max err/s", r2.max().item())
