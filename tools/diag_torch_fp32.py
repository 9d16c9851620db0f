"""How accurate are PyTorch-ROCm's own fp32 conv / matmul on this box (the ops the reference-order
model path leaves to torch)?  Relative error vs float64 of F.conv2d (MIOpen and, with cudnn
disabled, the native im2col + GEMM path) and torch.matmul, under the default and explicit
precision settings.  Usage: python tools/diag_torch_fp32.py"""
import torch
import torch.nn.functional as F

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(2, 64, 48, 96, device=dev, generator=g)
w = torch.randn(64, 64, 3, 3, device=dev, generator=g) / 24
a = torch.randn(512, 2048, device=dev, generator=g)
b = torch.randn(2048, 512, device=dev, generator=g)


def rel(t, r):
    return float((t.double() - r).abs().max() / r.abs().max())


ref_c = F.conv2d(x.double(), w.double(), padding=1)
ref_m = a.double() @ b.double()
print("matmul.allow_tf32", torch.backends.cuda.matmul.allow_tf32, "cudnn.allow_tf32", torch.backends.cudnn.allow_tf32,
      "fp32_precision", getattr(torch.backends.cuda.matmul, "fp32_precision", None), flush=True)
for cud in (True, False):
    for tf in (False, True):
        with torch.backends.cudnn.flags(enabled=cud, allow_tf32=tf):
            torch.backends.cuda.matmul.allow_tf32 = tf
            c = F.conv2d(x, w, padding=1)
            m = a @ b
        print(f"cudnn={cud} allow_tf32={tf}: conv rel err {rel(c, ref_c):.2e}  matmul rel err {rel(m, ref_m):.2e}", flush=True)
torch.backends.cuda.matmul.allow_tf32 = False
