"""Scale-1 offset conv (32 -> 54, 3x3, dil 2, 2 groups, C2 B=8 64x208, channels-last) in eval:
grouped exact-f32 engine vs the block-diagonal split-bf16 form (nets/_fuse.py dense_grouped_ok)."""
import os, sys, torch, torch.nn as nn
sys.path.insert(0, os.getcwd())
from aanet_amd.nets._fuse import conv_bn_act
from aanet_amd.nets.options import set_options
conv = nn.Conv2d(32, 54, 3, padding=2, dilation=2, groups=2).cuda().eval()
x = torch.randn(8, 32, 64, 208, device="cuda").relu_().contiguous(memory_format=torch.channels_last)
with torch.no_grad():
    for mode in ["0", "1", "0", "1"]:
        set_options(conv, dense_grouped=mode == "1")
        for _ in range(3): conv_bn_act(x, conv)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50): conv_bn_act(x, conv)
        e.record(); torch.cuda.synchronize()
        print("dense" if mode == "1" else "grouped", round(s.elapsed_time(e) / 50 * 1e3, 1), "us")
