"""Refinement conv_start (DeformConv2d(32, 32), dilation 2) at full resolution, B=8: offset conv and DCN forward with NCHW vs channels-last input."""
import torch, sys
sys.path.insert(0, '.')
from aanet_amd import ops
dev='cuda'
def t(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); ts=[]
    for _ in range(n):
        s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e))
    ts.sort(); return ts[n//2]*1e3
N,C,H,W=8,32,384,1248
x=torch.randn(N,C,H,W,device=dev); xl=x.contiguous(memory_format=torch.channels_last)
wo=torch.randn(54,C,3,3,device=dev)*0.01; bo=torch.randn(54,device=dev)
w=torch.randn(C,C,3,3,device=dev)/17; wp=ops.pack_weight_split(w); wop=ops.pack_weight_split(wo)
om=ops.conv2d_fused(x,wo,bo,1,2,2,1,None,packed_weight=wop)
for name,xx in (('nchw',x),('nhwc',xl)):
    a=t(lambda: ops.conv2d_fused(xx,wo,bo,1,2,2,1,None,packed_weight=wop))
    b=t(lambda: ops.mdcn_forward_fused(xx,om,w,None,None,None,'relu',1,2,2,2,2.0,packed_weight=wp))
    print(name,'offset conv %.1f us  dcn %.1f us'%(a,b))
