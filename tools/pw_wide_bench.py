import sys, torch
sys.path.insert(0, '.')
from aanet_amd import ops
dev = 'cuda'
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
for C, Co, H, W in [(32, 128, 128, 416), (64, 256, 64, 208), (64, 128, 64, 208), (128, 512, 32, 104)]:
    x = torch.randn(8, C, H, W, device=dev)
    w = torch.randn(Co, C, 1, 1, device=dev) * 0.1
    b = torch.randn(Co, device=dev)
    ws = ops.pack_weight_split(w); wp = ops.pack_weight(w)
    r = torch.randn(8, Co, H, W, device=dev)
    a = t(lambda: ops.conv2d_fused(x, w, b, act='relu', packed_weight=ws))
    bb = t(lambda: ops.conv2d_fused(x, w, b, act='relu', packed_weight=wp))
    c = t(lambda: ops.conv2d_fused(x, w, b, act='relu', residual=r, packed_weight=ws))
    by = 4 * 8 * H * W * (C + Co)
    print(f"{C}->{Co} {H}x{W}: split(pw if C<=64) {a:7.1f} us ({by/a/1e3:5.2f} TB/s)  engine-f32 {bb:7.1f} us  +residual {c:7.1f}", flush=True)
