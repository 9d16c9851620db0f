import sys, torch
sys.path.insert(0, '.')
import bench
from torch.profiler import profile, ProfilerActivity
dev = torch.device('cuda', 0)
m = bench.build_model(dev)
l, r = bench.make_features(8, 0, dev)
with torch.no_grad():
    for _ in range(3): m(l, r)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    with torch.no_grad():
        m(l, r)
    torch.cuda.synchronize()
evs = [e for e in prof.events() if 'copy' in e.name.lower() or 'Memcpy' in e.name]
from collections import Counter
print(Counter(e.name for e in evs).most_common(10))
for e in prof.events():
    if e.name in ('aten::copy_', 'aten::contiguous', 'aten::clone', 'aten::cat'):
        st = [s for s in (e.stack or []) if 'aanet_amd' in s or 'bench' in s][:3]
        print(e.name, e.input_shapes[:1] if e.input_shapes else '', st)
