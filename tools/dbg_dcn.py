import sys, numpy as np, torch
sys.path.insert(0, '.')
from aanet_amd import ops
from oracle import oracle
rng = np.random.default_rng(0)
N, C, H, W, Co, dg = 2, 64, 16, 52, 64, 2
x = rng.standard_normal((N, C, H, W)).astype(np.float32)
off = (rng.standard_normal((N, dg * 18, H, W)) * 2).astype(np.float32)
msk = rng.uniform(0, 1, (N, dg * 9, H, W)).astype(np.float32)
w = (rng.standard_normal((Co, C, 3, 3)) / 24).astype(np.float32)
ref = oracle.mdcn_forward(x, off, msk, w, None, 1, 2, 2, 1, dg)
d = lambda a: torch.from_numpy(a).cuda()
got = ops.mdcn_forward(d(x), d(off), d(msk), d(w), None, 1, 2, 2, 1, dg).cpu().numpy()
err = np.abs(got - ref)
print('max err', err.max())
bad = err.max(axis=1)  # N,H,W
p = np.arange(H * W)
for n in range(N):
    b = bad[n].reshape(-1) > 1e-3
    print('n', n, 'bad px', b.sum(), 'of', b.size)
    print(' bad px mod 64 hist', np.bincount((p[b] % 64), minlength=64))
    print(' first bad', p[b][:20])
# zero offsets -> compare
