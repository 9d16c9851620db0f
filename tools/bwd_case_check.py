import sys, numpy as np, torch
sys.path.insert(0, '.')
from aanet_amd import ops
from oracle import oracle
from tests.test_gpu_mdcn import make_case, BWD_CASES
for ci in range(len(BWD_CASES)):
    N, C, H, W, Co, k, s, p, d, dg = BWD_CASES[ci]
    x, off, msk, w, b = make_case(5, N, C, H, W, Co, k, s, p, d, dg, off_scale=0.7)
    Ho, Wo = off.shape[2:]
    go = np.random.default_rng(6).standard_normal((N, Co, Ho, Wo)).astype(np.float32)
    ref = oracle.mdcn_backward(x, off, msk, w, go, True, s, p, d, 1, dg)
    g = lambda a: torch.from_numpy(a).cuda()
    for det in (False, True):
        got = ops.mdcn_backward(g(x), g(off), g(msk), g(w), g(go), True, s, p, d, 1, dg, deterministic=det)
        errs = [float(np.abs(t.cpu().numpy() - r).max() / (np.abs(r).max() + 1e-12)) for t, r in zip(got, ref)]
        print(ci, BWD_CASES[ci][:5], 'det' if det else 'atomic', ['%.1e' % e for e in errs], flush=True)
