"""Diagnostic: hot-path disparity (pair 0 of the bench workload) against the CPU oracle (fp32):
max/mean |d| and where the max sits.  Contraction mode from the environment
(AANET_EXACT_F32=1, AANET_NO_HALO=1); saves gpurun_out/diag_<tag>.npy."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from oracle import aggregation as oagg  # noqa: E402

tag = sys.argv[1]
dev = torch.device("cuda", 0)
model = bench.build_model(dev)
left, right = bench.make_features(int(os.environ.get("DIAG_B", "8")), 0, dev)
sd = {k: v.detach().cpu().numpy() for k, v in model.aggregation.state_dict().items()}
lp = [t[:1].cpu().numpy() for t in left]
rp = [t[:1].cpu().numpy() for t in right]
ref = oagg.hot_path(lp, rp, sd, bench.MAXD, intermediate_supervision=False)[0][0].astype(np.float64)
with torch.no_grad():
    d = model(left, right)[0][0].cpu().numpy().astype(np.float64)
np.save(f"gpurun_out/diag_{tag}.npy", d)
np.save("gpurun_out/diag_ref.npy", ref)
e = np.abs(d - ref)
i = np.unravel_index(np.argmax(e), e.shape)
print(f"{tag:11s} max {e.max():.3e} at {i} (ref {ref[i]:.4f} got {d[i]:.4f}) mean {e.mean():.3e} "
      f"p99.99 {np.quantile(e, 0.9999):.3e}  n>1e-4 {(e > 1e-4).sum()}  n>3e-4 {(e > 3e-4).sum()}")
