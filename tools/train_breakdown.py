"""Per-step kernel-time breakdown of a rocprofv3 trace of `bench.py --train` (7 steps traced)."""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4   # last `steps` complete steps
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# step boundaries: the last optimizer (multi_tensor_apply) kernel of each burst
opt = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
ends = [i for j, i in enumerate(opt) if j + 1 == len(opt) or opt[j + 1] > i + 40]
rows = rows[ends[-steps - 1] + 1: ends[-1] + 1]
agg = collections.defaultdict(lambda: [0, 0.0])


def short(n):
    for k in ("direct_copy", "sigmoid", "smooth_l1", "FillFunctor", "CUDAFunctor_add", "im2col",
              "col2im", "upsample_bilinear2d_backward", "upsample_bilinear2d", "BatchNormBwd",
              "BatchNormFwdTrain", "batched_transpose", "Cijk", "igemm_wrw", "igemm_bwd",
              "igemm_fwd", "miopenSp3AsmConv", "mdcn_bwd_data", "mdcn_bwd_weight", "conv_fwd_kernel",
              "corr_volume", "disp_regress", "rocblas_gemv", "copyBuffer", "softmax", "index",
              "reduce_kernel", "adam", "Adam", "threshold", "mul", "add"):
        if k in n:
            return k
    return n[:70]


tot = 0.0
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    a = agg[short(r["Kernel_Name"])]
    a[0] += 1
    a[1] += d
    tot += d
print(f"total {tot / steps:.3f} ms/step over {steps} steps")
for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{d / steps:8.3f} ms {c / steps:7.1f} calls  {k}")
