"""Loading helpers for the committed golden fixtures (data only, no pickles)."""
import functools
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_names(prefix):
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR) if f.startswith(prefix) and f.endswith(".npz"))


@functools.lru_cache(maxsize=None)
def golden(name):
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def state_dict_of(g):
    """Fixture keys 'param.<name>' -> {name: array} (reference state-dict keys)."""
    return {k[len("param."):]: v for k, v in g.items() if k.startswith("param.")}


def synthetic_value(name, shape, seed):
    """Deterministic value of one state-dict entry, keyed by its name (torch CPU generator).
    Shared by tests/golden/make_model_golden.py (filling the REFERENCE model) and the tests
    (filling ours): equal names + shapes => equal tensors, so the full-model fixtures need not
    carry megabytes of weights, and a name mismatch is a checkpoint-compatibility failure."""
    import zlib

    import torch
    g = torch.Generator().manual_seed((zlib.crc32(name.encode()) * 1000003 + seed) % (1 << 62))
    leaf = name.rsplit(".", 1)[-1]
    shape = tuple(shape)
    if leaf == "num_batches_tracked":
        return torch.zeros(shape, dtype=torch.long)
    if leaf == "running_mean":
        return 0.1 * torch.randn(shape, generator=g)
    if leaf == "running_var":
        return 0.5 + torch.rand(shape, generator=g)
    if leaf == "bias":
        return (0.5 if "offset_conv" in name else 0.1) * torch.randn(shape, generator=g)
    if len(shape) == 1:  # norm-layer gamma
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    fan_in = 1
    for s in shape[1:]:
        fan_in *= s
    return (2 * torch.rand(shape, generator=g) - 1) * (3.0 / fan_in) ** 0.5


def fill_synthetic(module, seed):
    """Overwrite every parameter and buffer of `module` with synthetic_value; returns the
    (name, shape) list in state-dict order."""
    import torch
    sd = module.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            v.copy_(synthetic_value(k, v.shape, seed).to(v.dtype))
    return [(k, tuple(v.shape)) for k, v in sd.items()]


def synthetic_pair(B, H, W, seed):
    """Seeded synthetic stereo pair for the full-model fixtures (torch CPU generator): right =
    left shifted 6 px left + noise, so the matching has a real answer."""
    import torch
    gm = torch.Generator().manual_seed(1000 + seed)
    left = torch.rand(B, 3, H, W, generator=gm) * 2 - 1
    right = torch.roll(left, shifts=-6, dims=3) + 0.05 * torch.randn(B, 3, H, W, generator=gm)
    return left, right
