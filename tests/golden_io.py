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
