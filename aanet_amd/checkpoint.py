"""Checkpoint save / load compatible with the reference's .pth files (utils/utils.py:50-143;
SURVEY.md §8f row f2).

A reference AANet checkpoint is `{'epoch', 'num_iter', 'epe', 'best_epe', 'best_epoch',
'state_dict'}` (or a bare state dict).  Our modules keep the reference's attribute names, so the
state dict loads into aanet_amd.nets.AANet unchanged.  Loading uses torch.load(weights_only=True):
tensors and plain containers only, nothing executed from the file.

The reference loader does not strip the `module.` prefix that DistributedDataParallel adds to
every key (the stripping code is commented out, utils.py:108-110): with no_strict=True a DDP
checkpoint then loads NOTHING and only prints the missing keys.  That is the default here too;
`strip_module_prefix=True` removes the prefix when the target module does not carry it.
"""
import os
from collections import OrderedDict
from glob import glob

import torch

_META = ("epoch", "num_iter", "best_epe", "best_epoch")


def _strip_module(weights, net):
    if any(k.startswith("module.") for k in net.state_dict()):
        return weights
    return OrderedDict((k[len("module."):] if k.startswith("module.") else k, v)
                       for k, v in weights.items())


def load_pretrained_net(net, pretrained_path, return_epoch_iter=False, resume=False,
                        no_strict=False, strip_module_prefix=False, verbose=True):
    """utils.py:88-130.  Returns (epoch, num_iter, best_epe, best_epoch) when return_epoch_iter
    (None for absent fields), else (missing_keys, unexpected_keys).  `resume` is accepted for
    signature parity (the reference only used it in its commented-out prefix stripping)."""
    if pretrained_path is None:
        return (None,) * 4 if return_epoch_iter else ([], [])
    device = "cuda" if torch.cuda.is_available() else "cpu"
    state = torch.load(pretrained_path, map_location=device, weights_only=True)
    weights = state["state_dict"] if "state_dict" in state else state
    if strip_module_prefix:
        weights = _strip_module(weights, net)
    missing, unexpected = net.load_state_dict(weights, strict=not no_strict)
    if verbose:
        print(f"missing_keys:{missing}")
        print(f"unexpected_keys:{unexpected}")
    if return_epoch_iter:
        return tuple(state.get(k) for k in _META)
    return missing, unexpected


def save_checkpoint(save_path, optimizer, aanet, epoch, num_iter, epe, best_epe, best_epoch,
                    filename=None, save_optimizer=True):
    """utils.py:50-85: aanet_epoch_XXX.pth (+ optimizer_epoch_XXX.pth)."""
    os.makedirs(save_path, exist_ok=True)
    meta = {"epoch": epoch, "num_iter": num_iter, "epe": epe, "best_epe": best_epe,
            "best_epoch": best_epoch}
    name = "aanet_epoch_{:0>3d}.pth".format(epoch) if filename is None else filename
    torch.save(dict(meta, state_dict=aanet.state_dict()), os.path.join(save_path, name))
    if save_optimizer:
        torch.save(dict(meta, state_dict=optimizer.state_dict()),
                   os.path.join(save_path, name.replace("aanet", "optimizer")))


def resume_latest_ckpt(checkpoint_dir, net, net_name):
    """utils.py:133-143."""
    ckpts = sorted(glob(os.path.join(checkpoint_dir, net_name + "*.pth")))
    if not ckpts:
        raise RuntimeError("=> No checkpoint found while resuming training")
    return load_pretrained_net(net, ckpts[-1], True, True)
