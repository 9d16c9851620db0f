"""Disparity warp of the refinement path (nets/warp.py).  `disp_warp` is one HIP kernel
(aanet_disp_warp_f32) instead of meshgrid + cat + normalise + two grid_sample calls + two
masked assignments; its autograd (to the disparity, and to the image when that requires grad)
is aanet_disp_warp_bwd_f32.  meshgrid / normalize_coords are kept for API parity (torch ops,
they are not on any hot path).
"""
import torch

from .. import ops


def normalize_coords(grid):
    """nets/warp.py:5-16: image-scale [B, 2, H, W] -> [-1, 1] grid [B, H, W, 2]."""
    assert grid.size(1) == 2
    h, w = grid.shape[2:]
    gx = 2 * (grid[:, 0] / (w - 1)) - 1
    gy = 2 * (grid[:, 1] / (h - 1)) - 1
    return torch.stack((gx, gy), dim=-1)


def meshgrid(img, homogeneous=False):
    """nets/warp.py:19-38: [B, 2(+1), H, W] pixel grid, grid[:, :, i, j] = (j, i[, 1])."""
    b, _, h, w = img.shape
    ys, xs = torch.meshgrid(torch.arange(h, device=img.device, dtype=img.dtype),
                            torch.arange(w, device=img.device, dtype=img.dtype), indexing="ij")
    planes = [xs, ys] + ([torch.ones_like(xs)] if homogeneous else [])
    return torch.stack(planes).unsqueeze(0).expand(b, len(planes), h, w)


def disp_warp(img, disp, padding_mode='border'):
    """nets/warp.py:41-64 -> (warped_img [B,C,H,W], valid_mask [B,C,H,W]).  img: [B,C,H,W],
    disp: [B,1,H,W] (non-negative in the reference, which asserts it with a host sync; the
    kernel warps any value and does not sync).  Only 'border' padding is used by AANet."""
    if padding_mode != 'border':
        raise NotImplementedError("disp_warp: only padding_mode='border' (nets/refinement.py)")
    img, disp = img.contiguous(), disp.contiguous()
    if torch.is_grad_enabled() and (img.requires_grad or disp.requires_grad):
        warped = ops.DispWarpFunction.apply(img, disp)
        with torch.no_grad():
            valid = ops.disp_warp(img, disp)[1]
        return warped, valid
    return ops.disp_warp(img, disp)
