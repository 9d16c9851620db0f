"""Inference front-end of the reference (inference.py:85-206, dataloader/transforms.py:19-56):
image normalisation, top/right padding to the network size, the last disparity of the pyramid,
upsampling to the padded size, cropping back, and saving as png / pfm / npy.
"""
import os

import numpy as np
import torch
import torch.nn.functional as F

from . import io

IMAGENET_MEAN = [0.485, 0.456, 0.406]   # inference.py:17-18
IMAGENET_STD = [0.229, 0.224, 0.225]


def to_network_input(img, device=None):
    """transforms.ToTensor + Normalize: [H, W, 3] in [0, 255] -> [1, 3, H, W] ImageNet-normalised."""
    t = torch.from_numpy(np.ascontiguousarray(np.transpose(img, (2, 0, 1)))).float() / 255.
    mean = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(3, 1, 1)
    t = ((t - mean) / std).unsqueeze(0)
    return t if device is None else t.to(device)


def pad_pair(left, right, img_height, img_width):
    """inference.py:154-163: zero-pad top and right up to (img_height, img_width) when smaller;
    -> (left, right, top_pad, right_pad)."""
    h, w = left.shape[2:]
    if h < img_height or w < img_width:
        top_pad, right_pad = img_height - h, img_width - w
        left = F.pad(left, (0, right_pad, top_pad, 0))
        right = F.pad(right, (0, right_pad, top_pad, 0))
        return left, right, top_pad, right_pad
    return left, right, 0, 0


@torch.no_grad()
def predict(model, left, right, img_height, img_width):
    """inference.py:150-188 -> [B, H, W] disparity at the input size."""
    ori_h, ori_w = left.shape[2:]
    left, right, top_pad, right_pad = pad_pair(left, right, img_height, img_width)
    pred = model(left, right)[-1]
    if pred.size(-1) < left.size(-1):
        pred = F.interpolate(pred.unsqueeze(1), (left.size(-2), left.size(-1)), mode='bilinear',
                             align_corners=False) * (left.size(-1) / pred.size(-1))
        pred = pred.squeeze(1)
    if ori_h < img_height or ori_w < img_width:
        pred = pred[:, top_pad:, :-right_pad] if right_pad != 0 else pred[:, top_pad:]
    return pred


def save_disparity(disp, save_name, save_type='png', visualize=False):
    """inference.py:190-204: png = KITTI uint16 x256 (default); pfm (+ a png when visualize);
    npy.  Returns the written path."""
    disp = np.asarray(disp, np.float32)
    os.makedirs(os.path.dirname(save_name) or '.', exist_ok=True)
    if save_type == 'pfm':
        if visualize:
            io.write_kitti_disp(save_name, disp)
        save_name = save_name[:-3] + 'pfm'
        io.write_pfm(save_name, disp)
    elif save_type == 'npy':
        save_name = save_name[:-3] + 'npy'
        np.save(save_name, disp)
    else:
        io.write_kitti_disp(save_name, disp)
    return save_name
