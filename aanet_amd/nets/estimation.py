"""Drop-in for nets/estimation.py: fused soft-argmin on the gfx950 kernel."""
import torch.nn as nn

from ..ops import DisparityRegressionFunction


class DisparityEstimation(nn.Module):
    def __init__(self, max_disp, match_similarity=True):
        """nets/estimation.py:7-11."""
        super(DisparityEstimation, self).__init__()
        self.max_disp = max_disp
        self.match_similarity = match_similarity

    def forward(self, cost_volume):
        """nets/estimation.py:13-30: disparity candidates are arange(cost_volume.size(1))
        whether or not that equals max_disp (the reference's two branches agree)."""
        assert cost_volume.dim() == 4  # [B, D, H, W]
        return DisparityRegressionFunction.apply(cost_volume, not self.match_similarity)
