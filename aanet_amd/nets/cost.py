"""Drop-in for nets/cost.py: CostVolume / CostVolumePyramid on the gfx950 kernels.

Same constructor signatures, defaults, forward arity and return types as the reference
(nets/cost.py:5-76).  All three similarity measures run as HIP kernels through the C ABI
(aanet_corr_volume_f32 / aanet_concat_volume_f32 / aanet_diff_volume_f32), with autograd.
"""
import torch.nn as nn

from ..ops import CorrelationPyramidFunction, CorrelationVolumeFunction, ShiftVolumeFunction


class CostVolume(nn.Module):
    def __init__(self, max_disp, feature_similarity='correlation'):
        """nets/cost.py:6-17."""
        super(CostVolume, self).__init__()
        self.max_disp = max_disp
        self.feature_similarity = feature_similarity

    def forward(self, left_feature, right_feature):
        """nets/cost.py:19-55: [B,D,H,W] (correlation) or [B,C',D,H,W] (concat / difference)."""
        if self.feature_similarity == 'correlation':
            return CorrelationVolumeFunction.apply(left_feature, right_feature, self.max_disp)
        if self.feature_similarity == 'concat':
            return ShiftVolumeFunction.apply(left_feature, right_feature, self.max_disp, True)
        if self.feature_similarity == 'difference':
            return ShiftVolumeFunction.apply(left_feature, right_feature, self.max_disp, False)
        raise NotImplementedError


class CostVolumePyramid(nn.Module):
    def __init__(self, max_disp, feature_similarity='correlation'):
        """nets/cost.py:58-62."""
        super(CostVolumePyramid, self).__init__()
        self.max_disp = max_disp
        self.feature_similarity = feature_similarity

    def forward(self, left_feature_pyramid, right_feature_pyramid):
        """nets/cost.py:64-76: scale s uses max_disp // 2**s; returns [H/3, H/6, H/12].
        Correlation: all scales in one launch (aanet_corr_pyramid_f32)."""
        num_scales = len(left_feature_pyramid)
        if self.feature_similarity == 'correlation' and num_scales > 0:
            return list(CorrelationPyramidFunction.apply(
                self.max_disp, num_scales, *left_feature_pyramid, *right_feature_pyramid))
        cost_volume_pyramid = []
        for s in range(num_scales):
            max_disp = self.max_disp // (2 ** s)
            cost_volume_pyramid.append(CostVolume(max_disp, self.feature_similarity)(
                left_feature_pyramid[s], right_feature_pyramid[s]))
        return cost_volume_pyramid
