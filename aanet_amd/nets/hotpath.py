"""The north-star path as one module: the part of AANet.forward between feature extraction and
refinement (nets/aanet.py:216-219), built from the drop-in modules.

  cost_volume_construction  nets/aanet.py:146-154
  aggregation               nets/aanet.py:93-101, 217 (adaptive only)
  disparity_computation     nets/aanet.py:156-167 (regresses in reverse scale order)

Attribute names (cost_volume, aggregation, disparity_estimation) match AANet's, so an AANet
state dict's `aggregation.*` keys load into this module unchanged.
"""
import torch.nn as nn

from .aggregation import AdaptiveAggregation
from .cost import CostVolume, CostVolumePyramid
from ._fuse import FoldCacheMixin
from .estimation import DisparityEstimation
from .options import get_option, set_options
from .._precision import fp32_convs


class AANetHotPath(FoldCacheMixin, nn.Module):
    def __init__(self, max_disp, feature_similarity='correlation', num_scales=3, num_fusions=6,
                 deformable_groups=2, mdconv_dilation=2, no_intermediate_supervision=False,
                 num_stage_blocks=1, num_deform_blocks=3, pyramid=True):
        """max_disp is the cost-volume disparity count (AANet's self.max_disp, i.e. the CLI
        --max_disp // 3 for the aanet feature extractor, nets/aanet.py:56-59)."""
        super().__init__()
        self.max_disp = max_disp
        self.num_scales = num_scales
        self.aggregation_type = 'adaptive'
        cost_cls = CostVolumePyramid if pyramid else CostVolume
        self.cost_volume = cost_cls(max_disp, feature_similarity=feature_similarity)
        self.aggregation = AdaptiveAggregation(max_disp=max_disp, num_scales=num_scales,
                                               num_fusions=num_fusions,
                                               num_stage_blocks=num_stage_blocks,
                                               num_deform_blocks=num_deform_blocks,
                                               mdconv_dilation=mdconv_dilation,
                                               deformable_groups=deformable_groups,
                                               intermediate_supervision=not no_intermediate_supervision)
        match_similarity = feature_similarity not in ['difference', 'concat']
        self.disparity_estimation = DisparityEstimation(max_disp, match_similarity)

    def set_options(self, **options):
        """Eval schedule options of the path (nets/options.py); returns self."""
        return set_options(self, **options)

    def cost_volume_construction(self, left_feature, right_feature):
        cost_volume = self.cost_volume(left_feature, right_feature)
        if isinstance(cost_volume, list):
            if self.num_scales == 1:
                cost_volume = [cost_volume[0]]  # ablation purpose for 1 scale only
        elif self.aggregation_type == 'adaptive':
            cost_volume = [cost_volume]
        return cost_volume

    def disparity_computation(self, aggregation):
        if isinstance(aggregation, list):
            disparity_pyramid = []
            length = len(aggregation)
            for i in range(length):
                disparity_pyramid.append(self.disparity_estimation(aggregation[length - 1 - i]))
            return disparity_pyramid
        return [self.disparity_estimation(aggregation)]

    @fp32_convs
    def forward(self, left_feature, right_feature):
        cost_volume = self.cost_volume_construction(left_feature, right_feature)
        aggregation, disp = self.aggregation._run(
            cost_volume, regress=self.regress_in_tail(),
            chains=get_option(self.aggregation, "batch_chains"))
        if disp is not None:  # final_conv + soft-argmin ran in the last tail kernel's epilogue
            return [disp]
        return self.disparity_computation(aggregation)

    def regress_in_tail(self):
        """Whether the last aggregation tail kernel may also run final_conv + the regression
        (eval; one output scale; the similarity soft-argmin of nets/estimation.py:13-30)."""
        return (not self.aggregation.intermediate_supervision and
                self.disparity_estimation.match_similarity and not self.training)
