"""The full AANet / AANet+ stereo model (nets/aanet.py): feature
extraction (+ FPN / pyramid), cost volume, aggregation, soft-argmin, hierarchical refinement.

Constructor arguments, module attributes (state-dict keys) and the forward's output pyramid
follow nets/aanet.py:14-229, so reference checkpoints load (aanet_amd.checkpoint) and the
training loss sees the same list.  Every stage runs the drop-in modules: HIP cost volumes,
adaptive aggregation, soft-argmin, DCN users in the feature extractors, the HIP disparity warp,
and (eval) the HIP conv engine for the 2-D convs.
"""
import torch.nn as nn
import torch.nn.functional as F

from .aggregation import AdaptiveAggregation
from .aggregation3d import (GCNetAggregation, PSMNetBasicAggregation, PSMNetHGAggregation,
                            StereoNetAggregation)
from .cost import CostVolume, CostVolumePyramid
from ._fuse import FoldCacheMixin
from .estimation import DisparityEstimation
from .options import get_option, set_options
from .feature import (FeaturePyramidNetwork, FeaturePyrmaid, GANetFeature, GCNetFeature,
                      PSMNetFeature, StereoNetFeature)
from .refinement import HourglassRefinement, StereoDRNetRefinement, StereoNetRefinement
from .resnet import AANetFeature
from .._precision import fp32_convs

_REFINEMENT = {'stereonet': StereoNetRefinement, 'stereodrnet': StereoDRNetRefinement,
               'hourglass': HourglassRefinement}


class AANet(FoldCacheMixin, nn.Module):
    def __init__(self, max_disp, useFeatureAtt=1, num_downsample=2, feature_type='aanet',
                 no_feature_mdconv=False, feature_pyramid=False, feature_pyramid_network=False,
                 feature_similarity='correlation', aggregation_type='adaptive', num_scales=3,
                 num_fusions=6, deformable_groups=2, mdconv_dilation=2,
                 refinement_type='stereodrnet', no_intermediate_supervision=False,
                 num_stage_blocks=1, num_deform_blocks=3):
        """nets/aanet.py:14-138.  `useFeatureAtt` is accepted and unused, as in the reference
        (whose inference.py omits it although it has no default there; it defaults here)."""
        super(AANet, self).__init__()
        self.refinement_type = refinement_type
        self.feature_type = feature_type
        self.feature_pyramid = feature_pyramid
        self.feature_pyramid_network = feature_pyramid_network
        self.num_downsample = num_downsample
        self.aggregation_type = aggregation_type
        self.num_scales = num_scales

        # feature extractor and the cost-volume disparity count (aanet.py:43-64)
        mdconv = not no_feature_mdconv
        if feature_type == 'stereonet':
            self.feature_extractor = StereoNetFeature(self.num_downsample)
            self.max_disp = max_disp // (2 ** num_downsample)
        elif feature_type == 'psmnet':
            self.feature_extractor = PSMNetFeature()
            self.max_disp = max_disp // (2 ** num_downsample)
        elif feature_type == 'gcnet':
            self.feature_extractor = GCNetFeature()
            self.max_disp = max_disp // 2
        elif feature_type == 'ganet':
            self.feature_extractor = GANetFeature(feature_mdconv=mdconv)
            self.max_disp = max_disp // 3
        elif feature_type == 'aanet':
            self.feature_extractor = AANetFeature(feature_mdconv=mdconv)
            self.max_disp = max_disp // 3
        else:
            raise NotImplementedError

        # multi-scale features (aanet.py:66-77)
        if feature_pyramid_network:
            in_channels = [32 * 4, 32 * 8, 32 * 16] if feature_type == 'aanet' else [32, 64, 128]
            self.fpn = FeaturePyramidNetwork(in_channels=in_channels, out_channels=32 * 4)
        elif feature_pyramid:
            self.fpn = FeaturePyrmaid()

        # cost volume (aanet.py:79-88)
        pyramid = feature_type == 'aanet' or feature_pyramid or feature_pyramid_network
        self.cost_volume = (CostVolumePyramid if pyramid else CostVolume)(
            self.max_disp, feature_similarity=feature_similarity)

        # aggregation (aanet.py:90-116)
        max_disp = self.max_disp
        in_channels = 64 if feature_similarity == 'concat' else 32
        if aggregation_type == 'adaptive':
            self.aggregation = AdaptiveAggregation(
                max_disp=max_disp, num_scales=num_scales, num_fusions=num_fusions,
                num_stage_blocks=num_stage_blocks, num_deform_blocks=num_deform_blocks,
                mdconv_dilation=mdconv_dilation, deformable_groups=deformable_groups,
                intermediate_supervision=not no_intermediate_supervision)
        elif aggregation_type == 'psmnet_basic':
            self.aggregation = PSMNetBasicAggregation(max_disp=max_disp)
        elif aggregation_type == 'psmnet_hourglass':
            self.aggregation = PSMNetHGAggregation(max_disp=max_disp)
        elif aggregation_type == 'gcnet':
            self.aggregation = GCNetAggregation()
        elif aggregation_type == 'stereonet':
            self.aggregation = StereoNetAggregation(in_channels=in_channels)
        else:
            raise NotImplementedError

        # soft-argmin (aanet.py:118-125): PSMNet upsamples the cost volume x4 and learns a
        # similarity for concatenation
        match_similarity = feature_similarity not in ['difference', 'concat']
        if 'psmnet' in self.aggregation_type:
            max_disp = self.max_disp * 4
            match_similarity = True
        self.disparity_estimation = DisparityEstimation(max_disp, match_similarity)

        # refinement (aanet.py:127-138)
        if self.refinement_type is not None and self.refinement_type != 'None':
            if self.refinement_type not in _REFINEMENT:
                raise NotImplementedError
            self.refinement = nn.ModuleList([_REFINEMENT[self.refinement_type]()
                                             for _ in range(num_downsample)])

    def set_options(self, **options):
        """Eval schedule options of the whole model (nets/options.py); returns self."""
        return set_options(self, **options)

    def feature_extraction(self, img):
        """aanet.py:140-144."""
        feature = self.feature_extractor(img)
        if self.feature_pyramid_network or self.feature_pyramid:
            feature = self.fpn(feature)
        return feature

    def cost_volume_construction(self, left_feature, right_feature):
        """aanet.py:146-154."""
        cost_volume = self.cost_volume(left_feature, right_feature)
        if isinstance(cost_volume, list):
            if self.num_scales == 1:
                cost_volume = [cost_volume[0]]  # ablation: 1 scale only
        elif self.aggregation_type == 'adaptive':
            cost_volume = [cost_volume]
        return cost_volume

    def disparity_computation(self, aggregation):
        """aanet.py:156-167: coarse-to-fine (the aggregation list is fine-to-coarse)."""
        if isinstance(aggregation, list):
            return [self.disparity_estimation(a) for a in reversed(aggregation)]
        return [self.disparity_estimation(aggregation)]

    def disparity_refinement(self, left_img, right_img, disparity):
        """aanet.py:169-209: refinement i runs at 1/2**(num_downsample-1-i) of the image."""
        pyramid = []
        if self.refinement_type is None or self.refinement_type == 'None':
            return pyramid
        for i in range(self.num_downsample):
            scale_factor = 1. / pow(2, self.num_downsample - i - 1)
            if scale_factor == 1.0:
                cur_left, cur_right = left_img, right_img
            else:
                cur_left = F.interpolate(left_img, scale_factor=scale_factor, mode='bilinear',
                                         align_corners=False)
                cur_right = F.interpolate(right_img, scale_factor=scale_factor, mode='bilinear',
                                          align_corners=False)
            disparity = self.refinement[i](disparity, cur_left, cur_right)
            pyramid.append(disparity)
        return pyramid

    @fp32_convs
    def forward(self, left_img, right_img):
        """aanet.py:211-229 -> disparity pyramid, coarse to fine (hot-path disparities, then
        one per refinement stage)."""
        left_feature = self.feature_extraction(left_img)
        right_feature = self.feature_extraction(right_img)
        cost_volume = self.cost_volume_construction(left_feature, right_feature)
        disp = None
        if isinstance(self.aggregation, AdaptiveAggregation):
            # eval, one output scale: final_conv + the soft-argmin may run in the last tail
            # kernel's epilogue (AdaptiveAggregation._run)
            regress = (not self.aggregation.intermediate_supervision and not self.training and
                       self.disparity_estimation.match_similarity)
            aggregation, disp = self.aggregation._run(
                cost_volume, regress=regress, chains=get_option(self.aggregation, "batch_chains"))
        else:
            aggregation = self.aggregation(cost_volume)
        disparity_pyramid = [disp] if disp is not None else self.disparity_computation(aggregation)
        disparity_pyramid += self.disparity_refinement(left_img, right_img, disparity_pyramid[-1])
        return disparity_pyramid
