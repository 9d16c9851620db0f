"""Drop-in replacements for the reference's modules: the hot path (nets/cost.py,
nets/estimation.py, nets/aggregation.py, nets/deform.py, nets/deform_conv/) and, around it, the
feature extractors, refinement, warp, 3-D aggregators and the full AANet model."""
from .aanet import AANet  # noqa: F401
from .aggregation import AdaptiveAggregation, AdaptiveAggregationModule  # noqa: F401
from .aggregation3d import (GCNetAggregation, PSMNetBasicAggregation,  # noqa: F401
                            PSMNetHGAggregation, PSMNetHourglass, StereoNetAggregation)
from .cost import CostVolume, CostVolumePyramid  # noqa: F401
from .deform import (DeformBottleneck, DeformConv2d, DeformSimpleBottleneck,  # noqa: F401
                     SimpleBottleneck)
from .deform_conv import DeformConv, ModulatedDeformConv, modulated_deform_conv  # noqa: F401
from .estimation import DisparityEstimation  # noqa: F401
from .feature import (BasicConv, Conv2x, FeaturePyramidNetwork, FeaturePyrmaid,  # noqa: F401
                      GANetFeature, GCNetFeature, PSMNetFeature, StereoNetFeature)
from .hotpath import AANetHotPath  # noqa: F401
from .options import set_options  # noqa: F401
from .refinement import HourglassRefinement, StereoDRNetRefinement, StereoNetRefinement  # noqa: F401
from .resnet import AANetFeature  # noqa: F401
from .warp import disp_warp  # noqa: F401
