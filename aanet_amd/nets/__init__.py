"""Drop-in replacements for the reference's hot-path modules (nets/cost.py, nets/estimation.py,
nets/aggregation.py [adaptive], nets/deform.py, nets/deform_conv/)."""
from .aggregation import AdaptiveAggregation, AdaptiveAggregationModule  # noqa: F401
from .cost import CostVolume, CostVolumePyramid  # noqa: F401
from .deform import DeformConv2d, DeformSimpleBottleneck, SimpleBottleneck  # noqa: F401
from .deform_conv import DeformConv, ModulatedDeformConv, modulated_deform_conv  # noqa: F401
from .estimation import DisparityEstimation  # noqa: F401
from .hotpath import AANetHotPath  # noqa: F401
