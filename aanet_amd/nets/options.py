"""Schedule options of the eval fast path, set explicitly per module tree.

The reference's modules are configured by their constructors alone (nets/aggregation.py:406-412);
the drop-ins keep those constructors unchanged and take the few MI355X schedule choices as
module attributes set by `set_options` (INTEGRATION.md level 2).  Nothing here reads the process
environment: two models in one process can run different schedules, and every option the tests
exercise is passed to the module under test.

Every option changes only the kernel schedule of the eval fast path; the result is the same
computation (bit-identical, or for `concurrent_scales` / `s2_sums` / `dense_grouped` within fp32
summation order; tests/test_gpu_production.py, test_gpu_post.py, test_gpu_dense_grouped.py).

  concurrent_scales  True: the coarse scales run on side HIP streams beside the scale-0 chain;
                     False: one stream.                              (AdaptiveAggregation)
  post_fusion        "all": the tail kernels also run the next module's conv1 and the last
                     module's final_conv + soft-argmin; "final": only the last one; "none".
                                                                      (AdaptiveAggregation)
  s2_sums            True: output branches 1 and 2 are summed in the stride-2 kernels'
                     epilogues; False: separate aanet_csa_sum_f32 kernels.
                                                                      (AdaptiveAggregationModule)
  prep_stream        True: a deformable scale-0 block's conv1 + offset conv run on a side stream
                     as soon as x[0] exists, beside the previous module's stride-2 heads;
                     False (default): on the current stream after the heads.  Measured round 6:
                     3.27 vs 3.22-3.23 ms (the heads slow down more than the prep gains;
                     bit-identical either way).                       (AdaptiveAggregationModule)
  batch_chains       k >= 1: the whole-model forwards (AANetHotPath, AANet) split the batch into
                     k chunks, each aggregated on its own stream (batch pipelining: one chunk's
                     small serial kernels beside another's large ones); 1: one chain.
                     Bit-identical results.  Measured round 6 (HIP graph): k = 2 / 3 / 4 3.34 /
                     3.96 / 3.79 ms against 3.22 (profiles/r06_chains_timeline.txt).
                                                                      (AdaptiveAggregation)
  pipeline           True: the cross-module pipelined schedule (AdaptiveAggregation.
                     _run_pipelined): each module's scale-0 block on a side stream beside the
                     previous module's stride-2 heads and this module's coarse blocks, branch 0's
                     sum + the next conv1 as their own kernels.  Within fp32 summation order of
                     the default.  Measured round 6 (HIP graph): 3.30 vs 3.15 ms -- the scale-0
                     tail beside the heads and coarse blocks slows from 220 to 305 us, i.e. the
                     step is throughput-bound, and the separate sum + conv1 cost 118 us a module
                     (profiles/r06_pipeline_timeline.txt).                (AdaptiveAggregation)
  dense_grouped      True: 2-group convs with 16-channel groups (the scale-1 offset conv) run as
                     one block-diagonal ungrouped conv on the split-bf16 engine; False: the
                     grouped exact-f32 engine.                        (every nn.Conv2d)
"""
import torch.nn as nn

DEFAULTS = {"concurrent_scales": True, "post_fusion": "all", "s2_sums": True,
            "prep_stream": False, "batch_chains": 1, "dense_grouped": True, "pipeline": False}
_POST = ("all", "final", "none")


def get_option(module, name):
    """The option `name` as set on `module` (its default when never set)."""
    return getattr(module, "aanet_" + name, DEFAULTS[name])


def set_options(module, **options):
    """Set schedule options on `module` and every submodule they apply to.  Unknown names or
    values raise ValueError; options left out keep their current value.  Returns `module`."""
    for name, value in options.items():
        if name not in DEFAULTS:
            raise ValueError(f"unknown aanet_amd option {name!r}; known: {sorted(DEFAULTS)}")
        if name == "post_fusion":
            if value not in _POST:
                raise ValueError(f"post_fusion must be one of {_POST}, got {value!r}")
        elif name == "batch_chains":
            if isinstance(value, bool) or not isinstance(value, int) or value < 1:
                raise ValueError(f"batch_chains must be an int >= 1, got {value!r}")
        elif not isinstance(value, bool):
            raise ValueError(f"{name} must be a bool, got {value!r}")
    from .aggregation import AdaptiveAggregation, AdaptiveAggregationModule
    targets = {"concurrent_scales": AdaptiveAggregation, "post_fusion": AdaptiveAggregation,
               "s2_sums": AdaptiveAggregationModule, "prep_stream": AdaptiveAggregationModule,
               "batch_chains": AdaptiveAggregation, "pipeline": AdaptiveAggregation,
               "dense_grouped": nn.Conv2d}
    for m in module.modules():
        for name, value in options.items():
            if isinstance(m, targets[name]):
                setattr(m, "aanet_" + name, value)
    return module
