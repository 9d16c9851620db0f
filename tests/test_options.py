"""The eval schedule options are explicit module state (nets/options.py), never read from the
process environment: set_options reaches the submodules each option applies to, rejects unknown
names and values, and the package's module layer has no environment reads at all."""
import os

import pytest

from aanet_amd import nets
from aanet_amd.nets.options import DEFAULTS, get_option, set_options


def test_defaults_and_propagation():
    m = nets.AANetHotPath(64, no_intermediate_supervision=True)
    agg = m.aggregation
    for k, v in DEFAULTS.items():
        target = {"concurrent_scales": agg, "post_fusion": agg, "s2_sums": agg.fusions[0],
                  "batch_chains": agg, "prep_stream": agg.fusions[4], "pipeline": agg,
                  "dense_grouped": agg.fusions[5].branches[1][0].conv2.offset_conv}[k]
        assert get_option(target, k) == v
    assert m.set_options(concurrent_scales=False, post_fusion="final", s2_sums=False,
                         dense_grouped=False, batch_chains=2, prep_stream=False,
                         pipeline=True) is m
    assert get_option(agg, "pipeline") is True
    assert all(get_option(f, "prep_stream") is False for f in agg.fusions)
    assert get_option(agg, "batch_chains") == 2
    assert get_option(agg, "concurrent_scales") is False
    assert get_option(agg, "post_fusion") == "final"
    assert all(get_option(f, "s2_sums") is False for f in agg.fusions)
    convs = [c for c in m.modules() if type(c).__name__ == "Conv2d"]
    assert convs and all(get_option(c, "dense_grouped") is False for c in convs)
    agg.set_options(post_fusion="none")          # options left out keep their value
    assert get_option(agg, "post_fusion") == "none" and not get_option(agg, "concurrent_scales")


def test_full_model_and_module_function():
    model = nets.AANet(192)
    set_options(model, s2_sums=False)
    assert all(get_option(f, "s2_sums") is False for f in model.aggregation.fusions)


@pytest.mark.parametrize("kw", [{"concurrent": True}, {"post_fusion": "0"},
                                {"s2_sums": 1}, {"dense_grouped": "no"},
                                {"batch_chains": 0}, {"batch_chains": True}, {"pipeline": 1}])
def test_rejects_unknown(kw):
    with pytest.raises(ValueError):
        nets.AANetHotPath(16).set_options(**kw)


def test_module_layer_reads_no_environment():
    root = os.path.join(os.path.dirname(__file__), "..", "aanet_amd", "nets")
    for fn in sorted(os.listdir(root)):
        if fn.endswith(".py"):
            src = open(os.path.join(root, fn)).read()
            assert "os.environ" not in src and "getenv" not in src, fn


def test_exact_f32_is_a_scoped_context_setting_not_an_environment_switch():
    """the split-bf16 / exact-f32 contraction choice is a per-context setting
    (`_lib.exact_f32()` scope, `set_exact_f32`), never read from the process environment, and it
    does not leak into other threads."""
    import os
    import subprocess
    import sys
    import threading

    from aanet_amd import _lib
    assert _lib.conv_flags() == 0 and not _lib.exact_f32_enabled()
    with _lib.exact_f32():
        assert _lib.conv_flags() == _lib.CONV_EXACT_F32
        seen = []
        t = threading.Thread(target=lambda: seen.append(_lib.exact_f32_enabled()))
        t.start()
        t.join()
        assert seen == [False]
    assert _lib.conv_flags() == 0
    code = "from aanet_amd import _lib; print(_lib.exact_f32_enabled())"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         env={**os.environ, "AANET_EXACT_F32": "1"}, cwd=repo).stdout.strip()
    assert out == "False"
