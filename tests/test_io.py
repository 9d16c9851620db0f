"""Output formats and the inference front-end: PFM byte-compatibility with
the reference's own writer, KITTI uint16x256 PNGs (the reference's demo prediction as the
fixture), and the pad / predict / upsample / crop / save sequence of inference.py."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import io, predict
from tests.golden_io import GOLDEN_DIR, golden

DEMO_PNG = os.path.join(GOLDEN_DIR, "kitti_demo_pred.png")


@pytest.mark.parametrize("name", ["gray", "color"])
def test_write_pfm_bytes_match_reference(tmp_path, name):
    g = golden("pfm_ref")
    path = tmp_path / f"{name}.pfm"
    io.write_pfm(str(path), g[name])
    assert path.read_bytes() == g[f"{name}_bytes"].tobytes()


@pytest.mark.parametrize("name", ["gray", "color"])
def test_read_pfm_of_reference_file(tmp_path, name):
    g = golden("pfm_ref")
    path = tmp_path / f"{name}.pfm"
    path.write_bytes(g[f"{name}_bytes"].tobytes())
    data, scale = io.read_pfm(str(path))
    assert scale == 1.0 and np.array_equal(data, g[name])
    if name == "gray":
        assert np.array_equal(io.read_disp(str(path)), g[name])
        assert np.array_equal(io.read_disp(str(path), subset=True), -g[name])


def test_pfm_rejects_bad_input(tmp_path):
    with pytest.raises(Exception):
        io.write_pfm(str(tmp_path / "x.pfm"), np.zeros((2, 2), np.float64))
    with pytest.raises(Exception):
        io.write_pfm(str(tmp_path / "x.pfm"), np.zeros((2, 2, 2), np.float32))
    (tmp_path / "bad.pfm").write_bytes(b"P6\n1 1\n1.0\n")
    with pytest.raises(Exception):
        io.read_pfm(str(tmp_path / "bad.pfm"))
    with pytest.raises(Exception):
        io.read_disp(str(tmp_path / "x.tiff"))


def test_read_kitti_demo_prediction_like_reference():
    s = golden("kitti_demo_stats")
    d = io.read_disp(DEMO_PNG)
    assert d.dtype == np.float32 and d.shape == tuple(s["shape"])
    assert float(d.astype(np.float64).sum()) == float(s["total"])
    assert int((d > 0).sum()) == int(s["nonzero"])
    assert np.array_equal(d[100], s["row100"])


def test_kitti_png_writer_round_trips_demo_losslessly(tmp_path):
    from PIL import Image
    d = io.read_kitti_disp(DEMO_PNG)
    out = tmp_path / "pred.png"
    io.write_kitti_disp(str(out), d)
    back = np.array(Image.open(str(out)))
    orig = np.array(Image.open(DEMO_PNG))
    assert back.dtype == orig.dtype == np.uint16 and np.array_equal(back, orig)
    assert np.array_equal(io.read_kitti_disp(str(out)), d)


def test_png_encoder_edge_values(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    a = rng.integers(0, 65536, (17, 23), dtype=np.uint16)
    a[0, 0], a[-1, -1], a[5] = 0, 65535, 65535
    p = tmp_path / "e.png"
    p.write_bytes(io.encode_png_u16(a))
    assert np.array_equal(np.array(Image.open(str(p))), a)
    # quantisation of the writer: floor(disp * 256) as uint16 (inference.py:204)
    io.write_kitti_disp(str(p), np.array([[0.0, 1.0 / 256 - 1e-4, 1.5, 255.99]], np.float32))
    assert np.array(Image.open(str(p))).tolist() == [[0, 0, 384, 65533]]


def test_network_input_normalisation():
    img = np.stack([np.full((2, 3), v, np.float32) for v in (0.0, 127.5, 255.0)], -1)
    t = predict.to_network_input(img)
    assert t.shape == (1, 3, 2, 3)
    want = [(0.0 - 0.485) / 0.229, (0.5 - 0.456) / 0.224, (1.0 - 0.406) / 0.225]
    assert torch.allclose(t[0, :, 0, 0], torch.tensor(want), atol=1e-6)


class _Stub(torch.nn.Module):
    """A model stand-in: the pyramid's last level = left channel 0 at 1/2 resolution."""

    def forward(self, left, right):
        return [left[:, 0, ::4, ::4], left[:, 0, ::2, ::2]]


def test_predict_pads_upsamples_and_crops_like_inference_py():
    torch.manual_seed(0)
    left, right = torch.rand(2, 3, 10, 13), torch.rand(2, 3, 10, 13)
    got = predict.predict(_Stub(), left, right, 16, 20)
    # restatement of inference.py:154-188
    lp = F.pad(left, (0, 7, 6, 0))
    pred = lp[:, 0, ::2, ::2]
    pred = F.interpolate(pred.unsqueeze(1), (16, 20), mode="bilinear", align_corners=False)
    pred = (pred * (20 / 10)).squeeze(1)[:, 6:, :-7]
    assert got.shape == (2, 10, 13) and torch.allclose(got, pred)
    # no padding needed: output at the input size, nothing cropped
    got2 = predict.predict(_Stub(), left[..., :8, :12], right[..., :8, :12], 8, 12)
    assert got2.shape == (2, 8, 12)
    # height-only padding (right_pad == 0 branch)
    got3 = predict.predict(_Stub(), left[..., :12], right[..., :12], 16, 12)
    assert got3.shape == (2, 10, 12)


@pytest.mark.parametrize("save_type", ["png", "pfm", "npy"])
def test_save_disparity(tmp_path, save_type):
    d = np.random.default_rng(1).random((6, 9)).astype(np.float32) * 50
    path = predict.save_disparity(d, str(tmp_path / "sub" / "img.png"), save_type,
                                  visualize=save_type == "pfm")
    back = io.read_disp(path)
    if save_type == "png":
        assert np.array_equal(back, np.floor(d * 256) / 256)
    else:
        assert np.array_equal(back, d)
    if save_type == "pfm":
        assert os.path.exists(str(tmp_path / "sub" / "img.png"))
