"""GPU test of the training-side drop-in boundary:
  * idn.roidb.prepare_roidb on a fake imdb (lib/roi_data_layer/roidb.py:19-50): the derived
    fields and the `noise_type` stamp the data layer reads;
  * idn.minibatch.get_minibatch (minibatch.py:42-75, _get_image_blob 77-1690) end to end against
    the oracle composition: the plan the reference's closure draws from the same global `random`
    state, executed by the oracle ops with the same numpy draws (noise_rng='numpy'), then
    prep_im_for_blob (f32 cast, mean subtraction, bilinear resize; blob.py:33-47) and
    im_list_to_blob (blob.py:17-30), plus gt_boxes / im_info (minibatch.py:64-74).
The image goes through a lossless PNG so the decode is exact on both sides."""
import random

import numpy as np
import pytest

from conftest import textured

MEANS = np.array([[[102.9801, 115.9465, 122.7717]]])


class FakeImdb:
    """the slice of lib/datasets/imdb.py prepare_roidb touches"""

    def __init__(self, paths, roidb, name="voc_2007_trainval"):
        self.name = name
        self._paths = list(paths)
        self.roidb = roidb
        self.image_index = list(range(len(paths)))
        self.num_images = len(paths)

    def image_path_at(self, i):
        return str(self._paths[i])


def _imdb(tmp_path, imgs):
    import scipy.sparse
    from PIL import Image
    paths, roidb = [], []
    for i, im in enumerate(imgs):
        p = tmp_path / f"im{i}.png"
        Image.fromarray(np.ascontiguousarray(im[..., ::-1])).save(p)  # BGR -> RGB file
        paths.append(p)
        ov = np.zeros((2, 21), np.float32)
        ov[0, 5] = 1.0
        ov[1, 12] = 0.7
        roidb.append({"boxes": np.array([[10, 20, 100, 120], [50, 60, 210, 199]], np.uint16),
                      "gt_classes": np.array([5, 12], np.int32),
                      "gt_overlaps": scipy.sparse.csr_matrix(ov),
                      "flipped": False})
    return FakeImdb(paths, roidb)


def test_prepare_roidb(tmp_path):
    from idn.roidb import prepare_roidb
    imgs = textured(2, 200, 300, seed=4)
    imdb = _imdb(tmp_path, imgs)
    prepare_roidb(imdb, "gaussian_mean_var0.1")
    for i, r in enumerate(imdb.roidb):
        assert r["image"] == imdb.image_path_at(i) and r["index"] == i
        assert (r["width"], r["height"]) == (300, 200)
        assert r["max_classes"].tolist() == [5, 12]
        assert np.allclose(r["max_overlaps"], [1.0, 0.7])
        assert r["noise_type"] == "gaussian_mean_var0.1"


@pytest.mark.gpu
@pytest.mark.parametrize("spec,flip", [("gaussian_mean_var0.1", False), ("sap_var0.8", True),
                                       ("poisson_median", False)])
def test_get_minibatch_matches_oracle(dev, tmp_path, spec, flip):
    import oracle
    from idn import minibatch, noise_spec as ns
    from idn.roidb import prepare_roidb
    from plan_oracle import run_plan
    img = textured(1, 300, 400, seed=len(spec))[0]
    imdb = _imdb(tmp_path, [img])
    prepare_roidb(imdb, spec)
    entry = dict(imdb.roidb[0], flipped=flip)

    random.seed(11)
    np.random.seed(21)
    blobs = minibatch.get_minibatch([entry], 21, mode="train_v0", noise_rng="numpy")

    # the oracle composition, from the same global states
    random.seed(11)
    np.random.seed(21)
    np.random.randint(0, high=1, size=1)  # get_minibatch's random_scale_inds draw
    plan = ns.plan(spec, "train_v0", random, hw=(300, 400))
    out, _ = run_plan(img, plan.steps, random)
    f = out.astype(np.float32, copy=False)
    if flip:
        f = f[:, ::-1, :]
    f = np.array(f, np.float32)
    f -= MEANS
    scale = 600 / 300  # min side 300 -> 600, max side 800 <= 1000
    ref = oracle.cvf.resize_linear_f32(f, scale, scale)

    data = blobs["data"]
    assert data.shape == (1,) + ref.shape and data.dtype == np.float32
    assert np.array_equal(data[0], ref), (spec, np.abs(data[0] - ref).max())
    boxes = entry["boxes"].astype(np.float32) * scale
    assert np.array_equal(blobs["gt_boxes"][:, :4], boxes)
    assert blobs["gt_boxes"][:, 4].tolist() == [5, 12]
    assert blobs["im_info"].tolist() == [600.0, 800.0, 2.0]
