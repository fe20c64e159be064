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


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["s420_opt_130x170.jpg", "s422_q85_120x200.jpg"])
def test_get_minibatch_gpu_decode_matches_libjpeg9_pixels(dev, tmp_path, name):
    """decode="gpu" (cv2.imread at minibatch.py:85 on the GPU): the blob equals the one built from
    the reference's pinned libjpeg 9d pixels of the same file (tests/golden/jpeg9.npz)"""
    import shutil
    from pathlib import Path
    from idn import minibatch
    from idn.roidb import prepare_roidb
    gold = Path(__file__).resolve().parent / "golden"
    px = np.load(gold / "jpeg9.npz")[name]
    imdb = _imdb(tmp_path, [px])
    shutil.copyfile(gold / "jpeg" / name, tmp_path / name)
    imdb._paths = [tmp_path / name]
    prepare_roidb(imdb, "gaussian_mean_var0.1")
    entry = dict(imdb.roidb[0], flipped=True)
    random.seed(5)
    np.random.seed(6)
    got = minibatch.get_minibatch([entry], 21, mode="train_v0", noise_rng="numpy", decode="gpu")
    random.seed(5)
    np.random.seed(6)
    ref = minibatch.get_minibatch([dict(entry, im=px)], 21, mode="train_v0", noise_rng="numpy")
    assert np.array_equal(got["data"], ref["data"])
    assert np.array_equal(got["im_info"], ref["im_info"])


@pytest.mark.gpu
def test_apply_noise_gpu_decode(dev):
    from pathlib import Path
    from idn import detect_blob
    from idn._lib import IdnError
    gold = Path(__file__).resolve().parent / "golden"
    name = "s420_q75_odd_37x53.jpg"
    px = np.load(gold / "jpeg9.npz")[name]
    random.seed(2)
    a = detect_blob.apply_noise(gold / "jpeg" / name, "gaussian_wavelet_var0.1", decode="gpu",
                                noise_rng="philox", image_id=4)
    random.seed(2)
    b = detect_blob.apply_noise(px, "gaussian_wavelet_var0.1", noise_rng="philox", image_id=4)
    assert a.dtype == b.dtype and np.array_equal(a, b)
    # no silent CPU fallback for files the decoder does not take (lossless coding)
    from test_jpeg import _lossless
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        bad = Path(d) / "lossless.jpg"
        bad.write_bytes(_lossless((gold / "jpeg" / "s444_q95_96x128.jpg").read_bytes()))
        with pytest.raises(IdnError):
            detect_blob.apply_noise(bad, "original", decode="gpu")
    # a progressive file is decoded (the scan path), as cv2.imread does
    prog = detect_blob.apply_noise(gold / "jpeg" / "progressive_64x64.jpg", "original",
                                   mode="canonical", decode="gpu")
    assert np.array_equal(prog, np.load(gold / "jpeg9.npz")["progressive_64x64.jpg"])


@pytest.mark.gpu
@pytest.mark.parametrize("flip", [False, True])
def test_minibatch_defers_final_gaussian_into_the_blob(dev, flip):
    """a recipe ending in a uint8 GaussianBlur at scale 1.0: _get_image_blob runs the blur and
    prep_im_for_blob as one pass (idn_gaussian_blob_f32); the blob equals the two-step result
    (flipped entries take the two steps)"""
    import torch
    from idn import minibatch, ops
    img = textured(1, 600, 1000, seed=8)[0]
    spec = "speckle_gaus_blur_var0.5"
    entry = {"im": img, "noise_type": spec, "flipped": flip, "index": 3}
    pre = minibatch._preprocessor(spec, "canonical", "numpy")
    random.seed(1)
    np.random.seed(2)
    _, ks, _ = pre.run_for_blob(torch.from_numpy(img).cuda()[None], image_ids=[3])
    assert ks[0] in (3, 5)
    random.seed(1)
    np.random.seed(2)
    blob, scales = minibatch._get_image_blob([entry], [0], mode="canonical", noise_rng="numpy")
    assert scales == [1.0]
    random.seed(1)
    np.random.seed(2)
    outs, _ = pre(torch.from_numpy(img).cuda()[None], image_ids=[3])
    ref = ops.blob(outs[0][None], flip=flip).cpu().numpy()
    assert np.array_equal(blob, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["s420_opt_130x170.jpg", "s422_q85_120x200.jpg",
                                  "prog_s444_q85_96x128.jpg"])
def test_host_decode_without_cv2_is_libjpeg9(dev, tmp_path, name):
    """decode="host" (the default) with no OpenCV: io.imread sends JPEGs to the GPU decoder, so
    the pixels -- and get_minibatch's blob -- are the reference's pinned libjpeg 9d decode, not
    PIL's libjpeg-turbo (tests/golden/jpeg9.npz)"""
    import importlib.util
    import shutil
    from pathlib import Path
    from idn import io, minibatch
    from idn.roidb import prepare_roidb
    if importlib.util.find_spec("cv2") is not None:
        pytest.skip("OpenCV present: io.imread is cv2.imread itself")
    gold = Path(__file__).resolve().parent / "golden"
    px = np.load(gold / "jpeg9.npz")[name]
    assert np.array_equal(io.imread(gold / "jpeg" / name), px)
    imdb = _imdb(tmp_path, [px])
    shutil.copyfile(gold / "jpeg" / name, tmp_path / name)
    imdb._paths = [tmp_path / name]
    prepare_roidb(imdb, "sap_median_var0.4")
    entry = dict(imdb.roidb[0])
    random.seed(5)
    np.random.seed(6)
    got = minibatch.get_minibatch([entry], 21, mode="train_v0", noise_rng="numpy")  # decode="host"
    random.seed(5)
    np.random.seed(6)
    ref = minibatch.get_minibatch([dict(entry, im=px)], 21, mode="train_v0", noise_rng="numpy")
    assert np.array_equal(got["data"], ref["data"])


@pytest.mark.gpu
def test_host_decode_without_cv2_raises_on_unsupported_jpeg(dev, tmp_path):
    """a JPEG the GPU decoder does not take (here a lossless-process frame, SOF3) raises: no
    silent libjpeg-turbo / PIL decode in its place"""
    import importlib.util
    from idn import io
    from idn._lib import IdnError
    from test_jpeg import _lossless
    if importlib.util.find_spec("cv2") is not None:
        pytest.skip("OpenCV present")
    import pathlib
    gold = pathlib.Path(__file__).resolve().parent / "golden" / "jpeg"
    (tmp_path / "lossless.jpg").write_bytes(_lossless((gold / "s444_q95_96x128.jpg").read_bytes()))
    with pytest.raises(IdnError):
        io.imread(tmp_path / "lossless.jpg")


@pytest.mark.gpu
def test_shared_preprocessor_is_reentrant(dev):
    """A cached Preprocessor shared by threads: run_for_blob's deferral and the bloom draws are
    per call (no instance state), so concurrent __call__ / run_for_blob calls return what the
    same calls return one at a time"""
    import threading
    import torch
    from idn.pipeline import Preprocessor
    imgs = torch.from_numpy(textured(2, 64, 96, seed=4)).cuda()
    pre = Preprocessor("speckle_gaus_blur_var0.5", "canonical", seed=3)
    plans = pre.plans(2, hw=(64, 96))
    ref_full, _ = pre(imgs, image_ids=[0, 1], plans=plans)
    ref_def, ref_ks, _ = pre.run_for_blob(imgs, image_ids=[0, 1], plans=plans)
    assert ref_ks == [5, 5] or ref_ks == [3, 3]
    errs = []

    def worker(k):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                for _ in range(20):
                    if k % 2:
                        o, ks, _ = pre.run_for_blob(imgs, image_ids=[0, 1], plans=plans)
                        ok = ks == ref_ks and all(torch.equal(a, b) for a, b in zip(o, ref_def))
                    else:
                        o, _ = pre(imgs, image_ids=[0, 1], plans=plans)
                        ok = all(torch.equal(a, b) for a, b in zip(o, ref_full))
                    torch.cuda.current_stream().synchronize()
                    if not ok:
                        errs.append(k)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
