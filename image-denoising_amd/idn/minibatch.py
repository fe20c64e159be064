# Portions of this file (get_minibatch's blob / label assembly) follow Fast R-CNN's
#   lib/roi_data_layer/minibatch.py -- Fast R-CNN, Copyright (c) 2015 Microsoft,
#   Licensed under The MIT License, written by Ross Girshick and Xinlei Chen.
# The drop-in keeps that function's behaviour (asserts and messages included) line for line.
"""Drop-in for the training-side data path: lib/roi_data_layer/minibatch.py get_minibatch (42-75)
and _get_image_blob (77-1690), with the per-image noise + denoise recipe of the roidb entry's
`noise_type` executed on the GPU (idn.pipeline) instead of the closures at minibatch.py:87-1673.

mode='train_v0' (default) reproduces minibatch.py as-is, quirks included (double filtering by the
post hook, float64 plain branches, sap var0.8 -> 0.6 ...); mode='canonical' follows the README.
"""
from __future__ import annotations

import random as _random
from types import SimpleNamespace

import numpy as np
import numpy.random as npr

from . import blobs as _blob
from . import io as _io
from .pipeline import Preprocessor

# the keys of lib/model/config.py this path reads (config.py:63,66,86,252,255)
cfg = SimpleNamespace(
    PIXEL_MEANS=np.array([[[102.9801, 115.9465, 122.7717]]]),
    RNG_SEED=3,
    TRAIN=SimpleNamespace(SCALES=(600,), MAX_SIZE=1000, BATCH_SIZE=128, USE_ALL_GT=True,
                          USE_FLIPPED=True),
)

_PREPROCESSORS = {}


def _preprocessor(noise: str, mode: str, noise_rng: str):
    key = (noise, mode, noise_rng)
    p = _PREPROCESSORS.get(key)
    if p is None:
        # Python-level choices come from the global `random`, as in the reference
        p = _PREPROCESSORS[key] = Preprocessor(noise, mode, seed=cfg.RNG_SEED, rng=_random,
                                               noise_rng=noise_rng)
    return p


def get_minibatch(roidb, num_classes, mode: str = "train_v0", noise_rng: str = "philox",
                  decode: str = "host"):
    """Given a roidb, construct a minibatch sampled from it (minibatch.py:42).  decode="gpu"
    reads the images with the GPU JPEG decoder (cv2.imread at minibatch.py:85 -> idn.io.imread_gpu,
    bit-exact with the pinned libjpeg 9d); a file it does not take raises IdnError."""
    num_images = len(roidb)
    random_scale_inds = npr.randint(0, high=len(cfg.TRAIN.SCALES), size=num_images)
    assert cfg.TRAIN.BATCH_SIZE % num_images == 0, \
        "num_images ({}) must divide BATCH_SIZE ({})".format(num_images, cfg.TRAIN.BATCH_SIZE)
    im_blob, im_scales = _get_image_blob(roidb, random_scale_inds, mode=mode, noise_rng=noise_rng,
                                         decode=decode)
    blobs = {"data": im_blob}
    assert len(im_scales) == 1, "Single batch only"
    assert len(roidb) == 1, "Single batch only"
    if cfg.TRAIN.USE_ALL_GT:
        gt_inds = np.where(roidb[0]["gt_classes"] != 0)[0]
    else:
        gt_inds = np.where(roidb[0]["gt_classes"] != 0 &
                           np.all(roidb[0]["gt_overlaps"].toarray() > -1.0, axis=1))[0]
    gt_boxes = np.empty((len(gt_inds), 5), dtype=np.float32)
    gt_boxes[:, 0:4] = roidb[0]["boxes"][gt_inds, :] * im_scales[0]
    gt_boxes[:, 4] = roidb[0]["gt_classes"][gt_inds]
    blobs["gt_boxes"] = gt_boxes
    blobs["im_info"] = np.array([im_blob.shape[1], im_blob.shape[2], im_scales[0]], dtype=np.float32)
    return blobs


def _get_image_blob(roidb, scale_inds, mode: str = "train_v0", noise_rng: str = "philox",
                    as_tensor: bool = False, decode: str = "host"):
    """Builds an input blob from the images in the roidb at the specified scales."""
    if decode not in ("host", "gpu"):
        raise ValueError("decode must be 'host' or 'gpu'")
    processed_ims, im_scales = [], []
    for i in range(len(roidb)):
        img = roidb[i].get("im")
        if img is None:
            img = (_io.imread_gpu([roidb[i]["image"]])[0] if decode == "gpu"
                   else _io.imread(roidb[i]["image"]))
        pre = _preprocessor(roidb[i]["noise_type"], mode, noise_rng)
        # a recipe that ends in a uint8 GaussianBlur leaves that blur to the blob builder: at
        # scale 1.0 without a flip the blur and prep_im_for_blob run as one pass
        outs, ks, _plans = pre.run_for_blob(_blob._to_device(img)[None],
                                            image_ids=[int(roidb[i].get("index", 0))])
        target_size = cfg.TRAIN.SCALES[scale_inds[i]]
        flip = bool(roidb[i].get("flipped", False))
        im, im_scale = _blob.prep_im_for_blob(outs[0], cfg.PIXEL_MEANS, target_size,
                                              cfg.TRAIN.MAX_SIZE, flip=flip, as_tensor=True,
                                              gaussian_ksize=ks[0])
        im_scales.append(im_scale)
        processed_ims.append(im)
    blob = _blob.im_list_to_blob(processed_ims, as_tensor=as_tensor)
    return blob, im_scales
