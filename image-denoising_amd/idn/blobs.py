"""Drop-in for lib/utils/blob.py (im_list_to_blob 17-30, prep_im_for_blob 33-47) on the GPU.

Accepts numpy images (as the reference passes them) or device tensors; computes on the GPU and
returns numpy by default (the detector is fed from host memory, network.py:476-485) or a device
tensor with as_tensor=True.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


def _to_device(im):
    if isinstance(im, torch.Tensor):
        return im if im.device.type == "cuda" else im.cuda()
    return torch.from_numpy(np.ascontiguousarray(im)).cuda()


def _to_host(t: torch.Tensor) -> np.ndarray:
    """A device tensor as a host numpy array, through page-locked memory from torch's caching host
    allocator: a 600x1000 float32 blob (7.2 MB) copied into fresh pageable memory paid its page
    faults on every call (~0.9 ms against ~0.15 ms); the block returns to the cache when the array
    is dropped, as the test loop drops each image's blobs."""
    if t.device.type != "cuda":
        return t.numpy()
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()


def im_scale_for(shape, target_size: int, max_size: int) -> float:
    """prep_im_for_blob's scale rule (blob.py:37-43)."""
    im_size_min = float(min(shape[0:2]))
    im_size_max = float(max(shape[0:2]))
    im_scale = float(target_size) / float(im_size_min)
    if np.round(im_scale * im_size_max) > max_size:
        im_scale = float(max_size) / float(im_size_max)
    return im_scale


def prep_im_for_blob(im, pixel_means, target_size, max_size, flip: bool = False,
                     as_tensor: bool = False, gaussian_ksize=None):
    """im (uint8 BGR or float64) -> (float32 mean-subtracted, resized image, im_scale).

    `flip` folds the roidb 'flipped' column reversal (minibatch.py:1675) into the same pass.
    gaussian_ksize: cv2.GaussianBlur(im, (k, k), 0) still to be applied to the uint8 image (a
    recipe's last step, idn.pipeline.Preprocessor.run_for_blob): at scale 1.0 without a flip the
    blur and the blob are one pass (idn_gaussian_blob_f32), else the blur runs first."""
    x = _to_device(im)
    means = np.asarray(pixel_means, np.float64).reshape(-1)
    if gaussian_ksize:
        if x.dtype != torch.uint8:
            raise TypeError("prep_im_for_blob: a deferred GaussianBlur needs a uint8 image")
        if not flip and im_scale_for(x.shape, target_size, max_size) == 1.0:
            f = ops.gaussian_blob(x, int(gaussian_ksize), means)[0]
            return (f if as_tensor else _to_host(f)), 1.0
        x = ops.gaussian_blur(x, int(gaussian_ksize))
    if x.dtype == torch.uint8:
        f = ops.blob(x, means, flip=flip)[0]
    elif x.dtype == torch.float64:
        f = ops.blob_from_f64(x, means, flip=flip)[0]
    elif x.dtype == torch.float32:
        f = ops.blob_from_f64(x.double(), means, flip=flip)[0]  # f32 -> f64 is exact
    else:
        raise TypeError(f"prep_im_for_blob: unsupported dtype {x.dtype}")
    im_scale = im_scale_for(f.shape, target_size, max_size)
    if im_scale != 1.0:
        f = ops.resize_linear(f, im_scale, im_scale)
    return (f if as_tensor else _to_host(f)), im_scale


def im_list_to_blob(ims, as_tensor: bool = False):
    """Zero-padded NHWC float32 blob of prepared images (numpy or device tensors)."""
    xs = [_to_device(im) for im in ims]
    if len(xs) == 1 and not as_tensor:  # nothing to pad: straight to the host
        return _to_host(xs[0].float().unsqueeze(0))
    hmax = max(int(x.shape[0]) for x in xs)
    wmax = max(int(x.shape[1]) for x in xs)
    blob = torch.zeros((len(xs), hmax, wmax, 3), dtype=torch.float32, device=xs[0].device)
    for i, x in enumerate(xs):
        blob[i, : x.shape[0], : x.shape[1], :] = x.float()
    return blob if as_tensor else _to_host(blob)
