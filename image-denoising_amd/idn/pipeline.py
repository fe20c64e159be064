"""Batch executor of noise-spec plans on the GPU.

`Preprocessor(noise, mode)` turns a batch of uint8 BGR images (device tensor (N,H,W,3)) into what
the reference's per-image loop body produces for each image (lib/model/test.py:189-1831 for
mode='test_v0', lib/roi_data_layer/minibatch.py:84-1677 for 'train_v0', the README grammar for
'canonical'): a uint8 or float64 image per input, plus the resolved Plan.  Images whose plans are
identical run as one sub-batch through each kernel (a mixed batch -- BASELINE config 5 -- is
grouped by plan), so a homogeneous batch is a single launch per step.

Randomness:
  rng        Python-level choices (mix noise type, gaussian level, bloom circles): `random`
             module semantics; default a `random.Random(seed)`
  noise_rng  'philox'  device Philox4x32 stream keyed by (seed, image id): fast, statistically
                        equivalent to numpy's draws
             'numpy'   draw the fields with numpy's global legacy RandomState exactly as
                        skimage.random_noise does, replay them on the GPU: bit-exact with the
                        reference for the same numpy state (host RNG cost, like the reference)
"""
from __future__ import annotations

import random as _random
from collections import OrderedDict
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import noise_spec as ns
from . import ops


class Preprocessor:
    def __init__(self, noise: str, mode: str = "canonical", seed: int = 3,
                 rng: Optional[_random.Random] = None, noise_rng: str = "philox"):
        if noise_rng not in ("philox", "numpy"):
            raise ValueError("noise_rng must be 'philox' or 'numpy'")
        self.noise = noise
        self.mode = mode
        self.seed = int(seed)
        self.rng = rng if rng is not None else _random.Random(seed)
        self.noise_rng = noise_rng

    # ---- planning ------------------------------------------------------------------------
    def plans(self, n: int, hw: Optional[Tuple[int, int]] = None) -> List[ns.Plan]:
        """n plans in image order; with hw = (H, W) bloom plans carry their circle draws (so the
        rng sequence is the reference's per-image order and does not depend on execution)."""
        return [ns.plan(self.noise, self.mode, self.rng, hw=hw) for _ in range(n)]

    # ---- execution -----------------------------------------------------------------------
    def __call__(self, batch: torch.Tensor, image_ids: Optional[Sequence[int]] = None,
                 plans: Optional[Sequence[ns.Plan]] = None):
        """Returns (outputs, plans): outputs[i] is a device tensor (H,W,3) uint8 or float64."""
        outs, _, plans = self._execute(batch, image_ids, plans, defer=False)
        return outs, plans

    def run_for_blob(self, batch: torch.Tensor, image_ids: Optional[Sequence[int]] = None,
                     plans: Optional[Sequence[ns.Plan]] = None):
        """Like __call__, but a plan that ends in a uint8 cv2.GaussianBlur stops before it:
        returns (outputs, ksizes, plans) with ksizes[i] the deferred blur's ksize (None if
        nothing was deferred), so the blob builder can run the blur and prep_im_for_blob as one
        pass (idn_gaussian_blob_f32) -- the filtered uint8 image never reaches HBM."""
        return self._execute(batch, image_ids, plans, defer=True)

    def _execute(self, batch, image_ids, plans, defer: bool):
        # all per-call state lives in locals / arguments: a Preprocessor may be shared between
        # threads (the drop-ins cache one per spec)
        if batch.dim() == 3:
            batch = batch.unsqueeze(0)
        n = batch.shape[0]
        plans = list(plans) if plans is not None else self.plans(n, hw=tuple(batch.shape[1:3]))
        ids = list(image_ids) if image_ids is not None else list(range(n))
        groups: "OrderedDict[tuple, List[int]]" = OrderedDict()
        for i, p in enumerate(plans):
            # numpy-stream mode draws image by image, in order, like the reference's loop;
            # bloom images share one launch whatever their (per-image) circle draws
            key = (i,) if self.noise_rng == "numpy" else _group_key(p.steps)
            groups.setdefault(key, []).append(i)
        outs: List[Optional[torch.Tensor]] = [None] * n
        ks: List[Optional[int]] = [None] * n
        for _, idx in groups.items():
            steps = plans[idx[0]].steps
            if len(idx) == n:
                sub = batch
            else:
                sub = batch.index_select(0, torch.as_tensor(idx, device=batch.device))
            bloom = [next((st.args for st in plans[i].steps if st.op == "bloom"), ()) for i in idx]
            res, k_def = self._run_steps(sub, steps, [ids[i] for i in idx], bloom, defer)
            for k, i in enumerate(idx):
                outs[i] = res[k]
                ks[i] = k_def
        return outs, ks, plans

    def run_batch(self, batch: torch.Tensor, image_ids=None, plans=None):
        """Like __call__ but stacks the outputs when they share dtype and shape."""
        outs, plans = self(batch, image_ids, plans)
        if len({(o.dtype, tuple(o.shape)) for o in outs}) == 1:
            return torch.stack(outs), plans
        return outs, plans

    def _noise(self, x: torch.Tensor, step: ns.Step, nxt: Optional[ns.Step], ids: List[int],
               bloom=()):
        op = step.op
        if op == "original":
            return x
        if op == "periodic":
            _, h, w, c = x.shape
            return ops.periodic_noise(x, ns.periodic_amplitude(step.args[0], h * w * c))
        if op == "shader":
            return ops.shader(x, 3.0)
        if op == "quant":
            if ids != list(range(ids[0], ids[0] + len(ids))):
                return ops.quantize(x, int(step.args[0]), seed=self.seed, image_ids=ids)
            return ops.quantize(x, int(step.args[0]), seed=self.seed, offset=int(ids[0]))
        if op == "bloom":
            draws = list(bloom)
            if len(draws) == x.shape[0] and all(draws):
                return ops.bloom(x, circles=[(np.asarray(c, np.int32), np.asarray(w, np.float32))
                                             for c, w in draws])
            return ops.bloom(x, rng=self.rng)  # a plan resolved without (H, W): draw now
        if op in ops.ADD_NOISE_KINDS:
            out = "u8" if (op == "brownian" or (nxt is not None and nxt.kind == "cast_u8")) else "f64"
            level = float(step.args[0])
            if self.noise_rng == "numpy":
                return ops.noise_add(x, op, level, replay=self._numpy_add_field(x, op), out=out)
            if ids != list(range(ids[0], ids[0] + len(ids))):
                # non-contiguous image ids (a mixed batch): one launch with the id array
                return ops.noise_add(x, op, level, seed=self.seed, image_ids=ids, out=out)
            return ops.noise_add(x, op, level, seed=self.seed, offset=int(ids[0]), out=out)
        mode = {"gaussian": "gaussian", "speckle": "speckle", "sap": "s&p", "poisson": "poisson"}[op]
        kw = {}
        if op in ("gaussian", "speckle"):
            kw["var"] = float(step.args[0])
        elif op == "sap":
            kw["amount"] = float(step.args[0])
        out = "u8" if (nxt is not None and nxt.kind == "cast_u8") else "f64"
        replay = self._numpy_field(x, mode, kw) if self.noise_rng == "numpy" else None
        offsets = ids
        if replay is None and offsets != list(range(offsets[0], offsets[0] + len(offsets))):
            # non-contiguous image ids (a mixed batch): one launch with the id array keeps the
            # (seed, id) stream of every image
            return ops.random_noise(x, mode, seed=self.seed, image_ids=offsets, out=out, **kw)
        return ops.random_noise(x, mode, seed=self.seed, offset=int(offsets[0]), replay=replay,
                                out=out, **kw)

    def _noise_ycc(self, x: torch.Tensor, step: ns.Step, ids: List[int]):
        """_noise's gaussian / speckle float64 branch with the wavelet's colour range (the same
        draws and the same image: ops.random_noise_ycc)"""
        kw = {"var": float(step.args[0])}
        replay = self._numpy_field(x, step.op, kw) if self.noise_rng == "numpy" else None
        if replay is None and ids != list(range(ids[0], ids[0] + len(ids))):
            return ops.random_noise_ycc(x, step.op, seed=self.seed, image_ids=ids, **kw)
        return ops.random_noise_ycc(x, step.op, seed=self.seed, offset=int(ids[0]),
                                    replay=replay, **kw)

    def _numpy_field(self, x: torch.Tensor, mode: str, kw) -> torch.Tensor:
        """The exact draws skimage.random_noise makes from numpy's global RandomState."""
        host = x.cpu().numpy()
        fields = []
        for img in host:
            if mode in ("gaussian", "speckle"):
                fields.append(np.random.normal(0.0, kw["var"] ** 0.5, img.shape))
            elif mode == "s&p":
                fields.append(np.stack([np.random.random_sample(img.shape),
                                        np.random.random_sample(img.shape)]))
            else:
                xf = img.astype(np.float64) * (1.0 / 255.0)
                vals = 2 ** np.ceil(np.log2(len(np.unique(xf))))
                fields.append(np.random.poisson(xf * vals).astype(np.float64))
        if mode == "s&p":
            f = np.stack([np.stack([a[0] for a in fields]), np.stack([a[1] for a in fields])])
        else:
            f = np.stack(fields)
        return torch.from_numpy(np.ascontiguousarray(f)).to(x.device)

    def _numpy_add_field(self, x: torch.Tensor, op: str) -> torch.Tensor:
        """numpy's unit draws for the additive closures, image by image, in the reference's
        order: np.random.uniform -> random_sample; scipy gamma.rvs -> standard_gamma(1.99);
        scipy rayleigh.rvs -> sqrt(chisquare(2)); brownian -> normal(size=n-1) at elements 1.."""
        shape = tuple(x.shape[1:])
        fields = []
        for _ in range(x.shape[0]):
            if op == "uniform":
                f = np.random.random_sample(shape)
            elif op == "gamma":
                f = np.random.standard_gamma(ops.GAMMA_SHAPE, shape)
            elif op == "rayleigh":
                f = np.sqrt(np.random.chisquare(2, shape))
            else:
                size = int(np.prod(shape))
                f = np.zeros(size)
                f[1:] = np.random.normal(size=size - 1)
                f = f.reshape(shape)
            fields.append(f)
        return torch.from_numpy(np.ascontiguousarray(np.stack(fields))).to(x.device)

    def _filter(self, x: torch.Tensor, step: ns.Step) -> torch.Tensor:
        op, a = step.op, step.args
        f64 = x.dtype == torch.float64
        if op == "gaus_blur":
            return ops.gaussian_blur_f64(x, a[0]) if f64 else ops.gaussian_blur(x, a[0])
        if op == "mean":
            return ops.blur_f64(x, a[0]) if f64 else ops.blur(x, a[0])
        if op == "median":
            if f64:
                raise RuntimeError("cv2.error: medianBlur does not support float64 input")
            return ops.median_blur(x, a[0])
        if op == "bilateral":
            if f64:
                raise RuntimeError("cv2.error: bilateralFilter supports only 8u and 32f images")
            return ops.bilateral_filter(x, a[0], a[1], a[2])
        if op == "wavelet":
            return ops.denoise_wavelet(x, a[0], a[1])
        raise ValueError(f"unknown filter step {op!r}")

    def _run_steps(self, x: torch.Tensor, steps: Tuple[ns.Step, ...], ids: List[int],
                   bloom=(), defer: bool = False):
        cur = x
        i = 0
        while i < len(steps):
            st = steps[i]
            nxt = steps[i + 1] if i + 1 < len(steps) else None
            if (nxt is None and defer and st.kind == "filter"
                    and st.op == "gaus_blur" and cur.dtype == torch.uint8):
                return list(cur.unbind(0)), int(st.args[0])  # left to the blob builder
            if (st.kind == "noise" and st.op in ("gaussian", "speckle") and nxt is not None
                    and nxt.kind == "filter" and nxt.op == "wavelet" and ops.ycc_fusable(cur)):
                # the float64 image goes straight into the wavelet (test_v0's live path): the
                # noise kernel reduces the wavelet's colour range while it writes the image
                cur, keys = self._noise_ycc(cur, st, ids)
                cur = ops.denoise_wavelet(cur, nxt.args[0], nxt.args[1], ycc_keys=keys)
                i += 2
                continue
            if st.kind == "noise":
                cur = self._noise(cur, st, nxt, ids, bloom)
                if nxt is not None and nxt.kind == "cast_u8":
                    i += 1  # fused into the noise kernel's U8 output
            elif st.kind == "cast_u8":
                raise RuntimeError("internal: a U8 cast must follow a noise step")
            else:
                cur = self._filter(cur, st)
            i += 1
        return list(cur.unbind(0)), None


def _group_key(steps: Tuple[ns.Step, ...]) -> tuple:
    return tuple(ns.Step(st.kind, st.op) if st.op == "bloom" else st for st in steps)


def blob_from_outputs(outs: Sequence[torch.Tensor], pixel_means=ops.PIXEL_MEANS,
                      flips: Optional[Sequence[bool]] = None) -> torch.Tensor:
    """im_list_to_blob(prep_im_for_blob(...)) at scale 1.0 for a list of device images (u8 or f64),
    zero-padded to the max H, W (lib/utils/blob.py:17-30)."""
    hmax = max(o.shape[0] for o in outs)
    wmax = max(o.shape[1] for o in outs)
    blob = torch.zeros((len(outs), hmax, wmax, 3), dtype=torch.float32, device=outs[0].device)
    flips = flips or [False] * len(outs)
    for i, o in enumerate(outs):
        h, w = o.shape[:2]
        if o.dtype == torch.uint8:
            b = ops.blob(o, pixel_means, flip=flips[i])
        else:
            b = ops.blob_from_f64(o, pixel_means, flip=flips[i])
        blob[i, :h, :w] = b[0]
    return blob
