"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

Sequential restatement of the `bloom` and `shader` noise types, pass by pass as the reference
runs them:

  add_bloom  lib/model/test.py:1590-1594 -> Automold.add_sun_flare (tools/Automold.py:588-627):
             add_sun_process (575-586): 8 x {filled circle on a cumulative overlay,
             cv2.addWeighted(overlay, a, output, 1-a, 0, output)}, then flare_source (553-563) on
             a fresh overlay: 40 concentric white circles, alpha = linspace(0,1,40)[39-i]**3.
  add_shader lib/model/test.py:1595-1601: PIL ImageEnhance.Brightness(3) -> RGB array.

cv2 is absent, so cv2.circle (LINE_8, thickness -1: imgproc/drawing.cpp Circle() midpoint spans)
and cv2.addWeighted (8U: float32 s1*a + s2*b + g, round half even, saturate) are restated here in
numpy.  Parity vs real cv2 is UNPINNED (no cv2 in the image); the GPU kernel evaluates the 48
blends per pixel in one pass and is checked against this literal sequential version.
"""
from __future__ import annotations

import math

import numpy as np


def circle_fill(img: np.ndarray, center, radius: int, color) -> None:
    """cv2.circle(img, center, radius, color, -1) for LINE_8 (in place)."""
    h, w = img.shape[:2]
    cx, cy = center
    col = np.asarray(color, img.dtype)

    def hline(y, x0, x1):
        if 0 <= y < h:
            x0, x1 = max(x0, 0), min(x1, w - 1)
            if x0 <= x1:
                img[y, x0:x1 + 1] = col

    err, dx, dy, plus, minus = 0, radius, 0, 1, 2 * radius - 1
    while dx >= dy:
        hline(cy - dy, cx - dx, cx + dx)
        hline(cy + dy, cx - dx, cx + dx)
        hline(cy - dx, cx - dy, cx + dy)
        hline(cy + dx, cx - dy, cx + dy)
        dy += 1
        err += plus
        plus += 2
        if err > 0:
            err -= minus
            dx -= 1
            minus -= 2


def add_weighted(src1, alpha, src2, beta, gamma=0.0):
    """cv2.addWeighted for uint8: float32 arithmetic, round half to even, saturate."""
    a, b, g = np.float32(alpha), np.float32(beta), np.float32(gamma)
    v = src1.astype(np.float32) * a + src2.astype(np.float32) * b + g
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def add_sun_flare(image, rng, flare_center=(100, 100), angle=-math.pi / 4, no_of_flare_circles=8,
                  src_radius=400, src_color=(255, 255, 255)):
    h, w = image.shape[:2]
    if angle != -1:
        angle = angle % (2 * math.pi)
    xs, ys = [], []
    for rx in range(0, w, 10):
        ry = math.tan(angle) * (rx - flare_center[0]) + flare_center[1]
        xs.append(rx)
        ys.append(2 * flare_center[1] - ry)
    overlay = image.copy()
    output = image.copy()
    for _ in range(no_of_flare_circles):
        alpha = rng.uniform(0.05, 0.2)
        r = rng.randint(0, len(xs) - 1)
        rad = rng.randint(1, h // 100 - 2)
        color = tuple(rng.randint(max(c - 50, 0), c) for c in src_color)
        circle_fill(overlay, (int(xs[r]), int(ys[r])), rad ** 3, color)
        output = add_weighted(overlay, alpha, output, 1 - alpha)
    overlay = output.copy()
    out2 = output.copy()
    n = src_radius // 10
    al = np.linspace(0.0, 1, num=n)
    rads = np.linspace(1, src_radius, num=n)
    for i in range(n):
        circle_fill(overlay, (int(flare_center[0]), int(flare_center[1])), int(rads[i]), src_color)
        a = al[n - i - 1] * al[n - i - 1] * al[n - i - 1]
        out2 = add_weighted(overlay, a, out2, 1 - a)
    return out2


def shader(img_bgr: np.ndarray, factor: float = 3.0) -> np.ndarray:
    """PIL ImageEnhance.Brightness(factor) of the RGB image (Pillow ImagingBlend vs black)."""
    rgb = img_bgr[..., ::-1].astype(np.float32)
    t = np.float32(factor) * rgb
    if 0.0 <= factor <= 1.0:
        return t.astype(np.int32).astype(np.uint8)
    return np.where(t <= 0, 0, np.where(t >= 255, 255, t)).astype(np.uint8)
