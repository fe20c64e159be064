"""Host-side parameters of the `bloom` noise type: Automold.add_sun_flare (tools/Automold.py:588-627).

The reference's add_bloom (lib/model/test.py:1590-1594) calls
    am.add_sun_flare(img, flare_center=(100, 100), angle=-math.pi/4)
which draws 8 random flare circles (add_sun_process, Automold.py:575-586) and 40 concentric source
circles (flare_source, Automold.py:553-563), each followed by cv2.addWeighted(overlay, a, output,
1 - a, 0, output).  The random draws are host scalars taken from Python's `random` exactly as the
reference takes them (same calls, same order), so a seeded `random` gives the reference's
parameters.  The filled LINE_8 circles are described by per-radius half-width tables of OpenCV's
midpoint algorithm (imgproc/drawing.cpp Circle(), fill=1), and the GPU evaluates all 48 blends
per pixel in one pass (csrc/misc.hip bloom_kernel).
"""
from __future__ import annotations

import math
import random as _random
from functools import lru_cache
from typing import List, Sequence

import numpy as np

ERR_FLARE_CIRCLE_COUNT = "Numeric value between 0 and 20 is allowed"  # Automold.py:552


def circle_half_widths(R: int) -> List[int]:
    """half-width of OpenCV's filled LINE_8 circle of radius R at row offset 0..R."""
    half = [-1] * (R + 1)
    err, dx, dy, plus, minus = 0, R, 0, 1, (R << 1) - 1
    while dx >= dy:
        half[dy] = max(half[dy], dx)
        half[dx] = max(half[dx], dy)
        dy += 1
        err += plus
        plus += 2
        mask = (1 if err <= 0 else 0) - 1
        err -= minus & mask
        dx += mask
        minus -= mask & 2
    return half


@lru_cache(maxsize=4)
def span_table(rmax: int) -> np.ndarray:
    """int16 table: half-width of radius R at row offset t lives at R*(R+1)/2 + t."""
    out = np.zeros((rmax + 1) * (rmax + 2) // 2, np.int16)
    for R in range(rmax + 1):
        out[R * (R + 1) // 2: R * (R + 1) // 2 + R + 1] = circle_half_widths(R)
    return out


def add_sun_flare_line(flare_center, angle, imshape):
    """Automold.py:565-573"""
    x, y = [], []
    for rand_x in range(0, imshape[1], 10):
        rand_y = math.tan(angle) * (rand_x - flare_center[0]) + flare_center[1]
        x.append(rand_x)
        y.append(2 * flare_center[1] - rand_y)
    return x, y


def sun_flare_circles(h: int, w: int, flare_center=(100, 100), angle=-math.pi / 4,
                      no_of_flare_circles: int = 8, src_radius: int = 400,
                      src_color: Sequence[int] = (255, 255, 255), rng=None):
    """The 48 (circle, blend) steps of add_sun_flare for one image.

    Returns (circles int32 [k, 8] = cx, cy, radius, c0, c1, c2, reset_overlay, 0;
             weights float32 [k, 2] = addWeighted alpha, beta).  Draws from `rng` (default: the
    global `random`, like the reference)."""
    rng = rng or _random
    if angle != -1:
        angle = angle % (2 * math.pi)
    if not (0 <= no_of_flare_circles <= 20):
        raise Exception(ERR_FLARE_CIRCLE_COUNT)
    imshape = (h, w, 3)
    if angle == -1:
        angle_t = rng.uniform(0, 2 * math.pi)
        if angle_t == math.pi / 2:
            angle_t = 0
    else:
        angle_t = angle
    if flare_center == -1:
        flare_center_t = (rng.randint(0, imshape[1]), rng.randint(0, imshape[0] // 2))
    else:
        flare_center_t = flare_center
    x, y = add_sun_flare_line(flare_center_t, angle_t, imshape)
    circ, wts = [], []
    for _ in range(no_of_flare_circles):  # add_sun_process
        alpha = rng.uniform(0.05, 0.2)
        r = rng.randint(0, len(x) - 1)
        rad = rng.randint(1, imshape[0] // 100 - 2)
        color = (rng.randint(max(src_color[0] - 50, 0), src_color[0]),
                 rng.randint(max(src_color[1] - 50, 0), src_color[1]),
                 rng.randint(max(src_color[2] - 50, 0), src_color[2]))
        circ.append([int(x[r]), int(y[r]), rad * rad * rad, *color, 0, 0])
        wts.append([np.float32(alpha), np.float32(1 - alpha)])
    point = (int(flare_center_t[0]), int(flare_center_t[1]))  # flare_source
    num_times = src_radius // 10
    alpha = np.linspace(0.0, 1, num=num_times)
    rad = np.linspace(1, src_radius, num=num_times)
    for i in range(num_times):
        alp = alpha[num_times - i - 1] * alpha[num_times - i - 1] * alpha[num_times - i - 1]
        circ.append([point[0], point[1], int(rad[i]), *src_color, 1 if i == 0 else 0, 0])
        wts.append([np.float32(alp), np.float32(1 - alp)])
    return np.asarray(circ, np.int32).reshape(-1, 8), np.asarray(wts, np.float32).reshape(-1, 2)
