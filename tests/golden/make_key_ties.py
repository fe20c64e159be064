"""Triples of u8 RGB whose YCbCr values tie in exact arithmetic but differ in fp64 (test data for
tests/test_wavelet_gpu.py::test_wavelet_color_minmax_key_ties).

skimage's rgb2ycbcr (the wavelet's colour step, oracle/wavelet.py) is c = offset_c +
sum_k M[c, k] * (v_k / 255) with M = 65.481 128.553 24.966 / -37.797 -74.203 112.0 / 112.0 -93.786
-18.214: 1000 M is an integer matrix, so the exact value of a channel is an integer key
K_c = sum_k 1000 M[c, k] v_k.  Triples with equal keys have equal exact values, but their fp64
values (numpy's fma chain, oracle.cv.matmul3_fma) can differ in the last bits.  Over all 2^24
triples, per channel: the LOWEST and the HIGHEST key whose triples have more than one fp64 value;
of that key's triples, the first (in r, g, b order) with the smallest fp64 value and the first
with the largest.  Each such pair reaches its channel's extreme in an image whose other pixels lie
in [40, 200] (checked here), which is what the test needs.

  python tests/golden/make_key_ties.py       (prints the list; about 10 s)
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def find_ties():
    from oracle.cv import matmul3_fma
    from oracle.wavelet import YCBCR_FROM_RGB, YCBCR_OFFSET
    v = np.arange(1 << 24, dtype=np.int64)
    rgb = np.stack([v >> 16, (v >> 8) & 255, v & 255], axis=1)
    ycc = matmul3_fma(rgb.astype(np.float64) * (1.0 / 255.0), YCBCR_FROM_RGB, post=YCBCR_OFFSET)
    M1000 = np.rint(YCBCR_FROM_RGB * 1000).astype(np.int64)
    assert np.allclose(M1000, YCBCR_FROM_RGB * 1000, rtol=0, atol=1e-9)  # decimal matrix
    out = []
    lo40, hi200 = np.full(3, 40, np.int64), np.full(3, 200, np.int64)
    for c in range(3):
        key = rgb @ M1000[c]
        val = ycc[:, c]
        order = np.lexsort((v, val, key))  # by key, then fp64 value, then raster index
        k_s, f_s = key[order], val[order]
        start = np.r_[True, k_s[1:] != k_s[:-1]]
        gid = np.cumsum(start) - 1
        first = np.flatnonzero(start)
        last = np.r_[first[1:], len(k_s)] - 1
        tied = f_s[first] != f_s[last]  # a key with more than one fp64 value
        # cube-corner bounds of this channel over [40, 200]^3
        lo_k = int(np.where(M1000[c] > 0, lo40, hi200) @ M1000[c])
        hi_k = int(np.where(M1000[c] > 0, hi200, lo40) @ M1000[c])
        for g in (np.flatnonzero(tied)[0], np.flatnonzero(tied)[-1]):
            a = order[first[g]]
            # the first triple (raster order) with the group's largest value
            grp = order[first[g]:last[g] + 1]
            b = int(grp[f_s[first[g]:last[g] + 1] == f_s[last[g]]].min())
            assert key[a] < lo_k or key[a] > hi_k, "tie does not reach the extreme"
            out.append((tuple(int(t) for t in rgb[a]), tuple(int(t) for t in rgb[b])))
        del key, val, order, k_s, f_s, start, gid
    return out


if __name__ == "__main__":
    print(find_ties())
