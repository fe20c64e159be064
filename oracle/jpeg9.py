"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

CPU restatement of `cv2.imread(path)` (IMREAD_COLOR -> uint8 BGR) for JPEG files, as the
reference's pinned stack decodes them: OpenCV 3.4.2 over IJG libjpeg 9d
(`/root/reference/requirements.txt:74,89`; call sites `lib/model/test.py:191`,
`lib/roi_data_layer/minibatch.py:85`).  libjpeg 9d is a third-party library absent from
/root/reference; its published algorithm is restated here:

  jdhuff.c     Huffman decoding: sequential (DC prediction, AC run/size, restart intervals) and
               progressive (decode_mcu_DC_first / _AC_first / _DC_refine / _AC_refine: spectral
               selection, successive approximation, EOB runs), one or several scans; a
               non-interleaved scan codes only the component's own blocks (width_in_blocks);
               damaged data as libjpeg treats it: zero bits past an interval's data, an MCU
               decoded only while the data lasted up to its start (insufficient_data), 17 bits
               and symbol 0 for a bad code, restart markers taken or resynchronised as
               jdmarker.c's jpeg_resync_to_restart does (_entropy, _intervals, _Bits)
  jdarith.c    arithmetic-coded files (SOF9 / SOF10): the QM-coder with libjpeg's statistics bins
               (DC 64 / AC 256 per table, reset per restart interval), the DC conditioning of the
               DAC parameters L / U and the AC split K; decode_mcu and the four progressive
               decoders (T.81 Table D.2 from oracle/jpeg_aritab.py)
  jdcoefct.c   progressive files are decoded into the whole coefficient buffer first; block
               smoothing (do_block_smoothing, smoothing_ok) then applies only if every component
               has DC data and nonzero quantisers Q00 Q01 Q10 Q20 Q11 Q02, and some component's AC
               coefficients 1..5 are not all known to full precision after the last scan (coef_bits
               != 0).  Encoders' standard scripts (jpeg_simple_progression) refine every one to
               Al = 0; files cut short of their last scans are smoothed: decompress_smooth_data
               estimates each still-zero AC01 AC10 AC20 AC11 AC02 from the 3x3 neighbourhood of
               quantised DC values (block_smooth below)
  jdmaster.c   IDCT scaling: with do_fancy_upsampling (the default) a component whose sampling
               factor divides the maximum by 2 gets a scaled IDCT of twice the size in that
               direction (libjpeg >= 7), so 4:2:0 chroma is decoded by jpeg_idct_16x16 and
               4:2:2 chroma by jpeg_idct_16x8 straight to full resolution; no upsampling pass
  jidctint.c   jpeg_idct_islow (8x8), jpeg_idct_16x16, jpeg_idct_16x8 (integer, CONST_BITS 13,
               PASS1_BITS 2, range centre folded into the DC term, 10-bit wrap range limit)
  jdcolor.c    ycc_rgb_convert with libjpeg 9's tables (FIX(1.402), FIX(1.772),
               FIX(0.714136286), FIX(0.344136286); SCALEBITS 16); RGB files (jdapimin.c
               default_decompress_parms: component IDs, JFIF / Adobe markers) are copied
OpenCV then swaps RGB -> BGR (grfmt_jpeg.cpp, no JCS_EXT_BGR in IJG libjpeg).

mode="turbo" instead restates libjpeg-turbo (the system Pillow's decoder): 8x8 IDCT for every
component, "fancy" triangular h2v1 / h2v2 upsampling (jdsample.c) and FIX(0.34414) for Cb->G.
(libjpeg-turbo >= 2.1 smooths differently -- nine coefficients from a 5x5 DC neighbourhood -- which
is not restated: mode="turbo" raises NotImplementedError for a file either library would smooth.)

Pinned by tests/golden/jpeg9.npz / jpeg9.json: the real libjpeg 9d decode of every fixture file
(tests/golden/make_jpeg9_fixtures.py, conda Pillow 8.4.0), and by jpeg9_damaged.* its decode of
168 damaged variants (tests/golden/make_jpeg_damaged.py); tests/test_jpeg.py checks this
restatement against both (and mode="turbo" against the system Pillow).
"""
from __future__ import annotations

import numpy as np

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
    20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58,
    59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])

CB, P1 = 13, 2  # CONST_BITS, PASS1_BITS


def FIX(x: float) -> int:
    return int(x * (1 << CB) + 0.5)


# ---- parsing + entropy decoding (jdmarker.c / jdhuff.c) ----------------------------------------
def _huff_lut(bits, vals):
    """16-bit peek -> (length, symbol)"""
    lut = [(0, 0)] * 65536
    code, k = 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln]):
            lo = code << (16 - ln)
            for x in range(lo, lo + (1 << (16 - ln))):
                lut[x] = (ln, vals[k])
            code += 1
            k += 1
        code <<= 1
    return lut


def _extend(v, s):
    return v - (1 << s) + 1 if v < (1 << (s - 1)) else v


def _entropy(data: bytes, i: int):
    """the entropy-coded data from data[i] as libjpeg's source manager delivers it: a list of
    segments (unstuffed bytes, code of the marker that ends them), up to the first marker that is
    neither RSTn nor below SOF0 (a valid non-restart marker, jdmarker.c resync_to_restart's
    action 3), and the index of that marker.  Stuffed 0xFF00 -> 0xFF, fill 0xFFs are skipped; the
    end of the data is jdatasrc.c's inserted EOI (JWRN_JPEG_EOF)."""
    segs, cur = [], bytearray()
    while True:
        if i >= len(data):
            segs.append((bytes(cur), 0xD9))
            return segs, len(data)
        b = data[i]
        if b != 0xFF:
            cur.append(b)
            i += 1
            continue
        j = i + 1
        while j < len(data) and data[j] == 0xFF:
            j += 1
        if j >= len(data):
            segs.append((bytes(cur), 0xD9))
            return segs, len(data)
        if data[j] == 0x00:
            cur.append(0xFF)
            i = j + 1
            continue
        segs.append((bytes(cur), data[j]))
        cur = bytearray()
        if not (0xD0 <= data[j] <= 0xD7 or data[j] < 0xC0):
            return segs, j - 1
        i = j + 1


def _intervals(segs, restart: int, n: int):
    """the data each of the scan's n restart intervals decodes, as libjpeg reads them: interval 0
    the first segment; at every restart, jdhuff.c process_restart -> jdmarker.c
    read_restart_marker: the marker that ends the current segment is the expected RSTn (taken,
    the next segment follows), or jpeg_resync_to_restart decides -- action 1 (the expected one, or
    one too far away) take it; action 2 (a marker below SOF0 or one of the two RSTs before the
    expected one) skip to the marker after the next segment and decide again; action 3 (a valid
    non-restart marker or one of the next two RSTs) leave it: the interval reads nothing.  Yields
    (bytes, reset) -- reset: the out-of-data flag is cleared (the marker was taken)."""
    j, stuck, want = 0, False, 0
    yield segs[0][0], True
    for _ in range(1, n if restart else 1):
        m = segs[min(j, len(segs) - 1)][1]
        while True:
            if m == 0xD0 + want:
                act = 1
            elif m < 0xC0:
                act = 2
            elif not 0xD0 <= m <= 0xD7:
                act = 3
            elif m in (0xD0 + ((want + 1) & 7), 0xD0 + ((want + 2) & 7)):
                act = 3
            elif m in (0xD0 + ((want - 1) & 7), 0xD0 + ((want - 2) & 7)):
                act = 2
            else:
                act = 1
            if act == 2 and j + 1 < len(segs):
                j += 1
                m = segs[j][1]
                continue
            break
        want = (want + 1) & 7
        if act == 1 and j + 1 < len(segs):
            j += 1
            yield segs[j][0], True
        else:  # the marker stays unread: this interval's segment is empty
            yield b"", False


class _Bits:
    """big-endian bit reader over one restart interval's bytes; zeros past their end (jdhuff.c
    jpeg_fill_bit_buffer), and `out` set once a read needed a bit past the end (the entropy
    decoder's insufficient_data)"""

    def __init__(self, buf: bytes, out: bool = False):
        self.avail = 8 * len(buf)
        self.v = int.from_bytes(buf, "big")
        self.n = self.avail
        self.pos = 0
        self.out = out

    def _ensure(self, k):
        while self.pos + k > self.n:
            self.v <<= 64
            self.n += 64

    def _take(self, k):
        self._ensure(k)
        r = (self.v >> (self.n - self.pos - k)) & ((1 << k) - 1)
        self.pos += k
        if self.pos > self.avail:
            self.out = True
        return r

    def get(self, s):
        return self._take(s) if s else 0

    def huff(self, lut):
        """one symbol; a bit pattern that is no code (jpeg_huff_decode's l > 16) takes 17 bits and
        decodes as 0 (JWRN_HUFF_BAD_CODE)"""
        self._ensure(16)
        ln, sym = lut[(self.v >> (self.n - self.pos - 16)) & 0xFFFF]
        self._take(ln if ln else 17)
        return sym


def _nat(k):
    """jpeg_natural_order with libjpeg's overrun guard (indices past 63 map to 63)"""
    return ZIGZAG[min(k, 63)]


def _decode_scan(sc, comps, coef, geo, dc, ac):
    """one scan (jdhuff.c: sequential decode_mcu, or the progressive decode_mcu_DC_first /
    _AC_first / _DC_refine / _AC_refine) into the coefficient arrays (natural order, int64)"""
    Ss, Se, Ah, Al = sc["Ss"], sc["Se"], sc["Ah"], sc["Al"]
    sel = sc["sel"]  # [(component index, td, ta)]
    prog = sc["progressive"]
    if len(sel) == 1:  # non-interleaved: the component's own blocks, MCU = one block
        ci = sel[0][0]
        bw, bh = geo["wib"][ci], geo["hib"][ci]
        units = [[(ci, by, bx)] for by in range(bh) for bx in range(bw)]
    else:
        units = []
        for my in range(geo["mcuy"]):
            for mx in range(geo["mcux"]):
                units.append([(ci, my * comps[ci]["v"] + dv, mx * comps[ci]["h"] + dh)
                              for ci, _, _ in sel for dv in range(comps[ci]["v"])
                              for dh in range(comps[ci]["h"])])
    tabs = {ci: (dc.get(td), ac.get(ta)) for ci, td, ta in sel}
    per = sc["restart"] if sc["restart"] else len(units)
    p1, m1 = 1 << Al, -(1 << Al)
    u = 0
    out = False
    nint = -(-len(units) // per)
    for iv, reset in _intervals(sc["segments"], sc["restart"], nint):
        if u >= len(units):
            break
        br = _Bits(iv, out and not reset)
        pred = {ci: 0 for ci, _, _ in sel}
        eobrun = 0
        for _ in range(min(per, len(units) - u)):
            if br.out:  # out of data: the MCU is left as it is (zeros / the earlier scans)
                u += 1
                continue
            for ci, by, bx in units[u]:
                blk = coef[ci][by, bx]
                dct, act = tabs[ci]
                if not prog:  # sequential: DC then AC of the block
                    s = br.huff(dct)
                    pred[ci] += _extend(br.get(s), s) if s else 0
                    blk[0] = pred[ci]
                    k = 1
                    while k < 64:
                        rs = br.huff(act)
                        r, s = rs >> 4, rs & 15
                        if s:
                            k += r
                            blk[_nat(k)] = _extend(br.get(s), s)
                            k += 1
                        elif r == 15:
                            k += 16
                        else:
                            break
                elif Ss == 0 and Ah == 0:  # DC first
                    s = br.huff(dct)
                    pred[ci] += _extend(br.get(s), s) if s else 0
                    blk[0] = pred[ci] << Al
                elif Ss == 0:  # DC refine
                    if br.get(1):
                        blk[0] |= p1
                elif Ah == 0:  # AC first
                    if eobrun:
                        eobrun -= 1
                        continue
                    k = Ss
                    while k <= Se:
                        rs = br.huff(act)
                        r, s = rs >> 4, rs & 15
                        if s:
                            k += r
                            blk[_nat(k)] = _extend(br.get(s), s) << Al
                        elif r != 15:
                            eobrun = (1 << r) + (br.get(r) if r else 0) - 1
                            break
                        else:
                            k += 15
                        k += 1
                else:  # AC refine
                    k = Ss
                    if eobrun == 0:
                        while k <= Se:
                            rs = br.huff(act)
                            r, s = rs >> 4, rs & 15
                            if s:
                                s = p1 if br.get(1) else m1
                            elif r != 15:
                                eobrun = (1 << r) + (br.get(r) if r else 0)
                                break
                            while k <= Se:
                                pos = _nat(k)
                                if blk[pos]:
                                    if br.get(1) and (blk[pos] & p1) == 0:
                                        blk[pos] += p1 if blk[pos] >= 0 else m1
                                else:
                                    r -= 1
                                    if r < 0:
                                        break
                                k += 1
                            if s:
                                blk[_nat(k)] = s
                            k += 1
                    if eobrun > 0:
                        while k <= Se:
                            pos = _nat(k)
                            if blk[pos] and br.get(1) and (blk[pos] & p1) == 0:
                                blk[pos] += p1 if blk[pos] >= 0 else m1
                            k += 1
                        eobrun -= 1
            u += 1
        out = br.out


# ---- arithmetic decoding (jdarith.c, libjpeg 9d) -------------------------------------------------
from oracle.jpeg_aritab import ARITAB  # noqa: E402  (T.81 Table D.2, generated)


class _Arith:
    """the QM-coder decoder over one restart interval's (unstuffed) bytes; past their end it reads
    0 (libjpeg supplies zeros once the interval's marker is reached)"""

    def __init__(self, buf: bytes):
        self.buf, self.i = buf, 0
        self.c, self.a, self.ct = 0, 0, -16  # force reading 2 initial bytes

    def decode(self, st, k):
        """arith_decode on statistics bin st[k] (a bytearray slot)"""
        while self.a < 0x8000:
            self.ct -= 1
            if self.ct < 0:
                data = self.buf[self.i] if self.i < len(self.buf) else 0
                self.i += 1
                self.c = (self.c << 8) | data
                self.ct += 8
                if self.ct < 0:
                    self.ct += 1
                    if self.ct == 0:
                        self.a = 0x8000  # got 2 initial bytes: a = 0x10000 after the shift
            self.a <<= 1
        sv = st[k]
        qe = ARITAB[sv & 0x7F]
        nl, nm, qe = qe & 0xFF, (qe >> 8) & 0xFF, qe >> 16
        temp = self.a - qe
        self.a = temp
        temp <<= self.ct
        if self.c >= temp:
            self.c -= temp
            if self.a < qe:  # conditional LPS exchange
                self.a = qe
                st[k] = (sv & 0x80) ^ nm
            else:
                self.a = qe
                st[k] = (sv & 0x80) ^ nl
                sv ^= 0x80
        elif self.a < 0x8000:  # conditional MPS exchange
            if self.a < qe:
                st[k] = (sv & 0x80) ^ nl
                sv ^= 0x80
            else:
                st[k] = (sv & 0x80) ^ nm
        return sv >> 7


class _BadCode(Exception):
    """jdarith.c's JWRN_ARITH_BAD_CODE: the rest of the interval decodes nothing (ct = -1)"""


def _arith_dc_diff(ar, dcs, ci, ctx, L, U):
    """Figures F.19 / F.21-F.24: a DC difference, updating the conditioning ctx[ci]"""
    s0 = ctx[ci]
    if ar.decode(dcs, s0) == 0:
        ctx[ci] = 0
        return 0
    sign = ar.decode(dcs, s0 + 1)
    st = s0 + 2 + sign
    m = ar.decode(dcs, st)
    if m:
        st = 20  # X1
        while ar.decode(dcs, st):
            m <<= 1
            if m == 0x8000:
                raise _BadCode
            st += 1
    if m < (1 << L) >> 1:
        ctx[ci] = 0
    elif m > (1 << U) >> 1:
        ctx[ci] = 12 + sign * 4
    else:
        ctx[ci] = 4 + sign * 4
    v = m
    st += 14
    m >>= 1
    while m:
        if ar.decode(dcs, st):
            v |= m
        m >>= 1
    v += 1
    return -v if sign else v


def _arith_ac_value(ar, acs, st, k, K, fixed):
    """Figures F.21-F.24 for an AC coefficient whose statistics run starts at st (= 3 (k - 1))"""
    sign = ar.decode(fixed, 0)
    st += 2
    m = ar.decode(acs, st)
    if m:
        if ar.decode(acs, st):
            m <<= 1
            st = 189 if k <= K else 217
            while ar.decode(acs, st):
                m <<= 1
                if m == 0x8000:
                    raise _BadCode
                st += 1
    v = m
    st += 14
    m >>= 1
    while m:
        if ar.decode(acs, st):
            v |= m
        m >>= 1
    v += 1
    return -v if sign else v


def _decode_scan_arith(sc, comps, coef, geo, dac):
    """one arithmetic-coded scan (jdarith.c decode_mcu, decode_mcu_DC_first / _AC_first /
    _DC_refine / _AC_refine): statistics bins per table, reset with the DC predictions and the
    conditioning at every restart interval"""
    Ss, Se, Ah, Al = sc["Ss"], sc["Se"], sc["Ah"], sc["Al"]
    sel = sc["sel"]
    prog = sc["progressive"]
    if len(sel) == 1:
        ci = sel[0][0]
        units = [[(ci, by, bx)] for by in range(geo["hib"][ci]) for bx in range(geo["wib"][ci])]
    else:
        units = []
        for my in range(geo["mcuy"]):
            for mx in range(geo["mcux"]):
                units.append([(ci, my * comps[ci]["v"] + dv, mx * comps[ci]["h"] + dh)
                              for ci, _, _ in sel for dv in range(comps[ci]["v"])
                              for dh in range(comps[ci]["h"])])
    tbl = {ci: (td, ta) for ci, td, ta in sel}
    per = sc["restart"] if sc["restart"] else len(units)
    p1, m1 = 1 << Al, -(1 << Al)
    u = 0
    for iv, _ in _intervals(sc["segments"], sc["restart"], -(-len(units) // per)):
        if u >= len(units):
            break
        ar = _Arith(iv)
        dcs = {t: bytearray(64) for t in range(16)}
        acs = {t: bytearray(256) for t in range(16)}
        fixed = bytearray([113])
        last = {ci: 0 for ci, _, _ in sel}
        ctx = {ci: 0 for ci, _, _ in sel}
        bad = False
        for _ in range(min(per, len(units) - u)):
            if bad:
                u += 1
                continue
            try:
                for ci, by, bx in units[u]:
                    blk = coef[ci][by, bx]
                    td, ta = tbl[ci]
                    if not prog or (Ss == 0 and Ah == 0):  # DC of a sequential / DC-first scan
                        last[ci] += _arith_dc_diff(ar, dcs[td], ci, ctx, dac["L"][td], dac["U"][td])
                        blk[0] = last[ci] << (Al if prog else 0)
                        if prog:
                            continue
                        k = 0  # sequential: the AC coefficients 1..63
                        while k < 63:
                            st = 3 * k
                            if ar.decode(acs[ta], st):
                                break  # EOB
                            while True:
                                k += 1
                                if ar.decode(acs[ta], st + 1):
                                    break
                                st += 3
                                if k >= 63:
                                    raise _BadCode
                            blk[_nat(k)] = _arith_ac_value(ar, acs[ta], st, k, dac["K"][ta], fixed)
                    elif Ss == 0:  # DC refine: the next bit of the two's-complement value
                        if ar.decode(fixed, 0):
                            blk[0] |= p1
                    elif Ah == 0:  # AC first
                        k = Ss - 1
                        while k < Se:
                            st = 3 * k
                            if ar.decode(acs[ta], st):
                                break
                            while True:
                                k += 1
                                if ar.decode(acs[ta], st + 1):
                                    break
                                st += 3
                                if k >= Se:
                                    raise _BadCode
                            blk[_nat(k)] = _arith_ac_value(ar, acs[ta], st, k, dac["K"][ta],
                                                           fixed) << Al
                    else:  # AC refine
                        kex = Se
                        while kex > 0 and not blk[_nat(kex)]:
                            kex -= 1
                        k = Ss - 1
                        while k < Se:
                            st = 3 * k
                            if k >= kex and ar.decode(acs[ta], st):
                                break
                            while True:
                                k += 1
                                pos = _nat(k)
                                if blk[pos]:
                                    if ar.decode(acs[ta], st + 2):
                                        blk[pos] += m1 if blk[pos] < 0 else p1
                                    break
                                if ar.decode(acs[ta], st + 1):
                                    blk[pos] = m1 if ar.decode(fixed, 0) else p1
                                    break
                                st += 3
                                if k >= Se:
                                    raise _BadCode
            except _BadCode:
                bad = True
            u += 1


def parse_and_decode(data: bytes):
    """-> dict(width, height, comps=[(h, v, q[64] natural)], coef=[int64 (bh, bw, 64) natural])

    Baseline / extended sequential (SOF0 / SOF1) and progressive (SOF2) Huffman files, one or
    several scans (tables and the restart interval may change between scans)."""
    assert data[:2] == b"\xff\xd8", "no SOI"
    q, dc, ac, comps, restart = {}, {}, {}, [], 0
    jfif, adobe = False, None
    arith = False
    # arithmetic conditioning per table (jdmarker.c get_soi defaults: L 0, U 1, K 5)
    dac = dict(L=[0] * 16, U=[1] * 16, K=[5] * 16)
    W = H = 0
    progressive = None
    coef = geo = None
    i = 2
    while i + 4 <= len(data):
        assert data[i] == 0xFF
        m = data[i + 1]
        if m == 0xFF:
            i += 1
            continue
        i += 2
        if m == 0xD8 or 0xD0 <= m <= 0xD7 or m == 0x01:
            continue
        if m == 0xD9:
            break
        ln = (data[i] << 8) | data[i + 1]
        s = data[i + 2:i + ln]
        end = i + ln
        if m in (0xC0, 0xC1, 0xC2, 0xC9, 0xCA):
            assert s[0] == 8
            progressive = m in (0xC2, 0xCA)
            arith = m in (0xC9, 0xCA)
            H, W, nc = (s[1] << 8) | s[2], (s[3] << 8) | s[4], s[5]
            comps = [dict(id=s[6 + 3 * c], h=s[7 + 3 * c] >> 4, v=s[7 + 3 * c] & 15,
                          tq=s[8 + 3 * c]) for c in range(nc)]
            if nc == 1:
                comps[0]["h"] = comps[0]["v"] = 1
            hmax = max(c["h"] for c in comps)
            vmax = max(c["v"] for c in comps)
            mcux, mcuy = -(-W // (8 * hmax)), -(-H // (8 * vmax))
            # blocks of each component that carry data (jdinput.c width_in_blocks): what a
            # non-interleaved scan codes
            geo = dict(mcux=mcux, mcuy=mcuy, hmax=hmax, vmax=vmax,
                       wib=[-(-(-(-W * c["h"] // hmax)) // 8) for c in comps],
                       hib=[-(-(-(-H * c["v"] // vmax)) // 8) for c in comps])
            coef = [np.zeros((mcuy * c["v"], mcux * c["h"], 64), np.int64) for c in comps]
            cbits = [[-1] * 6 for _ in comps]
        elif m == 0xC4:
            k = 0
            while k < len(s):
                tc, th = s[k] >> 4, s[k] & 15
                bits = [0] + list(s[k + 1:k + 17])
                n = sum(bits)
                tbl = _huff_lut(bits, list(s[k + 17:k + 17 + n]))
                (ac if tc else dc)[th] = tbl
                k += 17 + n
        elif m == 0xDB:
            k = 0
            while k < len(s):
                pq, tq = s[k] >> 4, s[k] & 15
                if pq:
                    z = [(s[k + 1 + 2 * i2] << 8) | s[k + 2 + 2 * i2] for i2 in range(64)]
                else:
                    z = list(s[k + 1:k + 65])
                nat = np.zeros(64, np.int64)
                nat[ZIGZAG] = z
                q[tq] = nat
                k += 1 + 64 * (2 if pq else 1)
        elif m == 0xDD:
            restart = (s[0] << 8) | s[1]
        elif m == 0xE0 and len(s) >= 14 and s[:5] == b"JFIF\0":  # jdmarker.c examine_app0
            jfif = True
        elif m == 0xEE and len(s) >= 12 and s[:5] == b"Adobe":   # examine_app14
            adobe = s[11]
        elif m in (0xDE, 0xDF) or 0xF0 <= m <= 0xFD:
            raise ValueError("reserved / extension marker (DHP, EXP, JPGn, LSE) not supported")
        elif m == 0xDA:
            ns = s[0]
            sel = []
            for k in range(ns):
                c = [cc["id"] for cc in comps].index(s[1 + 2 * k])
                sel.append((c, s[2 + 2 * k] >> 4, s[2 + 2 * k] & 15))
            ss = s[1 + 2 * ns:]
            segments, end = _entropy(data, end)
            sc = dict(sel=sel, Ss=ss[0], Se=ss[1], Ah=ss[2] >> 4, Al=ss[2] & 15,
                      progressive=progressive, restart=restart, segments=segments)
            if arith:
                _decode_scan_arith(sc, comps, coef, geo, dac)
            else:
                _decode_scan(sc, comps, coef, geo, dc, ac)
            for ci, _, _ in sel:  # jdphuff.c start_pass: coef_bits[k] = Al for k in Ss..Se
                for k in range(sc["Ss"], min(sc["Se"], 5) + 1):
                    cbits[ci][k] = sc["Al"]
        elif m == 0xCC:  # DAC (jdmarker.c get_dac): conditioning of arithmetic tables
            for k in range(0, len(s) - 1, 2):
                idx, val = s[k], s[k + 1]
                if idx >= 32:
                    raise ValueError("bad DAC table index")
                if idx >= 16:
                    dac["K"][idx - 16] = val
                else:
                    dac["L"][idx], dac["U"][idx] = val & 15, val >> 4
                    if dac["L"][idx] > dac["U"][idx]:
                        raise ValueError("bad DAC value")
        elif 0xC3 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            raise ValueError("lossless / hierarchical JPEG not supported")
        i = end
    assert coef is not None, "no frame"
    # jdcoefct.c smoothing_ok (libjpeg 9d): FALSE unless EVERY component has DC data and nonzero
    # quantisers Q00 Q01 Q10 Q20 Q11 Q02; then TRUE if some component's AC 1..5 stay imprecise
    smoothing_ok = progressive and all(
        cb[0] >= 0 and all(q[c["tq"]][i] != 0 for i in (0, 1, 8, 16, 9, 2))
        for cb, c in zip(cbits, comps)) and any(any(b != 0 for b in cb[1:]) for cb in cbits)
    return dict(width=W, height=H, hmax=geo["hmax"], vmax=geo["vmax"],
                comps=[(c["h"], c["v"], q[c["tq"]]) for c in comps], coef=coef,
                smooth=cbits if smoothing_ok else None, wib=geo["wib"], hib=geo["hib"],
                cids=[c["id"] for c in comps], jfif=jfif, adobe=adobe)


def cv_cmyk_to_bgr(cmyk):
    """OpenCV 3.4.2 icvCvt_CMYK2BGR_8u_C4C3R (imgcodecs utils.cpp, what grfmt_jpeg.cpp applies
    to libjpeg's JCS_CMYK output of a 4-component file): Adobe-inverted CMYK,
    c' = k - ((255 - c) k >> 8), written as B = y', G = m', R = c'.  (Restated from the
    published source; cv2 is not importable here, so this step is parity-unpinned.)"""
    c = cmyk.astype(np.int64)
    k = c[..., 3]
    out = [k - (((255 - c[..., j]) * k) >> 8) for j in (2, 1, 0)]
    return np.stack(out, -1).astype(np.uint8)


def color_space(d, mode: str) -> str:
    """jdapimin.c default_decompress_parms for 3 components: "ycc" (converted) or "rgb" (copied).
    libjpeg 9 decides by the component IDs first -- (1, 2, 3) YCbCr, (1, 0x22, 0x23) / 'r' 'g' 'b'
    big gamut (not restated), 'R' 'G' 'B' RGB -- then a JFIF marker (YCbCr), then Adobe's transform
    (0 RGB, else YCbCr), else YCbCr; libjpeg-turbo (6b's order) by JFIF, then Adobe, then the IDs
    'R' 'G' 'B', else YCbCr"""
    if len(d["cids"]) == 4:  # Adobe transform 0: CMYK as stored, else YCCK; no marker: CMYK
        return "ycck" if d["adobe"] not in (None, 0) else "cmyk"
    if len(d["cids"]) != 3:
        return "gray"
    ids = tuple(d["cids"])
    rgb_ids = ids == (0x52, 0x47, 0x42)
    adobe = None if d["adobe"] is None else ("rgb" if d["adobe"] == 0 else "ycc")
    if mode == "libjpeg9":
        if ids == (1, 2, 3):
            return "ycc"
        if ids in ((1, 0x22, 0x23), (0x72, 0x67, 0x62)):
            raise ValueError("big-gamut (BG_YCC / BG_RGB) JPEG not supported")
        if rgb_ids:
            return "rgb"
        if d["jfif"]:
            return "ycc"
        return adobe or "ycc"
    if d["jfif"]:
        return "ycc"
    if adobe:
        return adobe
    return "rgb" if rgb_ids else "ycc"


# jdcoefct.c decompress_smooth_data (libjpeg 9d): (coef_bits index = zigzag k, natural position,
# multiplier, the DC neighbourhood term) per estimated coefficient; DC1..DC9 are the quantised DC
# values of the 3x3 blocks around the current one (DC5), row by row
_SMOOTH = ((1, 1, 36, lambda d: d[4] - d[6]),                 # AC01
           (2, 8, 36, lambda d: d[2] - d[8]),                 # AC10
           (3, 16, 9, lambda d: d[2] + d[8] - 2 * d[5]),      # AC20
           (4, 9, 5, lambda d: d[1] - d[3] - d[7] + d[9]),    # AC11
           (5, 2, 9, lambda d: d[4] + d[6] - 2 * d[5]))       # AC02


def block_smooth(cf, q, cbits, wib: int, hib: int):
    """libjpeg 9d block smoothing of one component's quantised coefficients cf (bh, bw, 64)
    (jdcoefct.c decompress_smooth_data): over the blocks that carry data (width_in_blocks x
    height_in_blocks; the neighbourhood repeats the edge blocks), a coefficient whose coef_bits
    latch Al != 0 and whose value is still 0 becomes
        pred = ((Q_k << 7) + |num|) // (Q_k << 8),  num = mult * Q00 * term(DC1..DC9),
    capped at 2^Al - 1 when Al > 0, with the sign of num.  Works on a copy (the estimates never
    feed a neighbour)."""
    out = cf.copy()
    dc = cf[:hib, :wib, 0].astype(np.int64)
    pad = np.pad(dc, 1, mode="edge")
    d = [None] + [pad[r:r + hib, c:c + wib] for r in range(3) for c in range(3)]
    q00 = int(q[0])
    for k, pos, mult, term in _SMOOTH:
        al = cbits[k]
        if al == 0:
            continue
        qk = int(q[pos])
        num = mult * q00 * term(d)
        pred = ((qk << 7) + np.abs(num)) // (qk << 8)
        if al > 0:
            pred = np.minimum(pred, (1 << al) - 1)
        pred = np.where(num >= 0, pred, -pred)
        pred = ((pred + 32768) & 0xFFFF) - 32768  # (JCOEF) pred: a 16-bit store
        cur = out[:hib, :wib, pos]
        out[:hib, :wib, pos] = np.where(cur == 0, pred, cur)
    return out


# ---- IDCT kernels (jidctint.c) -------------------------------------------------------------------
# 1-D kernels over the last axis (8 inputs).  `first`: pass 1 (x0 << CONST_BITS plus the pass-1
# fudge; outputs >> CONST_BITS - PASS1_BITS); else pass 2 (range centre + fudge added to the DC
# workspace value, outputs >> CONST_BITS + PASS1_BITS + 3).
def _dc_term(x0, first):
    if first:
        return (x0 << CB) + (1 << (CB - P1 - 1))
    return (x0 + ((512 << (P1 + 3)) + (1 << (P1 + 2)))) << CB


def _idct8(x, first):
    x = [x[..., k] for k in range(8)]
    z2, z3 = x[2], x[6]
    z1 = (z2 + z3) * FIX(0.541196100)
    tmp2 = z1 + z2 * FIX(0.765366865)
    tmp3 = z1 - z3 * FIX(1.847759065)
    z2 = _dc_term(x[0], first)
    z3 = x[4] << CB
    tmp0, tmp1 = z2 + z3, z2 - z3
    tmp10, tmp13, tmp11, tmp12 = tmp0 + tmp2, tmp0 - tmp2, tmp1 + tmp3, tmp1 - tmp3
    tmp0, tmp1, tmp2, tmp3 = x[7], x[5], x[3], x[1]
    z2, z3 = tmp0 + tmp2, tmp1 + tmp3
    z1 = (z2 + z3) * FIX(1.175875602)
    z2 = z2 * -FIX(1.961570560) + z1
    z3 = z3 * -FIX(0.390180644) + z1
    z1 = (tmp0 + tmp3) * -FIX(0.899976223)
    tmp0 = tmp0 * FIX(0.298631336) + z1 + z2
    tmp3 = tmp3 * FIX(1.501321110) + z1 + z3
    z1 = (tmp1 + tmp2) * -FIX(2.562915447)
    tmp1 = tmp1 * FIX(2.053119869) + z1 + z3
    tmp2 = tmp2 * FIX(3.072711026) + z1 + z2
    sh = CB - P1 if first else CB + P1 + 3
    o = [tmp10 + tmp3, tmp11 + tmp2, tmp12 + tmp1, tmp13 + tmp0,
         tmp13 - tmp0, tmp12 - tmp1, tmp11 - tmp2, tmp10 - tmp3]
    return np.stack([v >> sh for v in o], -1)


def _idct16(x, first):
    x = [x[..., k] for k in range(8)]
    tmp0 = _dc_term(x[0], first)
    z1 = x[4]
    tmp1, tmp2 = z1 * FIX(1.306562965), z1 * FIX(0.541196100)
    tmp10, tmp11, tmp12, tmp13 = tmp0 + tmp1, tmp0 - tmp1, tmp0 + tmp2, tmp0 - tmp2
    z1, z2 = x[2], x[6]
    z3 = z1 - z2
    z4 = z3 * FIX(0.275899379)
    z3 = z3 * FIX(1.387039845)
    tmp0 = z3 + z2 * FIX(2.562915447)
    tmp1 = z4 + z1 * FIX(0.899976223)
    tmp2 = z3 - z1 * FIX(0.601344887)
    tmp3 = z4 - z2 * FIX(0.509795579)
    tmp20, tmp27 = tmp10 + tmp0, tmp10 - tmp0
    tmp21, tmp26 = tmp12 + tmp1, tmp12 - tmp1
    tmp22, tmp25 = tmp13 + tmp2, tmp13 - tmp2
    tmp23, tmp24 = tmp11 + tmp3, tmp11 - tmp3
    z1, z2, z3, z4 = x[1], x[3], x[5], x[7]
    tmp11 = z1 + z3
    tmp1 = (z1 + z2) * FIX(1.353318001)
    tmp2 = tmp11 * FIX(1.247225013)
    tmp3 = (z1 + z4) * FIX(1.093201867)
    tmp10 = (z1 - z4) * FIX(0.897167586)
    tmp11 = tmp11 * FIX(0.666655658)
    tmp12 = (z1 - z2) * FIX(0.410524528)
    tmp0 = tmp1 + tmp2 + tmp3 - z1 * FIX(2.286341144)
    tmp13 = tmp10 + tmp11 + tmp12 - z1 * FIX(1.835730603)
    z1 = (z2 + z3) * FIX(0.138617169)
    tmp1 = tmp1 + z1 + z2 * FIX(0.071888074)
    tmp2 = tmp2 + z1 - z3 * FIX(1.125726048)
    z1 = (z3 - z2) * FIX(1.407403738)
    tmp11 = tmp11 + z1 - z3 * FIX(0.766367282)
    tmp12 = tmp12 + z1 + z2 * FIX(1.971951411)
    z2 = z2 + z4
    z1 = z2 * -FIX(0.666655658)
    tmp1 = tmp1 + z1
    tmp3 = tmp3 + z1 + z4 * FIX(1.065388962)
    z2 = z2 * -FIX(1.247225013)
    tmp10 = tmp10 + z2 + z4 * FIX(3.141271809)
    tmp12 = tmp12 + z2
    z2 = (z3 + z4) * -FIX(1.353318001)
    tmp2 = tmp2 + z2
    tmp3 = tmp3 + z2
    z2 = (z4 - z3) * FIX(0.410524528)
    tmp10 = tmp10 + z2
    tmp11 = tmp11 + z2
    sh = CB - P1 if first else CB + P1 + 3
    lo = [tmp20 + tmp0, tmp21 + tmp1, tmp22 + tmp2, tmp23 + tmp3,
          tmp24 + tmp10, tmp25 + tmp11, tmp26 + tmp12, tmp27 + tmp13]
    hi = [tmp27 - tmp13, tmp26 - tmp12, tmp25 - tmp11, tmp24 - tmp10,
          tmp23 - tmp3, tmp22 - tmp2, tmp21 - tmp1, tmp20 - tmp0]
    return np.stack([v >> sh for v in lo + hi], -1)


def _range_limit(v):
    """IDCT_range_limit[(x) & RANGE_MASK]: (x + 512) & 1023, minus RANGE_SUBSET 384, clamped"""
    return np.clip((v & 1023) - 384, 0, 255).astype(np.uint8)


def idct_blocks(coef, q, rows: int, cols: int):
    """coef (..., 64) natural order, q (64,) -> (..., rows, cols) u8; rows, cols in {8, 16}"""
    x = (coef * q).reshape(coef.shape[:-1] + (8, 8))
    col = _idct16 if rows == 16 else _idct8
    row = _idct16 if cols == 16 else _idct8
    ws = col(np.swapaxes(x, -1, -2), True)   # (..., 8 cols, rows) — pass 1 down each column
    ws = np.swapaxes(ws, -1, -2)             # (..., rows, 8)
    return _range_limit(row(ws, False))      # (..., rows, cols)


def _fancy_h2v1(p, dw):
    p = p.astype(np.int64)
    out = np.empty(p.shape[:-1] + (2 * p.shape[-1],), np.int64)
    left = np.concatenate([p[..., :1], p[..., :-1]], -1)
    right = np.concatenate([p[..., 1:], p[..., -1:]], -1)
    out[..., 0::2] = (p * 3 + left + 1) >> 2
    out[..., 1::2] = (p * 3 + right + 2) >> 2
    out[..., 0] = p[..., 0]
    out[..., 2 * dw - 1] = p[..., dw - 1]
    return out


def _fancy_h2v2(p, dw, dh):
    p = p.astype(np.int64)
    above = np.concatenate([p[:1], p[:-1]], 0)
    below = np.concatenate([p[1:dh], p[dh - 1:dh], p[dh:]], 0)[:p.shape[0]]
    out = np.empty((2 * p.shape[0], 2 * p.shape[1]), np.int64)
    for par, nb in ((0, above), (1, below)):
        cs = p * 3 + nb
        left = np.concatenate([cs[:, :1], cs[:, :-1]], 1)
        right = np.concatenate([cs[:, 1:], cs[:, -1:]], 1)
        ev = (cs * 3 + left + 8) >> 4
        od = (cs * 3 + right + 7) >> 4
        ev[:, 0] = (cs[:, 0] * 4 + 8) >> 4
        od[:, dw - 1] = (cs[:, dw - 1] * 4 + 7) >> 4
        out[par::2, 0::2] = ev
        out[par::2, 1::2] = od
    return out


def imread(data: bytes, mode: str = "libjpeg9", orientation: bool = True) -> np.ndarray:
    """cv2.imread(..., IMREAD_COLOR) of a JPEG: (H, W, 3) uint8 BGR, turned by the file's EXIF
    orientation as OpenCV 3.4.2 does (oracle/exif.py; orientation=False:
    IMREAD_IGNORE_ORIENTATION)"""
    img = decode(data, mode)
    if orientation:
        from . import exif
        img = exif.apply(img, exif.orientation(data))
    return img


def decode(data: bytes, mode: str = "libjpeg9") -> np.ndarray:
    """the library's decode of a JPEG as OpenCV receives it (before the EXIF step): (H, W, 3)
    uint8 BGR"""
    d = parse_and_decode(data)
    W, H, hmax, vmax = d["width"], d["height"], d["hmax"], d["vmax"]
    if d["smooth"] is not None:
        if mode != "libjpeg9":
            raise NotImplementedError("libjpeg-turbo's block smoothing is not restated")
        d["coef"] = [block_smooth(cf, q, cb, wb, hb) for (_, _, q), cf, cb, wb, hb in
                     zip(d["comps"], d["coef"], d["smooth"], d["wib"], d["hib"])]
    planes = []
    for (h, v, q), cf in zip(d["comps"], d["coef"]):
        sh = 2 if (mode == "libjpeg9" and hmax % (2 * h) == 0 and h * 2 <= hmax) else 1
        sv = 2 if (mode == "libjpeg9" and vmax % (2 * v) == 0 and v * 2 <= vmax) else 1
        # IDCT sizes never differ by more than 2x between the directions (jdmaster.c)
        blk = idct_blocks(cf, q, 8 * sv, 8 * sh)
        bh, bw = cf.shape[:2]
        p = blk.transpose(0, 2, 1, 3).reshape(bh * 8 * sv, bw * 8 * sh)
        fh, fv = hmax // (h * sh), vmax // (v * sv)
        if fh == 1 and fv == 1:
            planes.append(p[:H, :W].astype(np.int64))
        elif fh == 2 and fv == 1:
            dw = -(-W * h // hmax)
            planes.append(_fancy_h2v1(p, dw)[:H, :W])
        elif fh == 2 and fv == 2:
            dw, dh = -(-W * h // hmax), -(-H * v // vmax)
            planes.append(_fancy_h2v2(p, dw, dh)[:H, :W])
        else:
            raise ValueError("unsupported sampling")
    if len(planes) == 1:
        y = planes[0].astype(np.uint8)
        return np.repeat(y[..., None], 3, -1)
    cs = color_space(d, mode)
    if cs == "rgb":  # jdcolor.c rgb_convert: a copy
        return np.stack(planes[::-1], -1).astype(np.uint8)
    Y, Cb, Cr = planes[:3]
    xb, xr = Cb - 128, Cr - 128
    one_half = 1 << 15
    cb_g = FIXS(0.344136286 if mode == "libjpeg9" else 0.34414)
    cr_g = FIXS(0.714136286 if mode == "libjpeg9" else 0.71414)
    r = Y + ((FIXS(1.402) * xr + one_half) >> 16)
    g = Y + ((-cb_g * xb + one_half - cr_g * xr) >> 16)
    b = Y + ((FIXS(1.772) * xb + one_half) >> 16)
    if cs == "cmyk":
        return cv_cmyk_to_bgr(np.stack(planes, -1))
    if cs == "ycck":  # jdcolor.c ycck_cmyk_convert: 255 - the RGB conversion, K unchanged
        cmy = [255 - np.clip(v, 0, 255) for v in (r, g, b)]
        return cv_cmyk_to_bgr(np.stack(cmy + [planes[3]], -1))
    return np.clip(np.stack([b, g, r], -1), 0, 255).astype(np.uint8)


def FIXS(x: float) -> int:  # jdcolor.c FIX with SCALEBITS 16
    return int(x * (1 << 16) + 0.5)
