"""Damaged variants of the JPEG fixtures: what cv2.imread meets in real datasets (files cut short,
bit errors in the entropy-coded data, restart markers lost or renumbered, stray markers).

Shared by tests/golden/make_jpeg_damaged.py (which decodes every variant with the real libjpeg 9d
and commits the pixels) and the tests (which rebuild the same bytes from the committed fixture
files).  Pure Python, deterministic: every position is derived from the file's own structure.

A recipe is (file name, op, argument):
  cut    f      keep the bytes up to fraction f of the file's entropy-coded data (all scans),
                then EOI (jdatasrc.c inserts the same EOI when a file just ends)
  cutrst k, a   cut at the k-th RST marker (in file order): a = 0 just before it, 2 just after it
  flip   seed   flip one bit in each of 1 + seed % 3 data bytes (never a 0xFF byte, never the byte
                after one, never producing 0xFF: no marker is made or broken)
  ones   f      three data bytes at fraction f replaced by FF00 FF00 FF00 (24 one bits: no
                Huffman code of a table with the all-ones code reserved, JWRN_HUFF_BAD_CODE)
  junk   f      the data byte at fraction f replaced by the marker FF 08 (below SOF0: libjpeg ends
                the segment there and resynchronises at the next restart marker)
  rstnum k, d   the k-th RST marker's number moved by d (libjpeg's jpeg_resync_to_restart)
  shortiv k, r  the data of the restart interval that the k-th RST marker ends cut to its first
                m bytes (m the largest <= 60 % of them whose unstuffed length is r mod 32, r in
                1..3): the interval's data run out mid-MCU a few bits past a 256-bit boundary of
                the decoder's sub-chunks, so symbols that start before it read libjpeg's zero fill
"""


def _markers(d: bytes):
    """(offset, code) of every marker after SOI"""
    out, i = [], 2
    while i + 1 < len(d):
        if d[i] == 0xFF and d[i + 1] not in (0x00, 0xFF):
            out.append((i, d[i + 1]))
            i += 2
        else:
            i += 1
    return out


def _spans(d: bytes):
    """[begin, end) of every scan's entropy-coded data (up to the marker after it that is not RSTn)"""
    ms = _markers(d)
    out = []
    for k, (o, m) in enumerate(ms):
        if m != 0xDA:
            continue
        begin = o + 2 + ((d[o + 2] << 8) | d[o + 3])
        end = next((o2 for o2, m2 in ms[k + 1:] if o2 >= begin and not 0xD0 <= m2 <= 0xD7),
                   len(d))
        out.append((begin, end))
    return out


def _at(d: bytes, f: float) -> int:
    """the byte at fraction f of all entropy-coded data"""
    sp = _spans(d)
    t = int(sum(e - b for b, e in sp) * f)
    for b, e in sp:
        if t < e - b:
            return b + t
        t -= e - b
    return sp[-1][1] - 1


def _safe(d: bytes, k: int) -> bool:
    """byte k is plain entropy data: not 0xFF, not after 0xFF (no stuffing / marker code)"""
    return d[k] != 0xFF and d[k - 1] != 0xFF


def _near_safe(d: bytes, k: int) -> int:
    """the first byte from k on (wrapping to the first scan's data) that starts three plain data
    bytes of one scan"""
    sp = _spans(d)
    ok = [j for b, e in sp for j in range(b + 1, e - 3)
          if _safe(d, j) and _safe(d, j + 1) and _safe(d, j + 2)]
    if not ok:
        raise ValueError("no plain entropy-coded bytes")
    return next((j for j in ok if j >= k), ok[0])


def damage(d: bytes, op: str, arg) -> bytes:
    if op == "cut":
        return d[:_at(d, arg)] + b"\xff\xd9"
    if op == "cutrst":
        k, a = arg
        off = [o for o, m in _markers(d) if 0xD0 <= m <= 0xD7][k]
        return d[:off + a] + b"\xff\xd9"
    if op == "flip":
        x = bytearray(d)
        state = 0x9E3779B9 ^ (arg * 0x85EBCA6B) ^ len(d)
        done = 0
        while done < 1 + arg % 3:
            state = (state * 6364136223846793005 + 1442695040888963407) & (2 ** 64 - 1)
            k = _at(d, ((state >> 11) & 0xFFFFFF) / float(1 << 24))
            bit = (state >> 40) & 7
            if _near_safe(x, k) == k and (x[k] ^ (1 << bit)) != 0xFF:
                x[k] ^= 1 << bit
                done += 1
        return bytes(x)
    if op == "ones":
        k = _near_safe(d, _at(d, arg))
        return d[:k] + b"\xff\x00\xff\x00\xff\x00" + d[k + 3:]
    if op == "junk":
        k = _near_safe(d, _at(d, arg))
        return d[:k] + b"\xff\x08" + d[k + 1:]
    if op == "rstnum":
        k, dd = arg
        off = [o for o, m in _markers(d) if 0xD0 <= m <= 0xD7][k]
        x = bytearray(d)
        x[off + 1] = 0xD0 + ((x[off + 1] - 0xD0 + dd) & 7)
        return bytes(x)
    if op == "shortiv":
        k, r = arg
        rst = [o for o, m in _markers(d) if 0xD0 <= m <= 0xD7]
        end = rst[k]
        begin = rst[k - 1] + 2 if k > 0 else next(b for b, e in _spans(d) if b <= end < e)
        body = d[begin:end]
        best, n_un = None, 0
        for m in range(1, len(body)):
            # unstuffed length of body[:m] (a stuffed FF00 is one data byte); never cut inside a pair
            n_un += 0 if body[m - 1] == 0x00 and m >= 2 and body[m - 2] == 0xFF else 1
            if m > 0.6 * len(body):
                break
            if body[m - 1] != 0xFF and n_un % 32 == r:
                best = m
        if best is None:
            raise ValueError("interval too short")
        return d[:begin + best] + d[end:]
    raise ValueError(op)


# the committed cases: baseline (the chunked and the restart-interval paths), progressive and
# multi-scan (the scan path), arithmetic, four components
_CUT_FILES = ["s420_q90_600x1000.jpg", "s444_q95_96x128.jpg", "s420_opt_130x170.jpg",
              "gray_q80_91x77.jpg", "s422_q85_120x200.jpg", "s420_rstrow_120x160.jpg",
              "s422_rst2_77x130.jpg", "s444_rst3_70x90.jpg", "gray_rst2_48x64.jpg",
              "prog_s444_q85_96x128.jpg", "prog_s420_rst4_120x160.jpg", "prog_gray_q80_91x77.jpg",
              "prog_s422_q75_odd_45x67.jpg", "arith_s444_96x128.jpg", "arith_rst_s422_120x200.jpg",
              "arith_prog_rst_s444_96x128.jpg", "cmyk_s444_40x56.jpg", "ycck_prog_s444_40x56.jpg"]
_RST_FILES = ["s420_rstrow_120x160.jpg", "s422_rst2_77x130.jpg", "s444_rst3_70x90.jpg",
              "gray_rst2_48x64.jpg"]


def cases():
    out = []
    for f in _CUT_FILES:
        for c in (0.02, 0.3, 0.71, 0.97):
            out.append((f, "cut", c))
        for s in range(3):
            out.append((f, "flip", s))
        out.append((f, "ones", 0.4))
    for f in _RST_FILES:
        out += [(f, "cutrst", (3, 0)), (f, "cutrst", (3, 2)), (f, "junk", 0.45),
                (f, "rstnum", (2, 3)), (f, "rstnum", (2, 1)), (f, "rstnum", (2, -1))]
        out += [(f, "shortiv", (2, r)) for r in (1, 2, 3)]
    return out


def key(case) -> str:
    f, op, arg = case
    a = "_".join(str(x) for x in arg) if isinstance(arg, tuple) else str(arg)
    return f"{f}:{op}:{a}"


def random_damage(d: bytes, rng) -> bytes:
    """one random damage of the kinds above at a random place (rng: random.Random); for fuzzing the
    decoder against the oracle beyond the libjpeg-pinned cases"""
    op = rng.choice(["cut", "flip", "flip", "ones", "junk", "rstnum", "mix"])
    rst = [o for o, m in _markers(d) if 0xD0 <= m <= 0xD7]
    if op == "cut":
        return damage(d, "cut", rng.random())
    if op == "flip":
        return damage(d, "flip", rng.randrange(1000))
    if op == "ones":
        return damage(d, "ones", rng.random() * 0.95)
    if op == "junk":
        return damage(d, "junk", rng.random() * 0.95)
    if op == "rstnum" and rst:
        return damage(d, "rstnum", (rng.randrange(len(rst)), rng.choice([-2, -1, 1, 2, 3, 4])))
    return damage(damage(d, "flip", rng.randrange(1000)), "cut", 0.3 + 0.7 * rng.random())
