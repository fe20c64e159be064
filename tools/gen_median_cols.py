#!/usr/bin/env python3
"""Median-of-25 selection networks over pre-sorted columns, for the 5x5 median kernel
(image-denoising_amd/csrc/median_cols.hpp).

The kernel sorts every 5-row window column once (SORT5, 9 comparators) and then needs, for a
CHAIN of 5 horizontally adjacent outputs of one channel, the medians of columns k..k+4
(k = 0..4) of 9 sorted columns.  Neighbouring outputs share 4 of their 5 columns, so the chain
is built by recursive halving: a group of outputs merges (Batcher odd-even merge) the columns
common to all its outputs into its parent's merged list; each output then takes rank 12 of
(its group's list, its own remaining columns) with the split formula
    s_k = min over j of max(A[k - j], B[j - 1])       (j elements taken from B).

Every value is simulated symbolically over EVERY 0/1 input consistent with the premise "each
column is sorted" (6^9 vectors, bit-packed).  A value whose truth table equals an existing
value's IS that value (two monotone min/max networks that agree on every 0/1 input of the
premise agree on every real input of it: thresholding keeps sorted columns sorted and commutes
with min/max -- the 0-1 principle, Knuth TAOCP 5.3.4), so ordered comparators, +-inf pads and
duplicate work fold away; the rest is pruned to what the 5 medians need and each output is
re-verified against the popcount median over the whole premise set.

Measured op counts (min/max per output): single output 140, pair 54, chain of 4 47.5,
chain of 5 55.2 (276 for 5) -- vs 202 for the unsorted 25-input Batcher network.  The header
carries the chain of 5 (16-byte lanes: two same-channel chains of 5) and the chain of 4 (24-byte
lanes: one chain per channel, u16 pairs of pixels p and p + 4).

  python tools/gen_median_cols.py            # writes the header, prints op counts
"""
from __future__ import annotations

import itertools
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent.parent / "image-denoising_amd" / "csrc" / "median_cols.hpp"
SORT5 = [(0, 1), (3, 4), (2, 4), (2, 3), (0, 3), (0, 2), (1, 4), (1, 3), (1, 2)]


def premise_inputs(ncols, nrank):
    """0/1 vectors with every column sorted ascending: column c rank r is 1 iff r >= z_c"""
    combos = np.array(list(itertools.product(range(nrank + 1), repeat=ncols)), dtype=np.int8)
    x = {}
    for c in range(ncols):
        for r in range(nrank):
            x[(c, r)] = combos[:, c] <= r
    return x, combos


class Net:
    """symbolic min/max values with bit-packed truth tables over the premise set"""

    def __init__(self, leaves):
        self.n = len(next(iter(leaves.values())))
        self.vals, self.tt, self.by_tt = [], [], {}
        for key, v in leaves.items():
            self._add(("in", key), np.packbits(v))
        self.leaf = {key: i for i, key in enumerate(leaves)}

    def _add(self, node, tt):
        k = tt.tobytes()
        if k in self.by_tt:
            return self.by_tt[k]
        self.vals.append(node)
        self.tt.append(tt)
        self.by_tt[k] = len(self.vals) - 1
        return len(self.vals) - 1

    def const(self, v):
        return self._add(("const", v), np.packbits(np.full(self.n, bool(v))))

    def mn(self, a, b):
        return self._add(("min", a, b), self.tt[a] & self.tt[b])

    def mx(self, a, b):
        return self._add(("max", a, b), self.tt[a] | self.tt[b])

    def truth(self, v):
        return np.unpackbits(self.tt[v])[: self.n].astype(bool)

    def live(self, outs):
        live, stack = set(), list(outs)
        while stack:
            v = stack.pop()
            if v in live:
                continue
            live.add(v)
            if self.vals[v][0] in ("min", "max"):
                stack.extend(self.vals[v][1:])
        return sorted(i for i in live if self.vals[i][0] in ("min", "max"))


def oe_merge(net, A, B, hi):
    """Batcher odd-even merge of two sorted lists (each padded with +inf to a power of two)"""
    n = 1
    while n < max(len(A), len(B)):
        n *= 2
    w = list(A) + [hi] * (n - len(A)) + list(B) + [hi] * (n - len(B))
    comps = []

    def merge(lo, cnt, r):
        step = r * 2
        if step < cnt:
            merge(lo, cnt, step)
            merge(lo + r, cnt, step)
            for i in range(lo + r, lo + cnt - r, step):
                comps.append((i, i + r))
        else:
            comps.append((lo, lo + r))

    merge(0, 2 * n, 1)
    for i, j in comps:
        a, b = w[i], w[j]
        w[i], w[j] = net.mn(a, b), net.mx(a, b)
    return w[: len(A) + len(B)]


def select_from_two(net, A, B, k):
    """k-th smallest (0-based) of sorted A u sorted B: min over j of max(A[k-j], B[j-1])"""
    lo = net.const(0)
    best = None
    for j in range(0, len(B) + 1):
        i = k + 1 - j
        if i < 0 or i > len(A):
            continue
        v = net.mx(A[i - 1] if i > 0 else lo, B[j - 1] if j > 0 else lo)
        best = v if best is None else net.mn(best, v)
    return best


def chain_net(nout):
    ncols = nout + 4
    leaves, _ = premise_inputs(ncols, 5)
    net = Net(leaves)
    hi = net.const(1)

    def col(c):
        return [net.leaf[(c, r)] for r in range(5)]

    def merge_lists(lists):
        lists = [l for l in lists if l]
        while len(lists) > 1:
            nxt = [oe_merge(net, lists[i], lists[i + 1], hi) for i in range(0, len(lists) - 1, 2)]
            if len(lists) % 2:
                nxt.append(lists[-1])
            lists = nxt
        return lists[0] if lists else []

    outs = {}

    def rec(lo, hi_, base, have):
        if hi_ - lo == 1:
            extra = merge_lists([col(c) for c in range(lo, lo + 5) if c not in have])
            outs[lo] = select_from_two(net, base, extra, 12) if base else extra[12]
            return
        common = set(range(hi_ - 1, lo + 5))
        new = merge_lists([col(c) for c in sorted(common - have)])
        cur = oe_merge(net, base, new, hi) if base and new else (base or new)
        mid = (lo + hi_ + 1) // 2
        rec(lo, mid, cur, have | common)
        rec(mid, hi_, cur, have | common)

    rec(0, nout, None, set())
    for k, o in outs.items():  # proof: every output is the median of its 5 columns
        cnt = np.zeros(net.n, np.int32)
        for c in range(k, k + 5):
            for r in range(5):
                cnt += leaves[(c, r)]
        if not np.array_equal(net.truth(o), cnt > 12):
            raise SystemExit(f"chain output {k} FAILED the 0-1 proof")
    return net, [outs[k] for k in range(nout)]


def verify_sort5():
    for bits in range(32):
        v = [(bits >> i) & 1 for i in range(5)]
        for i, j in SORT5:
            if v[i] > v[j]:
                v[i], v[j] = v[j], v[i]
        if v != sorted(v):
            raise SystemExit("SORT5 FAILED")


def emit_chain(net, outs, nout):
    """C++ text of median25_chain<nout>, the fused (3-input) program; returns (text, 2-input ops,
    instructions)"""
    ops = net.live(outs)
    name = {idx: f"x[{key[0]}][{key[1]}]" for key, idx in net.leaf.items()}
    lines = [f"// medians of columns k..k+4, k = 0..{nout - 1}, of {nout + 4} sorted 5-element "
             f"columns x[col][rank]: {len(ops)} min/max ops",
             "template <typename T, typename F>",
             f"__device__ __forceinline__ void median25_chain{nout}(const T (&x)[{nout + 4}][5], "
             f"T (&o)[{nout}], F ops) {{"]
    prog = fuse3(net, ops, outs)
    verify_program(net, prog, outs)
    for k, (v, kind, args) in enumerate(prog):
        name[v] = f"t{k}"
        fn = ("ops.mn" if kind == "min" else "ops.mx") + ("3" if len(args) == 3 else "")
        lines.append(f"  const T t{k} = {fn}({', '.join(name[a] for a in args)});")
    for k, o in enumerate(outs):
        lines.append(f"  o[{k}] = {name[o]};")
    lines += ["}", ""]
    return lines, len(ops), len(prog)


def emit(chains):
    lines = [
        "// GENERATED by tools/gen_median_cols.py -- do not edit.",
        "// 5x5 median over pre-sorted window columns (proven by the 0-1 principle under the",
        "// sorted-column premise; see the generator).  F must provide mn / mx / mn3 / mx3.",
        "#pragma once",
        "",
        "namespace idn {",
        "",
        "// ascending sort of 5 values, 9 comparators (18 min/max)",
        "template <typename T, typename F>",
        "__device__ __forceinline__ void sort5(T (&v)[5], F ops) {",
    ]
    for i, j in SORT5:
        lines.append(f"  {{ const T a = v[{i}], b = v[{j}]; v[{i}] = ops.mn(a, b); "
                     f"v[{j}] = ops.mx(a, b); }}")
    lines += ["}", ""]
    stats = []
    for net, outs, nout in chains:
        text, n, nf = emit_chain(net, outs, nout)
        lines += text
        stats.append((nout, n, nf))
    lines += ["}  // namespace idn", ""]
    OUT.write_text("\n".join(lines))
    return stats


def fuse3(net, ops, outs):
    """3-input min/max (v_pk_minimum3_f16 / v_pk_maximum3_f16): a node z = op(x, y) absorbs a
    2-input child x of the same op that nothing else reads.  Greedy from the outputs down."""
    fan = {}
    for v in ops:
        for a in net.vals[v][1:]:
            fan[a] = fan.get(a, 0) + 1
    for o in outs:
        fan[o] = fan.get(o, 0) + 1
    args = {v: list(net.vals[v][1:]) for v in ops}
    kind = {v: net.vals[v][0] for v in ops}
    gone = set()
    for z in reversed(ops):
        if z in gone or len(args[z]) == 3:
            continue
        for i, x in enumerate(args[z]):
            if x in kind and x not in gone and kind[x] == kind[z] and fan[x] == 1 \
                    and len(args[x]) == 2:
                args[z] = args[z][:i] + args[x] + args[z][i + 1:]
                gone.add(x)
                break
    return [(v, kind[v], args[v]) for v in ops if v not in gone]


def verify_program(net, prog, outs):
    """re-simulate the emitted (fused) program over the premise set: same truth tables"""
    tt = {idx: net.tt[idx] for idx in net.leaf.values()}
    for key, idx in net.by_tt.items():
        if net.vals[idx][0] == "const":
            tt[idx] = net.tt[idx]
    for v, kind, args in prog:
        acc = tt[args[0]]
        for a in args[1:]:
            acc = (acc & tt[a]) if kind == "min" else (acc | tt[a])
        tt[v] = acc
    for o in outs:
        if not np.array_equal(tt[o], net.tt[o]):
            raise SystemExit("fused program FAILED")


def main():
    verify_sort5()
    chains = []
    for nout in (5, 4):
        net, outs = chain_net(nout)
        chains.append((net, outs, nout))
    for nout, n, nf in emit(chains):
        print(f"chain of {nout}: {n} 2-input ops ({n / nout:.1f} per output), {nf} after "
              f"3-input fusion; 0-1 principle PROVEN")
    print(f"sort5: 9 comparators PROVEN; wrote {OUT}")


if __name__ == "__main__":
    main()
