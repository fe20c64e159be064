"""Summarise tools/clock_probe.sh output: per op spec, median GB/s of the blocks after the first
two (steady state), with the amd-smi power / GFX clock samples taken during them."""
import bisect
import json
import re
import sys

d = sys.argv[1]
txt = open(f"{d}/smi.txt").read()
samples = []
for blk in txt.split("=== abs=")[1:]:
    t = float(blk.split("\n")[0])
    pw = re.search(r"SOCKET_POWER: (\d+) W", blk)
    clks = [int(x) for x in re.findall(r"GFX_\d+:\n\s+CLK: (\d+) MHz", blk)]
    if pw and clks:
        samples.append((t, int(pw.group(1)), sum(clks) / len(clks)))
st = [s[0] for s in samples]
runs = {}
order = []
for line in open(f"{d}/probe.jsonl"):
    p = json.loads(line)
    if p["blk"] == 0:
        order.append(p["op"] + f"#{len(order)}")
    runs.setdefault(order[-1], []).append(p)
for k in order:
    bl = runs[k][2:]
    g = sorted(b["GBps"] for b in bl)
    lo, hi = bl[0]["abs"], bl[-1]["abs"]
    i0, i1 = bisect.bisect_left(st, lo), bisect.bisect_right(st, hi)
    ss = samples[i0:i1] or samples[max(i0 - 1, 0):i0 + 1]
    pw = sum(s[1] for s in ss) / len(ss)
    ck = sum(s[2] for s in ss) / len(ss)
    print(json.dumps({"op": k.split("#")[0], "blocks": len(bl), "GBps_median": g[len(g) // 2],
                      "ms_median": round(921.6e6 / g[len(g) // 2] / 1e6, 4),
                      "power_W": round(pw), "gfx_MHz": round(ck), "smi_samples": len(ss)}))
