#!/usr/bin/env python3
"""Round-4 counter evidence (tools only): fold the rocprofv3 passes of tools/pmc_r04.sh into one
JSON record per op, and the ops' HBM traffic into profiles/pmc_traffic.json.

  python tools/pmc_r04.py <pass_root> <out_json_dir>

<pass_root>/<op>/{fetch,write,sq1,sq2}/ hold counter_collection.csv files and
<pass_root>/<op>/ks/ the kernel-trace stats of the same command.  Per kernel (averaged over its
dispatches):
  hbm_read_bytes   FETCH_SIZE x 2 x 1024 (gfx950 reports half the bytes of a 16 B/lane streaming
                   read, MI355X_MICROARCH.md "HBM"; other access widths are uncalibrated there --
                   the raw KiB are kept next to it)
  hbm_write_bytes  WRITE_SIZE x 1024
  valu_issue       SQ_INSTS_VALU x 4 cycles / (kernel time x 2.4 GHz x 1024 SIMDs) -- a lower
                   bound: the chip clocks below 2.4 GHz under load
  wait_share       SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier); issue_stall_share
                   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES; active_share SQ_ACTIVE_INST_ANY /
                   SQ_WAVE_CYCLES (the three are disjoint, MI355X_MICROARCH.md "PMC slots")
  lds_conflict_share  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  valu_per_pixel   SQ_INSTS_VALU (wave instructions) x 64 lanes / pixels of the launch
"""
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PIX = 600 * 1000
BATCH = {"cfg2": 256, "cfg3": 1024, "cfg4": 512, "cfg5": 512}
ALG_BPP = {"gauss5_blob": 15, "wavelet_bior15_f64": 27}
CLK, SIMDS = 2.4e9, 1024


def counters(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def stats(d):
    out = {}
    for f in Path(d).rglob("*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Name"].split("(")[0].replace("void ", "")
            out[name] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def main():
    root, dest = Path(sys.argv[1]), Path(sys.argv[2])
    dest.mkdir(parents=True, exist_ok=True)
    traffic_path = ROOT / "profiles" / "pmc_traffic.json"
    traffic = json.loads(traffic_path.read_text()) if traffic_path.exists() else {}
    for opdir in sorted(p for p in root.iterdir() if p.is_dir()):
        op = opdir.name
        n = BATCH.get(op, 256)
        merged = collections.defaultdict(dict)
        for sub in ("fetch", "write", "sq1", "sq2"):
            if (opdir / sub).exists():
                for k, cs in counters(opdir / sub).items():
                    merged[k].update(cs)
        ks = stats(opdir / "ks") if (opdir / "ks").exists() else {}
        rec = {"op": op, "batch": n, "pixels_per_launch": n * PIX, "kernels": {}}
        tot_r = tot_w = 0.0
        for k, m in merged.items():
            if not (k.startswith("idn::") or "idn::" in k):
                continue
            e = {"counters": {c: round(v, 1) for c, v in sorted(m.items())}}
            if "FETCH_SIZE" in m:
                e["hbm_read_bytes"] = int(2 * m["FETCH_SIZE"] * 1024)
                tot_r += e["hbm_read_bytes"]
            if "WRITE_SIZE" in m:
                e["hbm_write_bytes"] = int(m["WRITE_SIZE"] * 1024)
                tot_w += e["hbm_write_bytes"]
            t = ks.get(k, {}).get("avg_us")
            if t:
                e["avg_us"] = round(t, 2)
            wc = m.get("SQ_WAVE_CYCLES")
            if "SQ_INSTS_VALU" in m:
                e["valu_per_pixel"] = round(m["SQ_INSTS_VALU"] * 64 / (n * PIX), 2)
                if t:
                    e["valu_issue"] = round(m["SQ_INSTS_VALU"] * 4 / (t * 1e-6 * CLK * SIMDS), 3)
            if wc:
                for c, key in (("SQ_WAIT_ANY", "wait_share"), ("SQ_WAIT_INST_ANY", "issue_stall_share"),
                               ("SQ_ACTIVE_INST_ANY", "active_share")):
                    if c in m:
                        e[key] = round(m[c] / wc, 3)
            if m.get("SQ_LDS_IDX_ACTIVE"):
                e["lds_conflict_share"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 3)
            rec["kernels"][k] = e
        alg = ALG_BPP.get(op, 6) * n * PIX
        rec["op_hbm_bytes_per_step"] = int(tot_r + tot_w)
        rec["algorithmic_bytes_per_step"] = alg
        rec["traffic_over_algorithmic"] = round((tot_r + tot_w) / alg, 3) if alg else None
        (dest / f"{op}.json").write_text(json.dumps(rec, indent=1) + "\n")
        if tot_r and tot_w:
            old = traffic.get(op, {})
            traffic[op] = {
                "kernel": "all idn:: kernels of one step" if len(rec["kernels"]) > 1 else next(iter(rec["kernels"])),
                "kernels": {k: {"read": v.get("hbm_read_bytes"), "write": v.get("hbm_write_bytes")}
                            for k, v in rec["kernels"].items()},
                "hbm_read_bytes_per_launch": int(tot_r),
                "hbm_write_bytes_per_launch": int(tot_w),
                "hbm_bytes_per_launch": int(tot_r + tot_w),
                "algorithmic_bytes_per_launch": float(alg),
                "traffic_over_algorithmic": rec["traffic_over_algorithmic"],
                "correction": "FETCH_SIZE x2 (gfx950 16B/lane streaming reads; other widths "
                              "uncalibrated), WRITE_SIZE as-is",
                "source": f"{dest.resolve().relative_to(ROOT)}/{op}.json (rocprofv3 --pmc, separate "
                          f"FETCH / WRITE passes)",
            }
            if "kernel_form" in old and old.get("kernel") == traffic[op]["kernel"]:
                traffic[op]["kernel_form"] = old["kernel_form"]
        print(op, json.dumps({k: {x: v[x] for x in v if x != "counters"} for k, v in rec["kernels"].items()}))
    traffic_path.write_text(json.dumps(traffic, indent=1) + "\n")


if __name__ == "__main__":
    main()
