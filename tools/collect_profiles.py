#!/usr/bin/env python3
"""Copy one profile_round.sh run from gpurun_out/<run> into profiles/<run>/ (tracked).

  python tools/collect_profiles.py r01b

bench_lines.jsonl = the JSON line of every bench_*.log; kernel_stats[_<op>].csv = rocprofv3
--stats summaries; pytest_gpu.txt = the tail of the GPU test run.
"""
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    run = sys.argv[1]
    src = ROOT / "gpurun_out" / run
    dst = ROOT / "profiles" / run
    dst.mkdir(parents=True, exist_ok=True)
    lines = []
    for log in sorted(src.glob("bench_*.log")):
        for ln in log.read_text().splitlines():
            if ln.startswith("{") and '"metric"' in ln:
                lines.append(json.dumps(json.loads(ln)))
    (dst / "bench_lines.jsonl").write_text("\n".join(lines) + "\n")
    for d in sorted(src.glob("prof*")):
        f = d / "stats_kernel_stats.csv"
        if d.is_dir() and f.exists():
            tag = d.name[len("prof"):]
            shutil.copy(f, dst / f"kernel_stats{tag}.csv")
    t = src / "pytest_gpu.log"
    if t.exists():
        (dst / "pytest_gpu.txt").write_text("\n".join(t.read_text().splitlines()[-15:]) + "\n")
    print(f"{len(lines)} bench lines -> {dst}")


if __name__ == "__main__":
    main()
