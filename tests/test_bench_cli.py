"""CPU: bench.py's multi-GPU contract without a GPU (--dry-run resolves ranks and shards only).

`bench.py --gpus N` with no WORLD_SIZE must start N ranks itself (one child
torch.distributed.run process group) and relay rank 0's line; under a WORLD_SIZE that disagrees
with --gpus it must exit non-zero instead of silently measuring another rank count."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _run(args, env_extra=None, drop_world=True):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if drop_world:
            env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=240)


def _json_line(out: str):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_n_launches_n_ranks_weak():
    r = _run(["--gpus", "2", "--batch", "3", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["scaling"] == "weak"
    assert rec["total_images"] == 6
    assert sorted(rec["shards"]) == [[0, 0, 3], [1, 3, 6]]


def test_gpus_n_strong_scaling_splits_a_fixed_batch():
    r = _run(["--gpus", "3", "--scaling", "strong", "--batch", "10", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 3 and rec["total_images"] == 10
    assert sorted(rec["shards"]) == [[0, 0, 4], [1, 4, 7], [2, 7, 10]]


def test_gpus_mismatching_world_size_exits_nonzero():
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1"}, drop_world=False)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_single_gpu_default_is_one_rank():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 1 and rec["shards"] == [[0, 0, 256]]


def test_roofline_names_the_binding_roof():
    """The line carries the VALU roofline beside the HBM one where a committed PMC record gives
    the op's VALU lane-ops per pixel, and `bound` names the higher fraction."""
    sys.path.insert(0, str(ROOT))
    import bench
    pix = 256 * bench.H * bench.W
    # median 5x5 at its measured 0.479 ms: ~110 VALU/px -> ~0.9 of the VALU peak, 0.24 of HBM
    rl, _ = bench.roofline_fields("median5", 6, pix, 0.479, None, "median_u8")
    assert rl["bound"] == "valu"
    assert rl["valu"]["valu_per_pixel"] > 50 and 0.6 < rl["valu"]["frac"] < 1.2
    assert rl["hbm"]["frac"] < 0.3 and rl["frac"] == rl["valu"]["frac"]
    assert rl["unit"] == "T lane-ops/s" and rl["valu"]["valu_source"].startswith("profiles/")
    # the headline stays HBM-bound: 19 VALU/px at 0.151 ms is ~0.5 of the VALU peak
    rl, gbs = bench.roofline_fields("gauss5", 6, pix, 0.151, 9.4e8, "stencil_u8")
    assert rl["bound"] == "hbm" and rl["frac"] == rl["hbm"]["frac"] > 0.7
    assert rl["valu"]["frac"] < rl["hbm"]["frac"] and abs(rl["achieved"] - gbs) < 0.1
    # end-to-end ops claim no fraction
    rl, _ = bench.roofline_fields("detect_e2e", 6, bench.H * bench.W, 1.7, None, "e2e")
    assert rl["frac"] is None and "valu" not in rl
