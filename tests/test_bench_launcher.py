"""bench.py's multi-rank launcher: ``python bench.py --gpus N`` with no
torch.distributed launcher around it starts N ranks itself (before any GPU call), a rank
count that differs from --gpus is refused, and the JSON line carries the world size the
process group saw.  CPU only: ``--dry-run`` runs the launcher and process-group path with gloo
ranks on the CPU and a stub step."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=240)


def _line(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr
    return json.loads(lines[0])


def test_gpus_2_starts_two_ranks():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "0", "--dry-run"], {"FVO_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    j = _line(r)
    assert j["n_gpus"] == 2 and j["world_size_seen"] == 2 and j["backend"] == "gloo" and j["steps"] == 3
    # the exchange record (the bench's per-step map exchange, run here on host
    # tensors of the bench shapes: B = 64 frames, cap = 2 * 1000 + 64 keypoints)
    x = j["exchange"]
    send = 64 * (16 * 8 + 4 + (2 * 1000 + 64) * 3 * 4 + 4)
    assert send == 1_593_856  # DESIGN.md §6 / dist.exchange_bytes: 1.59 MB per rank per step at 600p
    assert x["mode"].startswith("all-gather") and x["send_bytes_per_rank_per_step"] == send
    # two ranks: each receives the other's slice over the link (its own never leaves it)
    assert x["recv_bytes_per_rank_per_step"] == send and x["gathered_bytes_per_step"] == 2 * send
    assert x["steps_timed"] == 3 and x["host_ms_per_step"] > 0
    assert "stream_ms_per_step" in x and "collective_ms_per_step" in x


def test_gpus_2_map_on_rank0_gathers():
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "0", "--dry-run", "--map-rank0", "1"],
             {"FVO_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    x = _line(r)["exchange"]
    assert x["mode"].startswith("gather to rank 0") and x["steps_timed"] == 2


def test_gpus_1_is_one_process():
    r = _run(["--gpus", "1", "--steps", "2", "--warmup", "0", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _line(r)
    assert j["n_gpus"] == 1 and j["world_size_seen"] == 1
    assert j["exchange"]["mode"].startswith("off") and j["exchange"]["send_bytes_per_rank_per_step"] == 0


def test_rank_count_other_than_gpus_is_refused():
    r = _run(["--gpus", "2", "--steps", "1", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--gpus 2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
