"""bench.py's multi-GPU launch contract (CPU: no GPU is touched).

`bench.py --gpus N` started without WORLD_SIZE launches its N ranks itself (torch.distributed.run on
127.0.0.1) and exits with their status; fewer than N visible GPUs, or a WORLD_SIZE that differs from
N, fail non-zero instead of running one rank."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=240, cwd=ROOT)


def test_gpus_n_spawns_n_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted((d["rank"], d["local_rank"], d["world_size"]) for d in lines) == [(0, 0, 2), (1, 1, 2)]


def test_gpus_n_without_gpus_fails():
    import torch
    if torch.cuda.device_count() >= 2:
        return  # (a GPU box: the real launch is the driver's to run)
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and "visible" in (r.stderr + r.stdout)


def test_world_size_must_equal_gpus():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_launches_per_step_leaves_reruns_out(tmp_path):
    """A profiled run's re-run passes (SDH_TRACE attempt lines, counted into meta.json by
    profiles/summarize.py) are not per-step work: C2 2 + 1 pushes with one re-run launch -> 1 launch
    per step; C5 4 pushes per step with 2 launches each and one re-run pass."""
    import json
    import bench
    (tmp_path / "meta.json").write_text(json.dumps({"steps": 2, "warmup": 1, "reruns": 1, "workload": "c2"}))
    assert bench.launches_per_step({"calls": 4}, str(tmp_path)) == 1.0
    (tmp_path / "meta.json").write_text(json.dumps({"steps": 2, "warmup": 1, "reruns": 1, "workload": "c5"}))
    assert bench.launches_per_step({"calls": 26}, str(tmp_path)) == 8.0
    (tmp_path / "meta.json").write_text(json.dumps({"steps": 3, "warmup": 1, "workload": "c3"}))
    assert bench.launches_per_step({"calls": 12}, str(tmp_path)) == 3.0
