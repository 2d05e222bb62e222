"""bench.py --gpus N starts N ranks itself (torch.distributed.run child) when no torchrun environment is
set, and refuses a WORLD_SIZE that disagrees with --gpus. CPU dry run over gloo: no kernels, the same
launcher, barrier and max-over-ranks timing as the GPU path."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(argv, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_launcher_world2_gloo_dry_run():
    r = _run(["--gpus", "2", "--device", "cpu", "--backend", "gloo", "--steps", "5", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    j = _line(r.stdout)
    assert j["dry_run"] is True
    assert j["n_gpus"] == 2 and j["dist_world_size"] == 2
    assert sorted(j["ranks_reported"]) == [0, 1]
    assert j["steps"] == 5 and j["value"] > 0


def test_launcher_world1_unchanged():
    r = _run(["--gpus", "1", "--device", "cpu", "--steps", "3", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    j = _line(r.stdout)
    assert j["n_gpus"] == 1 and j["ranks_reported"] == [0]


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "4", "--device", "cpu"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "refusing" in (r.stderr + r.stdout)
