"""bench.py's launch contract on CPU: `--gpus N` never silently runs fewer GPUs
(`--gpus` was parsed and ignored).  Without torchrun it spawns N rank
processes itself, which here (no GPU) must stop with a non-zero status before any
rank starts; under a launcher whose WORLD_SIZE disagrees it refuses."""
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=300)


def test_gpus_more_than_visible_fails_loudly():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "GPU" in r.stderr and "--gpus 2" in r.stderr


def test_gpus_disagreeing_with_launcher_world_size_fails():
    r = _run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
