"""bench.py's launch contract (CPU only; nothing here touches a GPU).

  * `bench.py --gpus N` (N > 1) outside torchrun starts torchrun with N ranks as a CHILD process
    (the plan is printed by --dry-run): the driver's 8-GPU run cannot silently measure one GPU.
  * Under torchrun a WORLD_SIZE that differs from --gpus exits non-zero before any work.
  * No flags: one GPU, in process.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, world=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if world is not None:
        env["WORLD_SIZE"] = str(world)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=120)


def test_gpus_n_launches_torchrun_child():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["plan"] == "launch"
    cmd = plan["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    i = cmd.index(BENCH)
    assert cmd[i + 1:] == ["--gpus", "2", "--steps", "3", "--warmup", "1"]  # --dry-run not forwarded


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--dry-run"], world=4)
    assert r.returncode != 0 and json.loads(r.stdout.strip())["plan"] == "error"
    r = _run(["--gpus", "2", "--steps", "1"], world=4)  # the real run: refused before any work
    assert r.returncode != 0 and "WORLD_SIZE=4" in r.stderr


def test_default_is_one_gpu_in_process():
    for args, world in (([], None), (["--gpus", "1"], None), ([], 2), (["--gpus", "2"], 2)):
        r = _run(args + ["--dry-run"], world=world)
        assert r.returncode == 0 and json.loads(r.stdout.strip())["plan"] == "run", (args, world, r.stdout)
