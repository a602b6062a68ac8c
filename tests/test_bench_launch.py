"""bench.py's self-launch path: `python bench.py --gpus N`
outside torch.distributed.run starts N fresh rank processes itself (the parent
never imports torch), rank 0's JSON line is the output and the exit code is
the worst rank's.  The plumbing runs here on CPU through the hidden
--launch-selftest hook (gloo group, one all-reduce); tests/test_gpu_bench.py
runs the real bench through the same path on the GPU box."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=180)


def test_self_launch_two_ranks():
    r = _bench(["--gpus", "2", "--launch-selftest"])
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["world"] == 2 and rec["sum_ranks_plus_1"] == 3
    assert rec["env"]["WORLD_SIZE"] == "2" and rec["env"]["RANK"] == "0" and rec["env"]["MASTER_ADDR"] == "127.0.0.1"


def test_self_launch_four_ranks():
    r = _bench(["--gpus", "4", "--launch-selftest"])
    assert r.returncode == 0, r.stderr[-4000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["world"] == 4 and rec["sum_ranks_plus_1"] == 10


def test_self_launch_failing_rank_fails_the_run():
    # rank 1 exits 3 before joining; rank 0 blocks in the rendezvous and is
    # killed after the grace period: the parent returns the worst code
    r = _bench(["--gpus", "2", "--launch-selftest"], {"MPCR_SELFTEST_FAIL_RANK": "1", "TORCH_DIST_INIT_BARRIER": "0"})
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_parent_does_not_import_torch():
    # the launcher returns before the parent imports torch (so it cannot
    # initialise the GPU): bench.py keeps torch imports inside main()'s rank path
    src = open(os.path.join(ROOT, "bench.py")).read()
    head = src.split("def main():")[0]
    assert "\nimport torch" not in head and "\nfrom torch" not in head
    body = src.split("def main():")[1]
    assert body.index("launch_ranks(") < body.index("import torch")
