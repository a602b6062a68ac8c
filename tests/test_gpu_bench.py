"""bench.py's own multi-rank code path (it had never run with
world > 1).  Two ranks share the box's one GPU over gloo (RCCL refuses two
ranks on one device): torch.distributed.run launches bench.py exactly as the
driver does for N > 1, with --backend gloo; the global batch is fixed
(--scaling strong), so the reduced best key and the global top-E of the
elite exchange must equal a one-process run over the same batch."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--config", "c3", "--scaling", "strong", "--candidates", "512", "--steps", "2", "--warmup", "1",
          "--exchange", "elite", "--no-cpu-baseline", "--no-contact-report"]


def _port():
    """A free port below the ephemeral range (32768..): an ephemeral pick can
    be taken, before the rendezvous binds it, by a client socket of the
    spawned ranks (the Manager connection) -- EADDRINUSE on the box, r05."""
    import random
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
        return p
    raise RuntimeError("no free port in 20000..32000")


def _run(cmd):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    # a rank's traceback sits in the middle of torchrun's stderr: keep its lines
    ranks = "\n".join(ln for ln in r.stderr.splitlines() if ln.startswith("[rank"))[-6000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], ranks or r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_equal_one_gpu():
    one = _run([sys.executable, "bench.py"] + COMMON)
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                "--backend", "gloo"] + COMMON)
    assert one["config"]["world_size_seen"] == 1
    assert two["config"]["world_size_seen"] == 2 and two["config"]["backend"] == "gloo"
    assert two["n_gpus"] == 2 and two["config"]["candidates_per_gpu"] == 256
    # the global best (8-byte key MIN all-reduce) and the global top-E of the
    # elite exchange (local top-E, all-gather, global top-E), both in the timed step
    assert two["best"] == one["best"], (one["best"], two["best"])
    assert two["elites"]["k"] == one["elites"]["k"] == int(0.05 * 512)
    assert two["elites"]["exchanges_timed"] == 2
    assert two["elites"]["cost_sum"] == one["elites"]["cost_sum"]
    assert two["elites"]["first"] == one["elites"]["first"]


def test_bench_self_launch_two_ranks_equal_one_gpu():
    """`python bench.py --gpus 2` without torchrun: the
    parent spawns the two ranks itself; same best and elites as one GPU, and
    the multi-rank line carries no borrowed one-GPU counters."""
    one = _run([sys.executable, "bench.py"] + COMMON)
    env_clean = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo"] + COMMON, cwd=ROOT,
                       env=env_clean, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    two = json.loads(lines[0])
    assert two["config"]["launcher"] == "bench.py self-launch"
    assert two["config"]["world_size_seen"] == 2 and two["config"]["backend"] == "gloo"
    assert "gloo" in two["config"]["exchange"] and "RCCL" not in two["config"]["exchange"]
    assert two["roofline"]["traffic"] is None and "valu" not in two["roofline"]
    assert two["best"] == one["best"]
    assert two["elites"]["cost_sum"] == one["elites"]["cost_sum"]
    assert two["elites"]["first"] == one["elites"]["first"]


SUB = ["--config", "c3", "--candidates", "4096", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
       "--no-contact-report"]


def test_bench_default_line_carries_strong_and_c5_at_two_ranks():
    """The default line's sub-records: at world 2 (gloo,
    two ranks sharing the box's GPU) the C3 strong reading (4096 global, 2048
    per rank) selects the same best candidate as one process, and the C5 tick
    (8192 global, 4096 per rank, 3 CEM iterations, graph replay with the
    exchange between replays) ends with the same per-iteration best costs."""
    one = _run([sys.executable, "bench.py"] + SUB)
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                "--backend", "gloo"] + SUB)
    for rec, w in ((one, 1), (two, 2)):
        st, c5 = rec["strong"], rec["c5"]
        assert st["scaling"] == "strong" and st["global_batch"] == 4096 and st["candidates_per_gpu"] == 4096 // w
        assert c5["scaling"] == "strong" and c5["global_batch"] == 8192 and c5["candidates_per_gpu"] == 8192 // w
        assert st["value"] > 0 and c5["value"] > 0 and len(c5["best_cost"]) == 3
    assert two["strong"]["best"] == one["strong"]["best"]
    # weak: each rank's own 4096 (rank 0's draw is the strong global batch)
    assert one["strong"]["best"] == one["best"]
    assert two["c5"]["best_cost"] == one["c5"]["best_cost"], (one["c5"], two["c5"])


def test_bench_c5_line():
    """--config c5: the closed-loop tick as the line (strong scaling), the
    rollout kernel's roofline from an eager call of the rank's share."""
    rec = _run([sys.executable, "bench.py", "--config", "c5", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    assert rec["scaling"] == "strong" and rec["config"]["global_batch"] == 8192
    assert rec["config"]["cem_iters"] == 3 and len(rec["best"]["cost_per_iteration"]) == 3
    assert rec["roofline"]["kernel_ms"] > 0 and 0 < rec["roofline"]["frac"] < 1
    assert abs(rec["value"] - 8192 * 3 * 2 / (2 * rec["ms_per_step"] * 1e-3)) < 0.01 * rec["value"]
