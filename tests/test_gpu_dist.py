"""The bench's collective path on real RCCL (one rank, --force-dist): process group, prompt
broadcast, per-step gather of the finished images, barriers and the max-over-ranks reduction --
the code every N > 1 run of the driver takes -- run as a child process under torch.distributed.run
with a 2-block model. Checks that it completes, prints one JSON line, and that the HIP hardware
queue count the bench raises before HIP initialises is what the rank ran with."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(*extra):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4")  # the box's default: bench.py must raise it
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--steps", "2", "--warmup", "1", "--layers", "2", "--no-cpu-baseline", "--force-dist", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_cfg_pairs_on_rccl_pair_of_one():
    """BASELINE configs[4]'s CFG axis on real RCCL: `--workload stream2-cfg --cfg-parallel` with one
    rank is a pair of one -- that rank carries both branches and the per-frame all_gather of the
    noise predictions, the pair group and the delivery group all run over RCCL (2-block model).
    The same run without --cfg-parallel (batched CFG, no exchange) must report the same batch."""
    line = _bench("--workload", "stream2-cfg", "--cfg-parallel")
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["value"] > 0
    assert "cfg-pair x1" in line["config"]["parallelism"] and line["config"]["global_batch"] == 4
    assert "configs[4]" in line["config"]["workload"]
    ref = _bench("--workload", "stream2-cfg")
    assert ref["config"]["global_batch"] == 4 and ref["config"]["parallelism"] == "single"


def test_bench_collective_path_one_rank():
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4")  # the box's default: bench.py must raise it
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--steps", "2", "--warmup", "1", "--layers", "2", "--no-cpu-baseline", "--force-dist"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["value"] > 0
    assert line["config"]["layers"] == 2 and line["config"]["global_batch"] == 2
    assert line["hip_hw_queues"] == 8
