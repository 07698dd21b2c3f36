"""The RCCL branch of the pose / result gathers (shard.py: all_gather_into_tensor under the
nccl backend), on the GPU: `torch.distributed.run --nproc-per-node 1` starts a fresh child
(tests/rccl_child.py) that initialises the nccl (= RCCL) process group on its GPU, solves a
ragged 7-pair batch with the library, and checks gather_poses (sync and async, the pose
buffers overwritten while the gather is in flight, as bench.py's loop does) and gather_rows
against the local solve bit for bit.  The parent only waits for the child (no re-exec).

One GPU box: world size 1 here (the driver's 8-GPU runs use the same calls at N = 2 / 4 / 8;
the N > 1 sharding and padding logic is covered with two gloo ranks in test_shard_gloo.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_pose_and_row_gathers_under_torchrun(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    out = tmp_path / "rccl.json"
    env = dict(os.environ, DPFT_RCCL_OUT=str(out), HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "rccl_child.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"child failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = json.loads(out.read_text())
    print("RCCL child:", res)
    assert res["backend"] == "nccl" and res["ok"], res
