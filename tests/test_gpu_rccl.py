"""RCCL itself on the one-GPU box: tests/rccl_loopback.py in a fresh child process (torch and
the GPU are initialised there, after the nccl rendezvous env is set) -- the nccl process group,
the gloo group next to it, records of a 2-rank vertex partition through RCCL on device tensors,
the engines' stream waits before the unpack, and the partitioned runs == one engine.
Anchor: the cross-host fan-out of NodeConnection.send, p2pnetwork/nodeconnection.py:107-160."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_world1_exchange_in_child():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", LOCAL_RANK="0",
               WORLD_SIZE="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_loopback.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    assert "RCCL OK" in p.stdout, p.stdout[-2000:]
    print(p.stdout.strip().splitlines()[-1])
