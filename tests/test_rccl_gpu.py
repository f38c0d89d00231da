"""RCCL on the MI355X (one rank, world of one, collectives forced on): the native communicator,
the fused DenseNet-121 data-parallel step with its bucket all-reduces issued by the C++ plan, the
secure-aggregation int32 masked SUM and the FedAvg packed reduce / broadcast, all over the ``nccl``
(= RCCL) backend (tests/rccl_worker.py).  Reference: the NCCL all-reduce of
``tf.distribute.MirroredStrategy`` (``dist_model_tf_vgg.py:115-117``,
``dist_model_tf_dense.py:16-28``)."""
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


@pytest.mark.timeout(600)
def test_rccl_world_of_one(tmp_path):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4", PYTHONUNBUFFERED="1",
               IDC_FORCE_COLLECTIVES="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "rccl_worker.py")]
    out_dir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else str(tmp_path)
    log = os.path.join(out_dir, "rccl_worker.log")
    with open(log, "w") as f:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT, timeout=540)
    text = open(log).read()
    cases = {json.loads(l.split("RCCLCASE ", 1)[1])["case"]: json.loads(l.split("RCCLCASE ", 1)[1])
             for l in text.splitlines() if "RCCLCASE " in l}
    assert r.returncode == 0, text[-4000:]
    assert set(cases) == {"native", "nonblocking", "dp_det", "dp_tuned", "central", "masked",
                          "fedavg"}, text[-4000:]
    for c in cases.values():
        assert c["ok"], c
