"""Data parallelism through the NATIVE executor on the GPU (the
reference is single-device, experiments_antisymmetric_resnet_v6.ipynb:361).

Two ranks launched by torch.distributed.run (fresh processes; this process
only launches them), both on cuda:0 of the one-GPU box: each runs
asr_net_forward_backward on its half of a fixed global batch, all-reduces the
fp32 gradient buffer, and applies one replicated Adam step with grad_scale
1/world.  Checked against this process's single-rank native gradient of the
concatenated batch (the batch-mean loss makes it the mean of the ranks'):
|g_sum/2 - g_full| <= 1e-5 * max|g_full| (fp32, reduction-order noise), the
broadcast made the ranks' parameters identical, the Adam step is identical
on both ranks and equals a single-process step on the global gradient.

Backends: "gloo" (device tensors through torch.distributed/gloo) and "rccl"
(asr_dist_init / asr_dist_allreduce_sum / asr_dist_broadcast on librccl).
RCCL refuses two ranks on one device ("Duplicate GPU"), so the rccl case
gives each rank its own NCCL_HOSTID (the ranks then connect over loopback
sockets); the 8-GPU scaling run exercises RCCL over xGMI.
"""
import os
import signal
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dp_worker as W  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(outdir, backend, extra_env=None, timeout=90):
    """Run the two ranks in their own process group; on a hang the whole
    group (launcher and ranks) is killed."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dp_worker.py"),
           str(outdir), backend]
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, _ = p.communicate()
        pytest.fail(f"{backend} ranks hung for {timeout} s:\n{out[-3000:]}")
    return p.returncode, out


def _check(outdir):
    from differential_equations_resnet_amd import runtime as rt
    r = [np.load(os.path.join(outdir, f"r{i}.npz")) for i in range(2)]
    np.testing.assert_array_equal(r[0]["p0"], r[1]["p0"])  # broadcast from rank 0
    np.testing.assert_array_equal(r[0]["p0"], W.params0(100))
    np.testing.assert_array_equal(r[0]["g"], r[1]["g"])  # every rank holds the same sum
    np.testing.assert_array_equal(r[0]["p1"], r[1]["p1"])  # replicated Adam
    assert float(r[0]["t"]) == float(r[1]["t"]) == 2.0  # max over ranks (control plane)
    # single-rank native gradient of the concatenated batch
    dev = rt.require_gpu()
    imgs, onehot = W.global_batch(2)
    ex = rt.NetExecutor(2 * W.B, 32, 32, 3, W.C, W.L, 10, W.H, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                        dtype="float32", input_u8=True, device=dev)
    p = torch.from_numpy(r[0]["p0"]).to(dev)
    loss, g = ex.forward_backward(p, torch.from_numpy(imgs).to(dev), torch.from_numpy(onehot).to(dev))
    g_full = g.cpu().numpy()
    g_mean = r[0]["g"] / 2
    assert np.abs(g_mean - g_full).max() <= 1e-5 * np.abs(g_full).max(), np.abs(g_mean - g_full).max()
    assert abs(0.5 * (float(r[0]["loss"][0]) + float(r[1]["loss"][0])) - loss.item()) <= 1e-5 * loss.item()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    rt.adam_update(p, torch.from_numpy(r[0]["g"]).to(dev), m, v, 1e-3, 0.9, 0.999, 1e-7, 1, 0.5)
    np.testing.assert_array_equal(p.cpu().numpy(), r[0]["p1"])


def test_two_ranks_gloo_native(tmp_path):
    rc, out = _launch(tmp_path, "gloo")
    assert rc == 0, out[-3000:]
    _check(tmp_path)


def test_two_ranks_rccl_c_abi(tmp_path):
    rc, out = _launch(tmp_path, "rccl", {"ASR_TEST_SPLIT_HOSTID": "1", "NCCL_SOCKET_IFNAME": "lo",
                                         "NCCL_IB_DISABLE": "1"})
    if rc != 0 and "Duplicate GPU" in out:
        pytest.skip("RCCL refuses two ranks on one device even with split host ids")
    assert rc == 0, out[-3000:]
    _check(tmp_path)
