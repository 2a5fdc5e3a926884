"""World-size-2 data-parallel tests on CPU (gloo): the sharding of
ArrayDataset, the gradient all-reduce / 1-over-world mean, parameter
broadcast and max-over-ranks timing used by Training and bench.py.

The per-rank gradient here comes from the oracle (CPU); on the GPU the same
distributed helpers carry the native executor's gradient buffer
(tests/test_gpu_api.py covers that path on one device)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

WORLD = 2
B = 3  # images per rank


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    rng = np.random.default_rng(11)
    imgs = rng.integers(0, 256, (12, 5, 4, 3)).astype(np.uint8)
    labels = rng.integers(0, 10, 12)
    return imgs, labels


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    from oracle import asr_oracle as O
    from differential_equations_resnet_amd import distributed
    from differential_equations_resnet_amd.dataset_utils import ArrayDataset
    distributed.init_from_env("gloo")
    assert distributed.world_size() == WORLD and distributed.rank() == rank
    spec = O.NetSpec(C=4, L=2, h=0.5, H=5, W=4)
    params = O.init_params(spec, np.random.default_rng(100 + rank), bias_std=0.1)  # differs per rank ...
    flat = torch.from_numpy(O.flatten(params))
    distributed.broadcast_params(flat, 0)  # ... until broadcast from rank 0
    params = O.unflatten(flat.numpy(), [p.shape for p in params])
    imgs, labels = _data()
    ds = ArrayDataset(imgs, labels, B, seed=4, num_classes=10, rank=rank, world_size=WORLD,
                      device=torch.device("cpu"))
    x, y = next(iter(ds))
    probs, cache = O.net_forward(spec, params, x.numpy())
    g = torch.from_numpy(O.flatten(O.net_backward(spec, params, cache, y.numpy().astype(np.float64))))
    distributed.allreduce_grads(g)
    g /= WORLD
    t = distributed.max_over_ranks(1.0 + rank)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), g=g.numpy(), flat=flat.numpy(), t=t, x=x.numpy())
    distributed.shutdown()


def test_two_rank_gradient_equals_global_batch(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(port, str(tmp_path)), nprocs=WORLD, start_method="spawn")
    r = [np.load(tmp_path / f"r{i}.npz") for i in range(WORLD)]
    from oracle import asr_oracle as O
    from differential_equations_resnet_amd.dataset_utils import ArrayDataset
    np.testing.assert_array_equal(r[0]["flat"], r[1]["flat"])  # broadcast
    np.testing.assert_array_equal(r[0]["g"], r[1]["g"])        # identical reduced gradient on every rank
    assert float(r[0]["t"]) == float(r[1]["t"]) == 2.0         # max over ranks
    # the reduced gradient is the gradient of the mean loss over the global batch
    imgs, labels = _data()
    full = ArrayDataset(imgs, labels, B * WORLD, seed=4, num_classes=10, device=torch.device("cpu"))
    x, y = next(iter(full))
    np.testing.assert_array_equal(np.concatenate([r[0]["x"], r[1]["x"]]), x.numpy())
    spec = O.NetSpec(C=4, L=2, h=0.5, H=5, W=4)
    shapes = [s for s in spec.param_shapes()]
    params = O.unflatten(r[0]["flat"], shapes)
    probs, cache = O.net_forward(spec, params, x.numpy())
    want = O.flatten(O.net_backward(spec, params, cache, y.numpy().astype(np.float64)))
    np.testing.assert_allclose(r[0]["g"], want, rtol=1e-10, atol=1e-13)
