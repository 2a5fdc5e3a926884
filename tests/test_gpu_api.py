"""GPU tests of the drop-in surface: the antisymmetric layers called eagerly
on device tensors (forward + autograd backward through the C ABI), a
builder-made Model lowered onto the native executor (predict and gradients
against the oracle), and the Training driver end to end.

Tolerances: fp32 as tests/test_gpu_kernels.py (|d| <= 2e-5 max|ref| +
1e-5 |ref|; weight gradients 1e-4 of max|ref|); bf16 layer outputs
2^-8 relative + 4e-3 max|ref|, bf16 weight gradients 1e-3 of max|ref|
(the oracle gets the same bf16-rounded inputs)."""
import csv
import os

import numpy as np
import pytest

from helpers import assert_close, bf16_round, w_bf16_balanced
from oracle import asr_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from differential_equations_resnet_amd import graph  # noqa: E402
from differential_equations_resnet_amd.graph import Input  # noqa: E402
from differential_equations_resnet_amd.layers import Conv2DAntisymmetric, Conv2DAntisymmetric3By3  # noqa: E402
from differential_equations_resnet_amd.models import tfkeras_resnets as R  # noqa: E402


def _layer_case(layer, shape, dtype, seed):
    N, H, W, C = shape
    graph.set_seed(seed)
    layer(Input(shape=(H, W, C)))
    rng = np.random.default_rng(seed)
    if layer.bias is not None:
        layer.bias.assign(rng.standard_normal(C) * 0.1)
    x_np = rng.standard_normal(shape).astype(np.float32)
    r_np = rng.standard_normal(shape).astype(np.float32)
    x = torch.from_numpy(x_np).cuda().to(dtype).requires_grad_(True)
    y = layer(x)
    y.backward(torch.from_numpy(r_np).cuda().to(dtype))
    th, b = layer.device_variables(x.device)
    bf = dtype == torch.bfloat16
    xo = bf16_round(x_np).astype(np.float64) if bf else x_np.astype(np.float64)
    ro = bf16_round(r_np).astype(np.float64) if bf else r_np.astype(np.float64)
    Wk = layer.get_kernel().astype(np.float64)
    src = layer.param_map().w_src
    sign = np.where(src & 1, -1, 1)
    osrc = np.where(src >= 0, src >> 1, -1)
    Wo = w_bf16_balanced(Wk, osrc, sign).astype(np.float64) if bf else Wk
    bias = layer.bias.value.astype(np.float64) if layer.bias is not None else 0.0
    want_y = O.conv2d_same(xo, Wo) + bias
    want_dx = O.conv2d_backprop_input(ro, Wo, xo.shape)
    dW = O.conv2d_backprop_filter(xo, ro)
    dth = O.project_dW(dW, osrc, sign, layer.theta_flat().size)
    return y, x.grad, th.grad, b.grad if b is not None else None, want_y, want_dx, dth, ro.sum(axis=(0, 1, 2)), bf


@pytest.mark.parametrize("make,shape,dtype", [
    (lambda: Conv2DAntisymmetric3By3(gamma=-0.1), (2, 7, 9, 5), torch.float32),
    (lambda: Conv2DAntisymmetric(3, gamma=0.2), (1, 6, 5, 4), torch.float32),
    (lambda: Conv2DAntisymmetric(3, antisymmetric=False), (2, 5, 6, 3), torch.float32),
    (lambda: Conv2DAntisymmetric3By3(), (2, 32, 32, 16), torch.bfloat16),
    (lambda: Conv2DAntisymmetric(3, antisymmetric=False), (2, 32, 32, 32), torch.bfloat16),
    (lambda: Conv2DAntisymmetric3By3(use_bias=False), (1, 8, 8, 6), torch.float32),
    # bf16 at the multi-stage nets' widths (k_convb's bare-conv modes, round 6)
    (lambda: Conv2DAntisymmetric3By3(gamma=-0.1), (2, 16, 16, 32), torch.bfloat16),
    (lambda: Conv2DAntisymmetric3By3(), (3, 7, 8, 64), torch.bfloat16),
    (lambda: Conv2DAntisymmetric(3, antisymmetric=False), (2, 16, 16, 16), torch.bfloat16),
])
def test_layer_eager_forward_backward(make, shape, dtype):
    y, dx, dth, db, want_y, want_dx, want_dth, want_db, bf = _layer_case(make(), shape, dtype, 5)
    sc = np.abs(want_y).max()
    if bf:
        assert_close(y.float().detach().cpu().numpy(), want_y, rtol=2 ** -8, atol=4e-3 * sc, what="bf16 y")
        assert_close(dx.float().cpu().numpy(), want_dx, rtol=2 ** -8, atol=4e-3 * np.abs(want_dx).max(),
                     what="bf16 dx")
        tol = 1e-3
    else:
        assert_close(y.detach().cpu().numpy(), want_y, rtol=1e-5, atol=2e-5 * sc, what="y")
        assert_close(dx.cpu().numpy(), want_dx, rtol=1e-5, atol=2e-5 * np.abs(want_dx).max(), what="dx")
        tol = 1e-4
    assert_close(dth.cpu().numpy(), want_dth, rtol=0, atol=tol * np.abs(want_dth).max(), what="dtheta")
    if db is not None:
        assert_close(db.cpu().numpy(), want_db, rtol=0, atol=tol * max(np.abs(want_db).max(), 1), what="dbias")


def test_layer_eager_is_native():
    """The eager layer runs in libasr (no torch conv): an unsupported shape
    fails loudly instead of falling back."""
    from differential_equations_resnet_amd._lib import AsrUnsupported
    layer = Conv2DAntisymmetric3By3()
    layer(Input(shape=(8, 8, 12)))
    with pytest.raises(AsrUnsupported):
        layer(torch.zeros(1, 8, 8, 12, device="cuda", dtype=torch.bfloat16))  # bf16 needs C in {16,32,64}
    strided = Conv2DAntisymmetric3By3(strides=(2, 2))
    strided(Input(shape=(8, 8, 4)))
    with pytest.raises(AsrUnsupported):
        strided(torch.zeros(1, 8, 8, 4, device="cuda"))


def _model(C, L, h, gamma=0.0, kernel_type="antisymmetric", seed=0):
    graph.set_seed(seed)
    fn = R.get_single_block_resnet_build_function(kernel_type=kernel_type, h=h, gamma=gamma, num_stages=2,
                                                  blocks_per_stage=[L], filters_per_block=[C], strides=[(1, 1)],
                                                  subtract_mean=127.5, divide_by_stddev=127.5, num_classes=10)
    return fn(Input(shape=(32, 32, 3)))


@pytest.mark.parametrize("kernel_type", ["antisymmetric", "regular"])
def test_model_lowering_matches_oracle(kernel_type):
    C, L, N = 16, 3, 5
    m = _model(C, L, 0.5, -0.05 if kernel_type == "antisymmetric" else 0.0, kernel_type)
    rng = np.random.default_rng(1)
    # non-zero biases exercise the path (the reference initialises zeros)
    ws = [w if w.ndim > 1 else (rng.standard_normal(w.shape) * 0.05).astype(np.float32) for w in m.get_weights()]
    m.set_weights(ws)
    imgs = rng.integers(0, 256, (N, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10)[rng.integers(0, 10, N)]
    spec = O.NetSpec(C=C, L=L, h=0.5, gamma=-0.05 if kernel_type == "antisymmetric" else 0.0,
                     kind="3by3" if kernel_type == "antisymmetric" else "regular",
                     antisymmetric=kernel_type == "antisymmetric")
    params = [w.astype(np.float64) for w in m.get_weights()]
    probs, cache = O.net_forward(spec, params, imgs)
    got = m.predict(imgs, batch_size=4, dtype="float32")  # 2 batches, the last zero-padded
    assert_close(got, probs, rtol=1e-5, atol=1e-6, what="predict")
    nm = m.compile_native(N, "float32")
    loss, grads, _ = nm.forward_backward(imgs, onehot.astype(np.float32))
    assert abs(loss.item() - O.net_loss(probs, onehot)) <= 1e-5 * O.net_loss(probs, onehot)
    g_want = O.net_backward(spec, params, cache, onehot)
    g_got = O.unflatten(grads.cpu().numpy().astype(np.float64), [p.shape for p in params])
    for i, (a, b) in enumerate(zip(g_got, g_want)):
        assert_close(a, b, rtol=0, atol=1e-4 * max(np.abs(b).max(), 1e-12), what=f"grad[{i}]")


def test_training_driver_end_to_end(tmp_path):
    from differential_equations_resnet_amd.dataset_utils import ArrayDataset
    from differential_equations_resnet_amd.training import AdamOptimizer, Training
    rng = np.random.default_rng(0)
    n, B = 64, 16
    feats = rng.integers(0, 256, (n, 32, 32, 3)).astype(np.uint8)
    labels = rng.integers(0, 10, n)
    ds = ArrayDataset(feats, labels, B, seed=1, num_classes=10)
    graph.set_seed(0)
    build = R.get_single_block_resnet_build_function(h=0.5, num_stages=2, blocks_per_stage=[3],
                                                     filters_per_block=[16], strides=[(1, 1)], subtract_mean=127.5,
                                                     divide_by_stddev=127.5, num_classes=10)
    tr = Training(build, "antisymmetric", AdamOptimizer(epsilon=1e-7), train_dataset=ds, val_dataset=ds,
                  summaries_dir=str(tmp_path), summaries_name="run", csv_logger_dir=str(tmp_path),
                  csv_logger_name="gradient_history", dtype="float32")
    # gradient mean-norms match a host recomputation from the same gradient buffer
    norms = tr.train_step(1e-3, with_norms=True)
    g = tr.native.executor(True).grads.cpu().numpy().astype(np.float64)
    plan = tr.native.plan
    want0 = np.linalg.norm(g[:plan.conv1.kernel.value.size]) / plan.conv1.kernel.value.size
    assert abs(norms[0] - want0) <= 1e-5 * want0
    assert len(norms) == 1 + 3
    tr.train(epochs=2, steps_per_epoch=4, learning_rate_schedule=lambda s: 1e-3, eval_dataset="val",
             eval_frequency=1, eval_steps=2, summaries_frequency=2)
    assert tr.g_step == 9
    rows = list(csv.reader(open(tmp_path / "run_gradient_history.csv"), delimiter=" "))
    assert rows[0][:3] == ["global_step", "mean_loss", "accuracy"]
    assert rows[0][3] == "conv1_kernel_gradient_mean_norm" and rows[0][4] == "res2_0_branch2_kernel_gradient_mean_norm"
    assert len(rows) > 2 and all(len(r) == len(rows[0]) for r in rows)
    ev = list(csv.reader(open(tmp_path / "run_evaluation_metrics.csv"), delimiter=" "))
    assert ev[0] == ["global_step", "mean_loss", "accuracy"] and len(ev) == 3
    res = tr.evaluate("val", 4)
    assert 0.0 <= res["accuracy"] <= 1.0 and np.isfinite(res["mean_loss"])
    # predict() and the evaluation metrics (native CE from the probabilities,
    # argmax accuracy) equal the oracle's on the trained parameters
    probs = tr.predict(feats[:B], argmax=False)
    spec = O.NetSpec(C=16, L=3, h=0.5)
    params = [w.astype(np.float64) for w in tr.model.get_weights()]
    want, _ = O.net_forward(spec, params, feats[:B])
    assert_close(probs, want, rtol=1e-5, atol=1e-6, what="Training.predict")
    one = ArrayDataset(feats[:B], labels[:B], B, shuffle=False, num_classes=10)
    tr._val_iter = iter(one)
    res1 = tr.evaluate("val", 1)
    onehot = np.eye(10)[labels[:B]]
    assert abs(res1["mean_loss"] - O.net_loss(want, onehot)) <= 1e-5 * O.net_loss(want, onehot)
    assert res1["accuracy"] == float((want.argmax(1) == labels[:B]).mean())
    path = tr.save(str(tmp_path / "ckpt"), "train_saver")
    assert path and os.path.exists(os.path.join(path, "variables.npz")) and "globalstep-9" in path
    w_before = tr.model.get_weights()
    tr.train_step(1e-3)
    tr.load_variables(path)
    for a, b in zip(tr.model.get_weights(), w_before):
        np.testing.assert_array_equal(a, b)
    assert tr.g_step == 9
    tr.close()


def test_training_overfits_one_batch():
    from differential_equations_resnet_amd.dataset_utils import ArrayDataset
    from differential_equations_resnet_amd.training import AdamOptimizer, Training
    rng = np.random.default_rng(2)
    labels = rng.integers(0, 4, 32)  # learnable: the class sets the image brightness
    feats = np.clip(labels[:, None, None, None] * 60 + 20 + rng.integers(-15, 16, (32, 32, 32, 3)), 0,
                    255).astype(np.uint8)
    ds = ArrayDataset(feats, labels, 32, shuffle=False, num_classes=10)
    graph.set_seed(0)
    build = R.get_single_block_resnet_build_function(h=0.25, num_stages=2, blocks_per_stage=[4],
                                                     filters_per_block=[16], strides=[(1, 1)], subtract_mean=127.5,
                                                     divide_by_stddev=127.5, num_classes=10)
    tr = Training(build, "antisymmetric", AdamOptimizer(epsilon=1e-7), train_dataset=ds, record_summaries=False)
    first = tr.evaluate("train", 1)["mean_loss"]
    for _ in range(60):
        tr.train_step(3e-3)
    last = tr.evaluate("train", 1)["mean_loss"]
    assert last < 0.5 * first, (first, last)


def _merged_theta_norms(spec, grads):
    """The reference's per-layer gradient mean-norms for an antisymmetric
    model (training.py:385-409, generalised from the hard-coded 20 variables):
    conv1's kernel, then per block ||merged theta gradient||_2 / size (bias
    excluded)."""
    out = [np.linalg.norm(grads[0]) / grads[0].size]
    nt = 4 + spec.C - 1
    i = 2
    for _ in range(spec.L):
        th = np.concatenate([g.ravel() for g in grads[i:i + nt]])
        out.append(np.linalg.norm(th) / th.size)
        i += nt + 1
    return out


def test_training_metrics_match_oracle(tmp_path):
    """Three Training.train_step calls on one fixed batch (fp32): every
    per-block merged-theta gradient mean-norm equals the oracle's on the same
    parameters (the device's, read back before each step; 1e-5 relative), and
    the streaming mean_loss / accuracy equal the oracle's means over the three
    steps (training.py:316-354, :385-409, :578-597).  The Adam update itself
    is checked against the oracle in test_gpu_kernels.py."""
    from differential_equations_resnet_amd.dataset_utils import ArrayDataset
    from differential_equations_resnet_amd.training import AdamOptimizer, Training
    rng = np.random.default_rng(5)
    B, C, L, h = 8, 16, 3, 0.5
    feats = rng.integers(0, 256, (B, 32, 32, 3)).astype(np.uint8)
    labels = rng.integers(0, 10, B)
    onehot = np.eye(10)[labels]
    ds = ArrayDataset(feats, labels, B, shuffle=False, num_classes=10)
    graph.set_seed(3)
    build = R.get_single_block_resnet_build_function(h=h, num_stages=2, blocks_per_stage=[L],
                                                     filters_per_block=[C], strides=[(1, 1)], subtract_mean=127.5,
                                                     divide_by_stddev=127.5, num_classes=10)
    tr = Training(build, "antisymmetric", AdamOptimizer(epsilon=1e-7), train_dataset=ds,
                  summaries_dir=str(tmp_path), summaries_name="run", csv_logger_dir=str(tmp_path),
                  csv_logger_name="gradient_history", dtype="float32")
    spec = O.NetSpec(C=C, L=L, h=h)
    losses, correct = [], 0
    tr._reset_metrics()
    for t in range(1, 4):
        params = [w.astype(np.float64) for w in tr.model.get_weights()]
        probs, cache = O.net_forward(spec, params, feats)
        grads = O.net_backward(spec, params, cache, onehot)
        losses.append(O.net_loss(probs, onehot))
        correct += int((probs.argmax(1) == labels).sum())
        want_norms = _merged_theta_norms(spec, grads)
        got_norms = tr.train_step(1e-3, with_norms=True)
        assert len(got_norms) == 1 + L
        assert_close(got_norms, want_norms, rtol=1e-5, what=f"step {t} gradient mean-norms")
    mean_loss, acc = tr._metric_values()
    assert abs(mean_loss - np.mean(losses)) <= 1e-5 * np.mean(losses)
    assert acc == correct / (3 * B)
    tr.close()


def test_native_state_shared_across_batch_sizes(tmp_path):
    """One device parameter set per Model: predict() at another batch size
    or dtype after training reads the trained parameters, get_weights and
    save/load_variables see them, and training continues from them (ADVICE
    r01: executors used to snapshot the weights when re-lowered)."""
    from differential_equations_resnet_amd.dataset_utils import ArrayDataset
    from differential_equations_resnet_amd.training import AdamOptimizer, Training
    rng = np.random.default_rng(9)
    feats = rng.integers(0, 256, (8, 32, 32, 3)).astype(np.uint8)
    labels = rng.integers(0, 10, 8)
    ds = ArrayDataset(feats, labels, 8, shuffle=False, num_classes=10)
    graph.set_seed(1)
    build = R.get_single_block_resnet_build_function(h=0.5, num_stages=2, blocks_per_stage=[2],
                                                     filters_per_block=[16], strides=[(1, 1)], subtract_mean=127.5,
                                                     divide_by_stddev=127.5, num_classes=10)
    tr = Training(build, "antisymmetric", AdamOptimizer(epsilon=1e-7), train_dataset=ds, record_summaries=False,
                  dtype="float32")
    spec = O.NetSpec(C=16, L=2, h=0.5)
    tr.train_step(1e-2)
    p1 = tr.model.predict(feats[:3], batch_size=3, dtype="float32")  # a new executor (batch 3)
    w1 = [w.astype(np.float64) for w in tr.model.get_weights()]
    assert_close(p1, O.net_forward(spec, w1, feats[:3])[0], rtol=1e-5, atol=1e-6, what="predict after step 1")
    tr.train_step(1e-2)  # continues from the trained parameters
    w2 = [w.astype(np.float64) for w in tr.model.get_weights()]
    assert any(np.abs(a - b).max() > 0 for a, b in zip(w1, w2))
    p2 = tr.model.predict(feats[:3], batch_size=3, dtype="float32")
    assert_close(p2, O.net_forward(spec, w2, feats[:3])[0], rtol=1e-5, atol=1e-6, what="predict after step 2")
    path = tr.save(str(tmp_path / "ckpt"), "train_saver")
    tr.train_step(1e-2)
    tr.load_variables(path)  # restores every executor's parameters, the training one included
    for a, b in zip(tr.model.get_weights(), w2):
        np.testing.assert_array_equal(a, b.astype(np.float32))
    p3 = tr.model.predict(feats[:3], batch_size=3, dtype="float32")
    np.testing.assert_array_equal(p3, p2)
    tr.close()
