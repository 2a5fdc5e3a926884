"""GPU parity of the RK2 (explicit midpoint) block and network — BASELINE
config 5, an extension the reference does not have (it integrates with
forward Euler, tfkeras_resnets.py:69-92).  Parity is against the oracle's
composition of the reference's Euler-block operations (oracle.rk2_fwd /
rk2_bwd, themselves pinned by finite differences in test_oracle.py).

Tolerances (as test_gpu_kernels.py / test_gpu_network.py):
  fp32: |gpu - oracle| <= 2e-5 * max|oracle| + 1e-5 * |oracle| (activations,
        dx); weight gradients within 1e-4 of max|oracle| (two conv stages).
  bf16: the oracle is fed the GPU's bf16 midpoint and masks and the same
        bf16-rounded inputs/W; outputs 2^-8 relative + 4e-3 * max|oracle|,
        weight gradients within 2e-3 of max|oracle|; network: probs within
        2e-2, loss within 1%, gradient relative L2 <= 2e-2 per group (conv1, each block's merged theta and bias, fc).
"""
import numpy as np
import pytest

from helpers import assert_close, assert_grad_groups_rel_l2, bf16_round, decode_mask, w_bf16_balanced
from oracle import asr_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def rt():
    from differential_equations_resnet_amd import runtime
    runtime.require_gpu()
    return runtime


def _theta(C, seed):
    return O.flatten(O.init_theta_3by3(C, np.random.default_rng(seed), np.float64)).astype(np.float32)


SHAPES = [("f32", (2, 32, 32, 16)), ("f32", (1, 7, 13, 5)), ("bf16", (2, 32, 32, 16)), ("bf16", (2, 32, 32, 32)),
          ("bf16", (2, 32, 32, 64)), ("bf16", (3, 11, 32, 64))]


@pytest.mark.parametrize("dtype_name,shape", SHAPES)
@pytest.mark.parametrize("gamma,h", [(0.0, 0.5), (-0.1, 1.0)])
def test_rk2_block_parity(rt, dtype_name, shape, gamma, h):
    N, H, W_, C = shape
    bf = dtype_name == "bf16"
    dtype = rt.ASR_BF16 if bf else rt.ASR_F32
    tdt = rt.torch_dtype(dtype)
    rng = np.random.default_rng(hash((shape, gamma, h)) % 2**32)
    x_np = rng.standard_normal(shape).astype(np.float32)
    dy_np = rng.standard_normal(shape).astype(np.float32)
    th = _theta(C, 13)
    b = (rng.standard_normal(C) * 0.1).astype(np.float32)
    dev = torch.device("cuda")
    pm = rt.param_map(C)
    w = rt.theta_to_w(torch.from_numpy(th).to(dev), C, pm, gamma, dtype)
    x = torch.from_numpy(x_np).to(dev).to(tdt).contiguous()
    bias = torch.from_numpy(b).to(dev)
    y, xm, m1, m2 = rt.rk2_forward(x, w, bias, h)
    dy = torch.from_numpy(dy_np).to(dev).to(tdt).contiguous()
    dx, dth, db, dw = rt.rk2_backward(dy, x, xm, m1, m2, w, pm, h, gamma, want_dw=True)

    src, sign = O.param_map(C)
    Wo = O.assemble_from_map(th.astype(np.float64), C, src, sign, gamma)
    q = (lambda a: bf16_round(a).astype(np.float64)) if bf else (lambda a: np.asarray(a, np.float64))
    Wo = w_bf16_balanced(Wo, src, sign).astype(np.float64) if bf else Wo
    xo, dyo = q(x_np), q(dy_np)
    # forward, stage by stage (stage 2 fed the GPU's midpoint)
    z1 = O.conv2d_same(xo, Wo) + b
    xm_want = xo + 0.5 * h * np.maximum(z1, 0)
    xm_gpu = xm.float().cpu().numpy().astype(np.float64)
    z2 = O.conv2d_same(xm_gpu, Wo) + b
    y_want = xo + h * np.maximum(z2, 0)
    if bf:
        lim = dict(rtol=2 ** -8)
        assert_close(xm_gpu, xm_want, atol=4e-3 * np.abs(xm_want).max(), what="bf16 xmid", **lim)
        assert_close(y.float().cpu().numpy(), y_want, atol=4e-3 * np.abs(y_want).max(), what="bf16 y", **lim)
    else:
        assert_close(xm_gpu, xm_want, rtol=1e-5, atol=2e-5 * np.abs(xm_want).max(), what="f32 xmid")
        assert_close(y.cpu().numpy(), y_want, rtol=1e-5, atol=2e-5 * np.abs(y_want).max(), what="f32 y")
    mk1 = decode_mask(m1.cpu().numpy(), N, H, W_, C)
    mk2 = decode_mask(m2.cpu().numpy(), N, H, W_, C)
    for m, z in ((mk1, z1), (mk2, z2)):
        sure = np.abs(z) > (2e-2 if bf else 1e-4) * np.abs(z).max()
        assert np.array_equal(m[sure], (z > 0)[sure]), "relu mask mismatch"
    # backward with the GPU's masks; bf16: the kernels stage dz in bf16 and
    # the inter-stage gradient g is a bf16 tensor
    dz2 = h * dyo * mk2
    dz2q = q(dz2)
    g = -O.conv2d_same(dz2q, Wo) + 2 * gamma * dz2q
    gq = q(g)
    dz1 = 0.5 * h * gq * mk1
    dz1q = q(dz1)
    dx_want = dyo + gq - O.conv2d_same(dz1q, Wo) + 2 * gamma * dz1q
    dW_want = O.conv2d_backprop_filter(xo, dz1q) + O.conv2d_backprop_filter(xm_gpu, dz2q)
    db_want = (dz1 + dz2).sum(axis=(0, 1, 2))
    dth_want = O.project_dW(dW_want, src, sign, pm.n_theta)
    sc = np.abs(dx_want).max()
    if bf:
        assert_close(dx.float().cpu().numpy(), dx_want, rtol=2 ** -7, atol=6e-3 * sc, what="bf16 dx")
        tol = 2e-3
    else:
        assert_close(dx.cpu().numpy(), dx_want, rtol=1e-5, atol=2e-5 * sc, what="f32 dx")
        tol = 1e-4
    assert_close(dw.cpu().numpy(), dW_want, rtol=0, atol=tol * np.abs(dW_want).max(), what="dW")
    assert_close(dth.cpu().numpy(), dth_want, rtol=0, atol=tol * np.abs(dth_want).max(), what="dtheta")
    assert_close(db.cpu().numpy(), db_want, rtol=0, atol=tol * max(np.abs(db_want).max(), 1), what="dbias")


def _setup(C, L, N, h, gamma=0.0, kind="3by3", anti=True, seed=0):
    spec = O.NetSpec(C=C, L=L, h=h, gamma=gamma, kind=kind, antisymmetric=anti, integrator="rk2")
    rng = np.random.default_rng(seed)
    params = [p.astype(np.float32).astype(np.float64) for p in O.init_params(spec, rng, np.float64, bias_std=0.05)]
    imgs = rng.integers(0, 256, (N, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10)[rng.integers(0, 10, N)]
    return spec, params, imgs, onehot


def _executor(spec, N, dtype):
    from differential_equations_resnet_amd.runtime import NetExecutor
    kinds = {"3by3": 0, "general": 1, "regular": 2}
    return NetExecutor(N, 32, 32, 3, spec.C, spec.L, 10, spec.h, spec.gamma, subtract_mean=127.5,
                       divide_by_stddev=127.5, dtype=dtype, input_u8=True, param_kind=kinds[spec.kind],
                       antisymmetric=spec.antisymmetric, integrator="rk2")


@pytest.mark.parametrize("gamma,kind,anti", [(-0.05, "3by3", True), (0.0, "regular", False)])
def test_rk2_network_fp32_parity(gamma, kind, anti):
    spec, params, imgs, onehot = _setup(16, 3, 4, 0.5, gamma, kind, anti)
    ex = _executor(spec, 4, "float32")
    flat = torch.from_numpy(O.flatten(params).astype(np.float32)).cuda()
    probs_gpu = ex.forward(flat, torch.from_numpy(imgs).cuda()).cpu().numpy()
    probs, cache = O.net_forward(spec, params, imgs)
    assert_close(probs_gpu, probs, rtol=1e-5, atol=1e-6, what="probs")
    loss, grads = ex.forward_backward(flat, torch.from_numpy(imgs).cuda(),
                                      torch.from_numpy(onehot.astype(np.float32)).cuda())
    want_loss = O.net_loss(probs, onehot)
    assert abs(loss.item() - want_loss) <= 1e-5 * abs(want_loss)
    g_want = O.net_backward(spec, params, cache, onehot)
    g_got = O.unflatten(grads.cpu().numpy().astype(np.float64), [p.shape for p in params])
    for i, (a, b) in enumerate(zip(g_got, g_want)):
        assert_close(a, b, rtol=0, atol=1e-4 * max(np.abs(b).max(), 1e-12), what=f"grad[{i}] {b.shape}")


@pytest.mark.parametrize("C", [16, 64])
def test_rk2_network_bf16_close(C):
    spec, params, imgs, onehot = _setup(C, 4, 8, 0.25, seed=1)
    ex = _executor(spec, 8, "bfloat16")
    flat = torch.from_numpy(O.flatten(params).astype(np.float32)).cuda()
    probs_gpu = ex.forward(flat, torch.from_numpy(imgs).cuda()).cpu().numpy()
    probs, cache = O.net_forward(spec, params, imgs)
    assert np.abs(probs_gpu - probs).max() < 2e-2
    loss, grads = ex.forward_backward(flat, torch.from_numpy(imgs).cuda(),
                                      torch.from_numpy(onehot.astype(np.float32)).cuda())
    assert abs(loss.item() - O.net_loss(probs, onehot)) <= 1e-2 * O.net_loss(probs, onehot)
    g_want = O.net_backward(spec, params, cache, onehot)
    g_got = O.unflatten(grads.cpu().numpy().astype(np.float64), [p.shape for p in params])
    assert_grad_groups_rel_l2(spec, g_got, g_want, 2e-2)


def test_rk2_model_lowering_matches_executor():
    """A Model built with integrator='rk2' lowers onto the RK2 executor and
    reproduces the oracle's probabilities (fp32)."""
    from differential_equations_resnet_amd import graph
    from differential_equations_resnet_amd.models import tfkeras_resnets as R
    graph.set_seed(4)
    fn = R.get_single_block_resnet_build_function(h=0.5, gamma=0.0, num_stages=2, blocks_per_stage=[2],
                                                  filters_per_block=[16], strides=[(1, 1)], subtract_mean=127.5,
                                                  divide_by_stddev=127.5, num_classes=10, integrator="rk2")
    m = fn(graph.Input(shape=(32, 32, 3)))
    imgs = np.random.default_rng(0).integers(0, 256, (4, 32, 32, 3)).astype(np.uint8)
    got = m.predict(imgs, batch_size=4, dtype="float32")
    spec = O.NetSpec(C=16, L=2, h=0.5, integrator="rk2")
    want, _ = O.net_forward(spec, [w.astype(np.float64) for w in m.get_weights()], imgs)
    assert_close(got, want, rtol=1e-5, atol=1e-6, what="rk2 model probs")


def test_rk2_forward_multiband(rt):
    """The RK2 second-stage forward (k_fwd_pipe<..., RESG>: residual read from
    global memory, loads issued one band ahead of their use) over a persistent
    run of several bands per workgroup: N=192 images of H=30 rows (8 bands
    each, the last band ragged: 30 is not a multiple of the band height 4)
    = 1536 items on a grid of at most 512 workgroups.  Every image's x_mid and
    y against the oracle (stage 2 fed the GPU's own bf16 midpoint), bf16
    tolerances as test_rk2_block_parity."""
    N, H, W_, C = 192, 30, 32, 64
    gamma, h = 0.0, 0.5
    rng = np.random.default_rng(4242)
    x_np = rng.standard_normal((N, H, W_, C)).astype(np.float32)
    th = _theta(C, 21)
    b = (rng.standard_normal(C) * 0.1).astype(np.float32)
    dev = torch.device("cuda")
    pm = rt.param_map(C)
    w = rt.theta_to_w(torch.from_numpy(th).to(dev), C, pm, gamma, rt.ASR_BF16)
    x = torch.from_numpy(x_np).to(dev).to(torch.bfloat16).contiguous()
    y, xm, m1, m2 = rt.rk2_forward(x, w, torch.from_numpy(b).to(dev), h)
    src, sign = O.param_map(C)
    Wo = w_bf16_balanced(O.assemble_from_map(th.astype(np.float64), C, src, sign, gamma), src, sign).astype(np.float64)
    xo = bf16_round(x_np).astype(np.float64)
    xm_want = xo + 0.5 * h * np.maximum(O.conv2d_same(xo, Wo) + b, 0)
    xm_gpu = xm.float().cpu().numpy().astype(np.float64)
    y_want = xo + h * np.maximum(O.conv2d_same(xm_gpu, Wo) + b, 0)
    assert_close(xm_gpu, xm_want, rtol=2 ** -8, atol=4e-3 * np.abs(xm_want).max(), what="multiband xmid")
    assert_close(y.float().cpu().numpy(), y_want, rtol=2 ** -8, atol=4e-3 * np.abs(y_want).max(), what="multiband y")
