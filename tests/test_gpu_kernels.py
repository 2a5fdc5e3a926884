"""GPU parity of the HIP kernels (through the C ABI) against the numpy oracle.

Tolerances (stated per north_star's "within a stated fp32 tolerance"):
  fp32 path  : |gpu - oracle| <= 2e-5 * max|oracle| + 1e-5 * |oracle|  (fp32 FMA chains of
               length 9C vs fp64)
  bf16 path  : the oracle is fed the SAME bf16-rounded inputs and W; the GPU
               accumulates in fp32 and rounds the output once, so
               |gpu - oracle| <= 2^-8 * |oracle| + 4e-3 * max|oracle| per element;
               weight gradients (fp32 outputs) within 1e-3 of max|oracle|.
Masks must agree exactly wherever |z| > 1e-4 * max|z| (fp32) / 2e-2 * max|z| (bf16).
"""
import numpy as np
import pytest

from helpers import assert_close, bf16_round, decode_mask, w_bf16_balanced
from oracle import asr_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def rt():
    from differential_equations_resnet_amd import runtime
    runtime.require_gpu()
    return runtime


def _theta(C, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    th = O.init_theta_3by3(C, rng, np.float64)
    return (O.flatten(th) * scale).astype(np.float32)


@pytest.mark.parametrize("C", [4, 16, 64])
@pytest.mark.parametrize("gamma", [0.0, -0.1])
def test_theta_to_w_f32_exact(rt, C, gamma):
    th = _theta(C, C)
    pm = rt.param_map(C)
    dev = torch.device("cuda")
    W = rt.theta_to_w(torch.from_numpy(th).to(dev), C, pm, gamma, rt.ASR_F32)[0].cpu().numpy()
    want = O.assemble_3by3_literal(O.unflatten(th.astype(np.float64), O.theta_shapes_3by3(C)), gamma)
    np.testing.assert_array_equal(W, want.astype(np.float32))


def test_theta_to_w_multi_layer(rt):
    C, L = 16, 3
    n = O.theta_count_3by3(C)
    stride = n + C
    flat = np.random.default_rng(5).standard_normal(L * stride).astype(np.float32)
    pm = rt.param_map(C)
    W = rt.theta_to_w(torch.from_numpy(flat).cuda(), C, pm, 0.0, rt.ASR_F32, layers=L, theta_stride=stride)
    W = W.cpu().numpy()
    src, sign = O.param_map(C)
    for l in range(L):
        want = O.assemble_from_map(flat[l * stride:l * stride + n].astype(np.float64), C, src, sign, 0.0)
        np.testing.assert_array_equal(W[l], want.astype(np.float32))


def _unpack_bf16(pack, C):
    """The MFMA W pack (include/asr.h) back to HWIO [3, 3, C, C] float32."""
    KS = (9 * C + 31) // 32
    o, kappa = np.meshgrid(np.arange(C), np.arange(9 * C), indexing="ij")
    idx = (((o // 16) * KS + kappa // 32) * 64 + (o % 16) + 16 * ((kappa % 32) // 8)) * 8 + kappa % 8
    Wt = pack[idx]  # [o, kappa = tap * C + i]
    return Wt.reshape(C, 9, C).transpose(1, 2, 0).reshape(3, 3, C, C)


@pytest.mark.parametrize("C,kind,anti,gamma,L", [(16, 0, True, 0.0, 3), (32, 0, True, -0.1, 2), (64, 0, True, 0.0, 2),
                                                 (64, 1, False, 0.05, 1), (32, 1, True, 0.0, 1), (16, 2, False, 0.0, 1),
                                                 (80, 0, True, 0.0, 1)])
def test_theta_to_w_bf16_pack_exact(rt, C, kind, anti, gamma, L):
    """asr_theta_to_w's bf16 pack bit for bit against helpers.w_bf16_balanced
    (the balanced rounding of the antisymmetric pairs: 3by3 and general maps,
    C <= 64), round-to-nearest for the regular kind and for C = 80 (above the
    balanced kernel's LDS)."""
    pm = rt.param_map(C, kind, anti)
    n = pm.n_theta
    stride = n + 8
    flat = (np.random.default_rng(C + kind).standard_normal(L * stride) * 0.2).astype(np.float32)
    w = rt.theta_to_w(torch.from_numpy(flat).cuda(), C, pm, gamma, rt.ASR_BF16, layers=L, theta_stride=stride)
    packs = w.view(torch.int16).cpu().numpy().reshape(L, -1)
    ws = pm.w_src.astype(np.int64)
    src, sign = np.where(ws >= 0, ws >> 1, -1), np.where(ws & 1, -1, 1)
    for l in range(L):
        W = O.assemble_from_map(flat[l * stride:l * stride + n].astype(np.float64), C, src, sign, gamma)
        want = w_bf16_balanced(W, src, sign) if C <= 64 else bf16_round(W)
        got = (packs[l].astype(np.uint16).astype(np.uint32) << 16).view(np.float32)
        np.testing.assert_array_equal(_unpack_bf16(got, C).view(np.uint32), want.view(np.uint32))
        if kind != 2 and C <= 64:  # balanced: differs from nearest somewhere, exactly antisymmetric off the diagonal
            assert not np.array_equal(want, bf16_round(W))


def _run_forward(rt, mode, x_np, th, b, C, gamma, h, dtype):
    dev = torch.device("cuda")
    pm = rt.param_map(C)
    tdt = rt.torch_dtype(dtype)
    x = torch.from_numpy(x_np).to(dev).to(tdt).contiguous()
    w = rt.theta_to_w(torch.from_numpy(th).to(dev), C, pm, gamma, dtype)
    N, H, W_, _ = x_np.shape
    mask = torch.zeros(rt.mask_bytes(N, H, W_, C), dtype=torch.uint8, device=dev)
    bias = torch.from_numpy(b).to(dev)
    y = rt.conv_forward(mode, x, w, bias, h, mask if mode == rt.ASR_MODE_EULER else None)
    return x, w, y, mask, pm


def _oracle_W(th, C, gamma, bf):
    src, sign = O.param_map(C)
    W = O.assemble_from_map(th.astype(np.float64), C, src, sign, gamma)
    return w_bf16_balanced(W, src, sign).astype(np.float64) if bf else W


SHAPES_BF16 = [(2, 32, 32, 16), (2, 32, 32, 32), (2, 32, 32, 64), (1, 11, 32, 64), (3, 5, 32, 16)]
# bf16 Euler blocks and bare convs (Conv2DAntisymmetric3By3.call, …3By3.py:157-171) at the multi-stage nets' widths
# (k_convb + k_wgradb: Euler mode since round 5, the bare conv since round 6)
SHAPES_BF16_W = [(2, 16, 16, 32), (3, 7, 16, 16), (2, 8, 8, 64), (2, 5, 8, 16), (1, 9, 8, 32), (2, 16, 16, 64),
                 (2, 32, 32, 64)]
SHAPES_F32 = [(2, 32, 32, 16), (1, 7, 13, 5), (2, 9, 32, 64), (1, 3, 3, 1), (2, 32, 32, 32), (3, 6, 32, 16),
              # the multi-stage nets' 16x16 / 8x8 stages on the same fp32 MFMA kernels (odd H: partial bands)
              (2, 16, 16, 32), (3, 7, 16, 16), (2, 8, 8, 64), (2, 5, 8, 16), (1, 9, 8, 32)]


@pytest.mark.parametrize("dtype_name,shape", [("f32", s) for s in SHAPES_F32] + [("bf16", s) for s in SHAPES_BF16]
                         + [("bf16w", s) for s in SHAPES_BF16_W])
@pytest.mark.parametrize("mode_name", ["euler", "conv"])
@pytest.mark.parametrize("gamma,h", [(0.0, 0.25), (-0.1, 1.0)])
def test_forward_parity(rt, dtype_name, shape, mode_name, gamma, h):
    N, H, W_, C = shape
    if dtype_name == "bf16w":
        if W_ == 32:
            pytest.skip("W = 32 runs the C=16/32/64 band kernels (SHAPES_BF16); k_convb at W = 32 via the stages")
    bf = dtype_name.startswith("bf16")
    dtype = rt.ASR_BF16 if bf else rt.ASR_F32
    mode = rt.ASR_MODE_EULER if mode_name == "euler" else rt.ASR_MODE_CONV
    rng = np.random.default_rng(hash((shape, mode_name, gamma)) % 2**32)
    x_np = rng.standard_normal(shape).astype(np.float32)
    th = _theta(C, 7, scale=1.0)
    b = (rng.standard_normal(C) * 0.1).astype(np.float32)
    x, w, y, mask, _ = _run_forward(rt, mode, x_np, th, b, C, gamma, h, dtype)
    xo = bf16_round(x_np).astype(np.float64) if bf else x_np.astype(np.float64)
    Wo = _oracle_W(th, C, gamma, bf)
    z = O.conv2d_same(xo, Wo) + b
    if mode == rt.ASR_MODE_EULER:
        want = xo + h * np.maximum(z, 0)
    else:
        want = z
    got = y.float().cpu().numpy()
    scale = np.abs(want).max()
    if bf:
        assert_close(got, want, rtol=2 ** -8, atol=4e-3 * scale, what="bf16 forward")
    else:
        assert_close(got, want, rtol=1e-5, atol=2e-5 * scale, what="f32 forward")
    if mode == rt.ASR_MODE_EULER:
        m = decode_mask(mask.cpu().numpy(), N, H, W_, C)
        sure = np.abs(z) > (2e-2 if bf else 1e-4) * np.abs(z).max()
        assert np.array_equal(m[sure], (z > 0)[sure]), "relu mask mismatch"


@pytest.mark.parametrize("dtype_name,shape", [("f32", s) for s in SHAPES_F32] + [("bf16", s) for s in SHAPES_BF16]
                         + [("bf16w", s) for s in SHAPES_BF16_W])
@pytest.mark.parametrize("mode_name", ["euler", "conv"])
@pytest.mark.parametrize("gamma,h", [(0.0, 0.25), (-0.1, 1.0)])
def test_backward_parity(rt, dtype_name, shape, mode_name, gamma, h):
    N, H, W_, C = shape
    if dtype_name == "bf16w":
        if W_ == 32:
            pytest.skip("W = 32 runs the C=16/32/64 band kernels (SHAPES_BF16); k_convb at W = 32 via the stages")
    bf = dtype_name.startswith("bf16")
    dtype = rt.ASR_BF16 if bf else rt.ASR_F32
    mode = rt.ASR_MODE_EULER if mode_name == "euler" else rt.ASR_MODE_CONV
    rng = np.random.default_rng(hash((shape, mode_name, gamma, 1)) % 2**32)
    x_np = rng.standard_normal(shape).astype(np.float32)
    dy_np = rng.standard_normal(shape).astype(np.float32)
    th = _theta(C, 11)
    b = (rng.standard_normal(C) * 0.1).astype(np.float32)
    x, w, y, mask, pm = _run_forward(rt, rt.ASR_MODE_EULER, x_np, th, b, C, gamma, h, dtype)
    dev = torch.device("cuda")
    dy = torch.from_numpy(dy_np).to(dev).to(rt.torch_dtype(dtype)).contiguous()
    dx, dth, db, dw = rt.conv_backward(mode, dy, x, mask if mode == rt.ASR_MODE_EULER else None, w, pm, h, gamma,
                                       want_dw=True)
    # oracle, fed the GPU's mask (the mask itself is checked in test_forward_parity)
    xo = bf16_round(x_np).astype(np.float64) if bf else x_np.astype(np.float64)
    dyo = bf16_round(dy_np).astype(np.float64) if bf else dy_np.astype(np.float64)
    Wo = _oracle_W(th, C, gamma, bf)
    if mode == rt.ASR_MODE_EULER:
        m = decode_mask(mask.cpu().numpy(), N, H, W_, C)
        dz_f = h * dyo * m
    else:
        dz_f = dyo
    dz_q = bf16_round(dz_f).astype(np.float64) if bf else dz_f
    dx_want = (dyo if mode == rt.ASR_MODE_EULER else 0.0) - O.conv2d_same(dz_q, Wo) + 2 * gamma * dz_q
    dW_want = O.conv2d_backprop_filter(xo, dz_q)
    db_want = dz_f.sum(axis=(0, 1, 2))
    src, sign = O.param_map(C)
    dth_want = O.project_dW(dW_want, src, sign, pm.n_theta)
    sc = np.abs(dx_want).max()
    if bf:
        assert_close(dx.float().cpu().numpy(), dx_want, rtol=2 ** -8, atol=4e-3 * sc, what="bf16 dx")
        tol = 1e-3
    else:
        assert_close(dx.cpu().numpy(), dx_want, rtol=1e-5, atol=2e-5 * sc, what="f32 dx")
        tol = 2e-5
    assert_close(dw.cpu().numpy(), dW_want, rtol=0, atol=tol * np.abs(dW_want).max(), what="dW")
    assert_close(dth.cpu().numpy(), dth_want, rtol=0, atol=tol * np.abs(dth_want).max(), what="dtheta")
    assert_close(db.cpu().numpy(), db_want, rtol=0, atol=2e-5 * max(np.abs(db_want).max(), 1), what="dbias")


def test_dgrad_identity_transpose(rt):
    """The kernel's dgrad (-A + 2 gamma I applied with the SAME W) equals the
    generic Conv2DBackpropInput of the oracle (no antisymmetry assumed)."""
    N, H, W_, C = 2, 32, 32, 16
    rng = np.random.default_rng(3)
    th = _theta(C, 3)
    x_np = rng.standard_normal((N, H, W_, C)).astype(np.float32)
    dz_np = rng.standard_normal((N, H, W_, C)).astype(np.float32)
    x, w, y, mask, pm = _run_forward(rt, rt.ASR_MODE_CONV, x_np, th, np.zeros(C, np.float32), C, -0.3, 1.0,
                                     rt.ASR_F32)
    dz = torch.from_numpy(dz_np).cuda()
    dx, *_ = rt.conv_backward(rt.ASR_MODE_CONV, dz, x, None, w, pm, 1.0, -0.3, want_dtheta=False, want_dbias=False)
    Wo = _oracle_W(th, C, -0.3, False)
    want = O.conv2d_backprop_input(dz_np.astype(np.float64), Wo, x_np.shape)
    assert_close(dx.cpu().numpy(), want, rtol=1e-5, atol=2e-5 * np.abs(want).max(), what="dgrad")


def test_adam_matches_tf1(rt):
    rng = np.random.default_rng(0)
    n = 1000
    p = rng.standard_normal(n).astype(np.float32)
    ps = [p.astype(np.float64).copy()]
    ms, vs = [np.zeros(n)], [np.zeros(n)]
    P = torch.from_numpy(p).cuda()
    M = torch.zeros(n, device="cuda")
    V = torch.zeros(n, device="cuda")
    for t in range(1, 4):
        g = rng.standard_normal(n).astype(np.float32)
        rt.adam_update(P, torch.from_numpy(g).cuda(), M, V, 1e-3, 0.9, 0.999, 1e-7, t, 1.0)
        O.adam_tf1(ps, [g.astype(np.float64)], ms, vs, t, 1e-3, 0.9, 0.999, 1e-7)
    assert_close(P.cpu().numpy(), ps[0], rtol=1e-6, atol=1e-7, what="adam")


@pytest.mark.parametrize("C", [16, 32, 64])
def test_backward_projection_in_epilogue(rt, C):
    """dtheta projected inside the backward kernel (slabs of n_theta + C)
    equals the projection of the separately reduced dW (slabs of 9C^2 + C)."""
    N, H, W_ = 3, 32, 32
    rng = np.random.default_rng(C)
    x_np = rng.standard_normal((N, H, W_, C)).astype(np.float32)
    dy = torch.from_numpy(rng.standard_normal((N, H, W_, C)).astype(np.float32)).cuda().to(torch.bfloat16)
    th = _theta(C, 2)
    b = (rng.standard_normal(C) * 0.1).astype(np.float32)
    x, w, y, mask, pm = _run_forward(rt, rt.ASR_MODE_EULER, x_np, th, b, C, -0.05, 0.5, rt.ASR_BF16)
    _, th_a, db_a, _ = rt.conv_backward(rt.ASR_MODE_EULER, dy, x, mask, w, pm, 0.5, -0.05)
    _, th_b, db_b, dw = rt.conv_backward(rt.ASR_MODE_EULER, dy, x, mask, w, pm, 0.5, -0.05, want_dw=True)
    a, bb = th_a.cpu().numpy(), th_b.cpu().numpy()
    assert np.abs(a - bb).max() <= 1e-5 * np.abs(bb).max()
    np.testing.assert_allclose(db_a.cpu().numpy(), db_b.cpu().numpy(), rtol=0, atol=1e-6)


@pytest.mark.parametrize("k", [5, 7])
@pytest.mark.parametrize("anti,gamma", [(True, 0.0), (True, -0.1), (False, 0.0)])
def test_general_k_layer_matches_oracle(rt, k, anti, gamma):
    """Conv2DAntisymmetric(kernel_size=k) on a device tensor (fp32 k x k kernels:
    asr_theta_to_w_k, asr_conv_forward_k, asr_conv_backward_k through the
    layer's autograd) against the literal restatement of the reference's
    assembly (oracle.assemble_general_literal, …Conv2DAntisymmetric.py:109-145)
    and fp64 conv / autodiff: y, dx, dtheta, dbias (fp32 tolerances)."""
    from differential_equations_resnet_amd.layers import Conv2DAntisymmetric
    C, N, H, W_ = 8, 2, 11, 13
    layer = Conv2DAntisymmetric(k, gamma=gamma, antisymmetric=anti, name=f"ca{k}")
    layer.build((None, H, W_, C))
    rng = np.random.default_rng(k * 10 + int(anti))
    for v in layer.theta_vars:
        v.assign((rng.standard_normal(v.shape) * 0.2).astype(np.float32))
    layer.bias.assign((rng.standard_normal(C) * 0.1).astype(np.float32))
    theta_list = [v.value.astype(np.float64) for v in layer.theta_vars]
    Wl = O.assemble_general_literal(theta_list, C, k, gamma, anti)
    np.testing.assert_array_equal(layer.get_kernel(), Wl.astype(np.float32))
    x_np = rng.standard_normal((N, H, W_, C)).astype(np.float32)
    dy_np = rng.standard_normal((N, H, W_, C)).astype(np.float32)
    x = torch.from_numpy(x_np).cuda().requires_grad_(True)
    y = layer.call_device(x)
    y.backward(torch.from_numpy(dy_np).cuda())
    th, b = layer.device_variables(x.device)
    b_np = layer.bias.value.astype(np.float64)
    y_want = O.conv2d_same(x_np.astype(np.float64), Wl) + b_np
    assert_close(y.detach().cpu().numpy(), y_want, rtol=1e-5, atol=2e-5 * np.abs(y_want).max(), what="y")
    dx_want = O.conv2d_backprop_input(dy_np.astype(np.float64), Wl, x_np.shape)
    assert_close(x.grad.cpu().numpy(), dx_want, rtol=1e-5, atol=2e-5 * np.abs(dx_want).max(), what="dx")
    src, sign = O.param_map(C, "general", k, anti)
    dth_want = O.project_dW(O.conv2d_backprop_filter(x_np.astype(np.float64), dy_np.astype(np.float64), k), src, sign,
                            th.numel())
    assert np.abs(th.grad.cpu().numpy() - dth_want).max() <= 1e-4 * np.abs(dth_want).max()
    db_want = dy_np.astype(np.float64).sum(axis=(0, 1, 2))
    assert np.abs(b.grad.cpu().numpy() - db_want).max() <= 1e-4 * np.abs(db_want).max()
