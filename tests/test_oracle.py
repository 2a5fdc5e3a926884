"""CPU tests of the oracle against the reference's own evidence (notebook
known-answer values and structural invariants), plus internal consistency
(closed form vs literal assembly, finite differences, second restatement).

The reference has no test suite; these fixtures are transcribed
from its notebooks' printed outputs (tests/golden/kat_*.json)."""
import json
import os

import numpy as np
import pytest

from oracle import asr_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_kat_conv2d_same_is_cross_correlation():
    """antisymmetric_conv_kernel.ipynb cells 1-3: tf.nn.conv2d(SAME, NHWC) of a
    printed 7x7 image with a printed 3x3 kernel (values printed to ~7 digits)."""
    k = _load("kat_conv7x7.json")
    x = np.array(k["image_hw"], np.float64)[None, :, :, None]
    W = np.array(k["kernel_hw"], np.float64)[:, :, None, None]
    want = np.array(k["conv2d_same_hw"])
    got = O.conv2d_same(x, W)[0, :, :, 0]
    assert np.abs(got - want).max() < 1e-6
    # a flipped (true) convolution does NOT match: pins cross-correlation
    flipped = O.conv2d_same(x, W[::-1, ::-1])[0, :, :, 0]
    assert np.abs(flipped - want).max() > 0.1


def test_kat_trained_kernel_structure():
    """experiments_antisymmetric_resnet_v6.ipynb cell 26: W[:,:,31,10] =
    -rot180(W[:,:,10,31]) and the diagonal block is anti-centrosymmetric with
    centre gamma = 0 — exactly the structure the oracle's assembly produces."""
    k = _load("kat_kernel_structure_v6.json")
    a = np.array(k["W_10_31"])
    b = np.array(k["W_31_10"])
    d = np.array(k["W_4_4"])
    assert np.array_equal(b, -a[::-1, ::-1])
    assert np.array_equal(d, -d[::-1, ::-1]) and d[1, 1] == 0.0
    # the oracle assembly has the same relations for every (i, o) pair
    rng = np.random.default_rng(0)
    C = 12
    W = O.assemble_3by3_literal(O.init_theta_3by3(C, rng), 0.0)
    for i in range(C):
        for o in range(C):
            assert np.array_equal(W[:, :, o, i], -W[::-1, ::-1, i, o])


def test_kat_prototype_offdiagonal_relation():
    """v6 cell 41 (numpy prototype, C=512): off-diagonal blocks are negated
    rot180 transposes of each other."""
    k = _load("kat_kernel_structure_v6_proto.json")
    for a, b in [("W_1_0", "W_0_1"), ("W_14_234", "W_234_14")]:
        assert np.array_equal(np.array(k[b]), -np.array(k[a])[::-1, ::-1])


@pytest.mark.parametrize("C", [1, 2, 3, 7, 16])
@pytest.mark.parametrize("gamma", [0.0, -0.25])
def test_assembly_closed_form_and_operator_antisymmetry(C, gamma):
    rng = np.random.default_rng(C)
    th = O.init_theta_3by3(C, rng)
    Wl = O.assemble_3by3_literal(th, gamma)
    src, sign = O.param_map(C)
    Wm = O.assemble_from_map(O.flatten(th), C, src, sign, gamma)
    assert np.array_equal(Wl, Wm)
    # conv operator A satisfies A + A^T = 2 gamma I (zero padding, stride 1)
    N, H, Wd = 1, 5, 4
    n = H * Wd * C
    A = np.zeros((n, n))
    for j in range(n):
        e = np.zeros(n)
        e[j] = 1.0
        A[:, j] = O.conv2d_same(e.reshape(N, H, Wd, C), Wl).ravel()
    assert np.abs(A + A.T - 2 * gamma * np.eye(n)).max() < 1e-12


@pytest.mark.parametrize("C,anti", [(3, True), (5, True), (4, False)])
def test_general_layer_assembly(C, anti):
    rng = np.random.default_rng(C)
    shapes, names = O.theta_shapes_general(C, 3, anti)
    th = [rng.standard_normal(s) for s in shapes]
    Wl = O.assemble_general_literal(th, C, 3, 0.2, anti)
    src, sign = O.param_map(C, "general", 3, anti)
    assert np.array_equal(Wl, O.assemble_from_map(O.flatten(th), C, src, sign, 0.2))
    assert names[0] == "centro_sym_0_0"


def _fd(f, v, eps=1e-6):
    g = np.zeros_like(v)
    for i in range(v.size):
        e = np.zeros_like(v)
        e.flat[i] = eps
        g.flat[i] = (f(v + e) - f(v - e)) / (2 * eps)
    return g


def test_euler_block_gradients_finite_difference():
    rng = np.random.default_rng(1)
    C, N, H, Wd, h, g = 3, 2, 4, 5, 0.3, -0.1
    th = O.flatten(O.init_theta_3by3(C, rng))
    b = rng.standard_normal(C) * 0.1
    src, sign = O.param_map(C)
    x = rng.standard_normal((N, H, Wd, C))
    R = rng.standard_normal((N, H, Wd, C))

    def f(t, bb, xx):
        y, _ = O.euler_fwd(xx, O.assemble_from_map(t, C, src, sign, g), bb, h)
        return (y * R).sum()

    W = O.assemble_from_map(th, C, src, sign, g)
    y, z = O.euler_fwd(x, W, b, h)
    dx, dW, db = O.euler_bwd(R, x, z, W, h, g)
    dth = O.project_dW(dW, src, sign, th.size)
    assert np.abs(_fd(lambda t: f(t, b, x), th) - dth).max() < 1e-6
    assert np.abs(_fd(lambda v: f(th, v, x), b) - db).max() < 1e-6
    assert np.abs(_fd(lambda v: f(th, b, v), x) - dx).max() < 1e-6
    # dgrad with the same W (A^T = -A + 2 gamma I) == generic transpose conv
    dz = h * R * (z > 0)
    assert np.abs(dx - (R + O.conv2d_backprop_input(dz, W, x.shape))).max() < 1e-12


@pytest.mark.parametrize("kind,anti", [("3by3", True), ("regular", False)])
def test_rk2_block_gradients_finite_difference(kind, anti):
    """RK2 midpoint block (extension, BASELINE config 5): analytic backward vs
    finite differences, for the antisymmetric (A^T = -A + 2 gamma I) and the
    generic transpose path."""
    rng = np.random.default_rng(5)
    C, N, H, Wd, h = 3, 2, 4, 5, 0.7
    g = -0.1 if anti else 0.0
    if kind == "3by3":
        th = O.flatten(O.init_theta_3by3(C, rng))
        src, sign = O.param_map(C)
    else:
        th = rng.standard_normal(9 * C * C) * 0.3
        src, sign = np.arange(9 * C * C), np.ones(9 * C * C, dtype=np.int64)
    b = rng.standard_normal(C) * 0.1
    x = rng.standard_normal((N, H, Wd, C))
    R = rng.standard_normal((N, H, Wd, C))

    def f(t, bb, xx):
        y, _ = O.rk2_fwd(xx, O.assemble_from_map(t, C, src, sign, g), bb, h)
        return (y * R).sum()

    W = O.assemble_from_map(th, C, src, sign, g)
    y, cache = O.rk2_fwd(x, W, b, h)
    dx, dW, db = O.rk2_bwd(R, x, cache, W, h, g, anti)
    dth = O.project_dW(dW, src, sign, th.size)
    assert np.abs(_fd(lambda t: f(t, b, x), th) - dth).max() < 1e-6
    assert np.abs(_fd(lambda v: f(th, v, x), b) - db).max() < 1e-6
    assert np.abs(_fd(lambda v: f(th, b, v), x) - dx).max() < 1e-6
    # the midpoint step is the composition of two Euler-block evaluations
    xm, _ = O.euler_fwd(x, W, b, 0.5 * h)
    assert np.abs(cache[0] - xm).max() < 1e-14


def test_rk2_network_gradients_finite_difference():
    rng = np.random.default_rng(6)
    spec = O.NetSpec(C=4, L=2, h=0.5, H=5, W=4, gamma=-0.1, integrator="rk2")
    params = O.init_params(spec, rng, bias_std=0.1)
    imgs = rng.integers(0, 256, (3, 5, 4, 3)).astype(np.uint8)
    oh = np.eye(10)[rng.integers(0, 10, 3)]
    probs, cache = O.net_forward(spec, params, imgs)
    g = O.flatten(O.net_backward(spec, params, cache, oh))
    flat = O.flatten(params)
    shapes = [p.shape for p in params]

    def loss(fl):
        pr, _ = O.net_forward(spec, O.unflatten(fl, shapes), imgs)
        return O.net_loss(pr, oh)

    for i in rng.choice(flat.size, 25, replace=False):
        e = np.zeros_like(flat)
        e[i] = 1e-6
        assert abs((loss(flat + e) - loss(flat - e)) / 2e-6 - g[i]) < 1e-6


@pytest.mark.parametrize("kind,anti", [("3by3", True), ("general", True), ("general", False), ("regular", False)])
def test_network_gradients_finite_difference(kind, anti):
    rng = np.random.default_rng(2)
    spec = O.NetSpec(C=4, L=2, h=0.5, H=5, W=4, gamma=-0.1 if anti else 0.0, kind=kind, antisymmetric=anti)
    params = O.init_params(spec, rng, bias_std=0.1)
    imgs = rng.integers(0, 256, (3, 5, 4, 3)).astype(np.uint8)
    oh = np.eye(10)[rng.integers(0, 10, 3)]
    probs, cache = O.net_forward(spec, params, imgs)
    g = O.flatten(O.net_backward(spec, params, cache, oh))
    flat = O.flatten(params)
    shapes = [p.shape for p in params]

    def loss(fl):
        pr, _ = O.net_forward(spec, O.unflatten(fl, shapes), imgs)
        return O.net_loss(pr, oh)

    for i in rng.choice(flat.size, 25, replace=False):
        e = np.zeros_like(flat)
        e[i] = 1e-6
        assert abs((loss(flat + e) - loss(flat - e)) / 2e-6 - g[i]) < 1e-6


def test_keras_cce_clip_gradient():
    """Saturated probabilities: the clip kills the gradient of the clipped
    entries exactly as TF's clip_by_value gradient does."""
    probs = np.array([[1.0 - 1e-9, 1e-9, 0.0]])
    onehot = np.array([[0.0, 1.0, 0.0]])
    loss = O.keras_cce(probs, onehot)
    assert np.isclose(loss[0], -np.log(1e-7))
    gl = O.keras_cce_grad_logits(probs, onehot, 1.0)
    assert np.all(np.isfinite(gl))


def test_adam_tf1_first_step():
    p = [np.array([1.0, -2.0])]
    g = [np.array([0.5, -0.25])]
    m = [np.zeros(2)]
    v = [np.zeros(2)]
    O.adam_tf1(p, g, m, v, 1, lr=0.1, eps=1e-7)
    # first step: m_hat/sqrt(v_hat) = sign(g)  ->  p -= lr * sign(g) (up to eps)
    assert np.allclose(p[0], [0.9, -1.9], atol=1e-6)


def test_torch_cpu_restatement_matches_numpy_oracle():
    torch = pytest.importorskip("torch")
    from oracle.torch_cpu_ref import RefNet
    rng = np.random.default_rng(3)
    spec = O.NetSpec(C=6, L=2, h=0.25, H=6, W=5)
    params = O.init_params(spec, rng, bias_std=0.1)
    imgs = rng.integers(0, 256, (3, 6, 5, 3)).astype(np.uint8)
    oh = np.eye(10)[rng.integers(0, 10, 3)]
    net = RefNet(params, 6, 2, 0.25)
    p_t = net.forward(imgs)
    probs, cache = O.net_forward(spec, params, imgs)
    assert np.abs(p_t.detach().numpy() - probs).max() < 1e-6
    loss = RefNet.keras_cce(p_t, torch.tensor(oh, dtype=torch.float32)).mean()
    loss.backward()
    g = O.net_backward(spec, params, cache, oh)
    for a, b in zip(net.params, g):
        assert np.abs(a.grad.numpy() - b).max() <= 1e-4 * max(np.abs(b).max(), 1e-6)


@pytest.mark.parametrize("H,W,S", [(6, 7, 2), (7, 7, 2), (5, 6, 1)])
def test_transition_oracle_finite_differences(H, W, S):
    """single_layer_conv_block's restatement (TF 'same' stride padding, 1x1
    'valid' shortcut) against central differences of its own forward."""
    rng = np.random.default_rng(H * 10 + S)
    x = rng.standard_normal((2, H, W, 3))
    K2, b2 = rng.standard_normal((3, 3, 3, 4)), rng.standard_normal(4) * 0.1
    K1, b1 = rng.standard_normal((1, 1, 3, 4)), rng.standard_normal(4)
    y, z = O.transition_fwd(x, K2, b2, K1, b1, S)
    assert y.shape == (2, -(-H // S), -(-W // S), 4)
    dy = rng.standard_normal(y.shape)
    dx, g = O.transition_bwd(dy, x, z, K2, K1, S)
    args = [x, K2, b2, K1, b1]
    grads = [dx] + g

    def f(a):
        return (O.transition_fwd(*a, S)[0] * dy).sum()
    for k in range(5):
        for _ in range(4):
            j = tuple(rng.integers(0, s) for s in args[k].shape)
            a = [v.copy() for v in args]
            a[k][j] += 1e-6
            fp = f(a)
            a[k][j] -= 2e-6
            fm = f(a)
            assert abs((fp - fm) / 2e-6 - grads[k][j]) < 1e-6 * max(1.0, abs(grads[k][j]))


def test_transition_oracle_same_padding_is_tf_asymmetric():
    """TF 'SAME' at stride 2 on an even input pads only bottom/right: output
    (0, 0) of a 3x3 reads input rows/cols 0..2, not -1..1."""
    x = np.zeros((1, 4, 4, 1))
    x[0, 0, 0, 0] = 1.0
    K2 = np.zeros((3, 3, 1, 1))
    K2[0, 0, 0, 0] = 1.0  # top-left tap
    y, _ = O.transition_fwd(x, K2, np.zeros(1), np.zeros((1, 1, 1, 1)), np.zeros(1), 2)
    assert y[0, 0, 0, 0] == 1.0


def test_stages_oracle_finite_differences():
    rng = np.random.default_rng(1)
    sp = O.StagesSpec(stages=[(4, 1, 0), (8, 2, 2), (8, 1, 0)], H=6, W=7, num_classes=5, h=0.7, gamma=0.1)
    P = O.stages_init_params(sp, rng, bias_std=0.1)
    imgs = rng.integers(0, 256, (3, 6, 7, 3)).astype(np.float64)
    oh = np.eye(5)[rng.integers(0, 5, 3)]
    pr, c = O.stages_forward(sp, P, imgs)
    g = O.stages_backward(sp, P, c, oh)
    assert [x.shape for x in g] == [tuple(s) for s in sp.param_shapes()]
    for k in range(len(P)):
        for _ in range(2):
            j = tuple(rng.integers(0, s) for s in P[k].shape)
            a = [v.copy() for v in P]
            a[k][j] += 1e-6
            fp = O.net_loss(O.stages_forward(sp, a, imgs)[0], oh)
            a[k][j] -= 2e-6
            fm = O.net_loss(O.stages_forward(sp, a, imgs)[0], oh)
            assert abs((fp - fm) / 2e-6 - g[k][j]) < 1e-7 + 1e-4 * abs(g[k][j])
