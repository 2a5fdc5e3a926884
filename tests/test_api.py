"""CPU tests of the drop-in host API: builders, layers (weights, names,
config, readback), lowering analysis, weight files, dataset pipeline.
Nothing here launches a kernel."""
import os
import pickle

import numpy as np
import pytest

from oracle import asr_oracle as O

from differential_equations_resnet_amd import _lib, graph
from differential_equations_resnet_amd.graph import Input
from differential_equations_resnet_amd.layers import Conv2DAntisymmetric, Conv2DAntisymmetric3By3
from differential_equations_resnet_amd.lowering import analyze
from differential_equations_resnet_amd.models import tfkeras_resnets as R


def _single_block(C=16, L=3, h=0.5, gamma=0.0, kernel_type="antisymmetric", **kw):
    fn = R.get_single_block_resnet_build_function(kernel_type=kernel_type, h=h, gamma=gamma, num_stages=2,
                                                  blocks_per_stage=[L], filters_per_block=[C], strides=[(1, 1)],
                                                  subtract_mean=127.5, divide_by_stddev=127.5, num_classes=10, **kw)
    return fn(Input(shape=(32, 32, 3)))


def test_builder_names_and_weight_layout_match_reference():
    graph.set_seed(0)
    m = _single_block(C=16, L=3)
    names = [l.name for l in m.layers]
    for n in ["identity_layer", "input_mean_shift", "input_scaling", "conv1", "res2_0_branch2", "scale2_0",
              "res2_2_branch2", "global_average_pooling", "fc"]:
        assert n in names
    assert m.name == "single_block_resnet_antisymmetric"
    assert isinstance(m.get_layer("res2_1_branch2"), Conv2DAntisymmetric3By3)
    shapes = [tuple(w.shape) for w in m.get_weights()]
    assert shapes == [tuple(s) for s in O.NetSpec(C=16, L=3).param_shapes()]
    lay = m.get_layer("res2_0_branch2")
    wn = [w.name.split("/")[-1] for w in lay.weights]
    assert wn[:5] == ["a", "b", "c", "d", "input_kernels_for_output_kernel_0"] and wn[-1] == "bias"
    assert m.count_params() == O.NetSpec(C=16, L=3).n_params()


def test_h_one_has_no_scale_lambda_and_errors():
    m = _single_block(h=1.0, L=2)
    assert not any(l.name.startswith("scale2_") for l in m.layers)
    with pytest.raises(ValueError):
        R.get_single_block_resnet_build_function(num_classes=None)
    with pytest.raises(ValueError):
        R.get_resnet_build_function(preset="resnet18", num_classes=10)
    with pytest.raises(ValueError):
        R.bottleneck_conv_block(Input(shape=(8, 8, 4)), 3, [4, None, 4], True, False, 2, 0, version=2)


def test_layer_config_and_shapes():
    layer = Conv2DAntisymmetric3By3(gamma=-0.1, name="x")
    y = layer(Input(shape=(8, 8, 5)))
    assert y.shape == (None, 8, 8, 5)
    c = layer.get_config()
    assert "gamma" not in c and c["use_bias"] and c["strides"] == (1, 1)
    assert layer.compute_output_shape((None, 8, 8, 5)) == (None, 8, 8, 5)
    g = Conv2DAntisymmetric(3, antisymmetric=False, name="g")
    g(Input(shape=(8, 8, 4)))
    assert g.get_config()["kernel_size"] == 3 and g.get_config()["antisymmetric"] is False
    shapes, names = O.theta_shapes_general(4, 3, False)
    assert [w.shape for w in g.weights[:-1]] == [tuple(s) for s in shapes]
    assert [w.name.split("/")[-1] for w in g.weights[:-1]] == names
    nb = Conv2DAntisymmetric3By3(use_bias=False)
    nb(Input(shape=(4, 4, 3)))
    with pytest.raises(ValueError):
        nb.get_bias()


def test_antisymmetric_initializer_stddev():
    graph.set_seed(1)
    layer = Conv2DAntisymmetric3By3()
    layer(Input(shape=(8, 8, 64)))
    th = layer.theta_flat()
    std = np.sqrt(2 / (9 * 64))
    assert np.abs(th).max() <= 2 * std + 1e-7           # 2-sigma truncation
    assert abs(th.std() / std - 0.8796) < 0.02           # std of a 2-sigma truncated normal


@pytest.mark.parametrize("C,gamma", [(3, 0.0), (7, -0.2)])
def test_get_kernel_matches_literal_assembly(C, gamma):
    layer = Conv2DAntisymmetric3By3(gamma=gamma)
    layer(Input(shape=(4, 4, C)))
    th = [w.value.astype(np.float64) for w in layer.weights[:-1]]
    want = O.assemble_3by3_literal(th, gamma)
    np.testing.assert_array_equal(layer.get_kernel(), want.astype(np.float32))


@pytest.mark.parametrize("anti", [True, False])
def test_general_get_kernel_matches_literal_assembly(anti):
    layer = Conv2DAntisymmetric(3, gamma=0.3, antisymmetric=anti)
    layer(Input(shape=(4, 4, 5)))
    th = [w.value.astype(np.float64) for w in layer.weights[:-1]]
    want = O.assemble_general_literal(th, 5, 3, 0.3, anti)
    np.testing.assert_array_equal(layer.get_kernel(), want.astype(np.float32))


def test_analyze_single_block_plan():
    m = _single_block(C=16, L=4, h=0.25, gamma=-0.05)
    p = analyze(m)
    assert (p.C, p.L, p.H, p.W, p.Cin, p.num_classes) == (16, 4, 32, 32, 3, 10)
    assert p.h == 0.25 and p.gamma == pytest.approx(-0.05) and p.param_kind == _lib.ASR_PARAM_3BY3
    assert p.subtract_mean == pytest.approx(127.5) and p.divide_by_stddev == pytest.approx(127.5)
    assert [v.name for v in p.weight_vars()] == [w.name for w in m.weights]
    r = analyze(_single_block(C=8, L=2, h=1.0, kernel_type="regular"))
    assert r.param_kind == _lib.ASR_PARAM_REGULAR and r.h == 1.0 and r.L == 2


@pytest.mark.parametrize("kernel_type,h", [("antisymmetric", 0.5), ("regular", 2.0)])
def test_rk2_builder_and_lowering(kernel_type, h):
    """integrator='rk2' (extension, BASELINE config 5): the same conv layer is
    applied twice per block (shared weights), so the weight list, names and
    parameter count are those of the Euler model; the lowering recognises the
    midpoint pattern."""
    m = _single_block(C=8, L=3, h=h, kernel_type=kernel_type, integrator="rk2")
    e = _single_block(C=8, L=3, h=h, kernel_type=kernel_type)
    assert [w.shape for w in m.weights] == [w.shape for w in e.weights]
    assert len(m.get_layer("res2_1_branch2").inbound_nodes) == 2
    names = [l.name for l in m.layers]
    assert ("scale2_0_half" in names) == (h != 2.0) and "scale2_0" in names
    p = analyze(m)
    assert p.integrator == "rk2" and p.L == 3 and p.h == h
    assert analyze(e).integrator == "euler"
    with pytest.raises(ValueError):
        _single_block(L=1, integrator="rk4")


def test_analyze_rejects_mixed_integrators():
    x = Input(shape=(32, 32, 3))
    y = graph.Conv2D(8, 3, padding="same", activation="relu", name="conv1")(x)
    y = R.single_layer_identity_block(y, 3, True, False, 2, 0, h=0.5)
    y = R.single_layer_identity_block(y, 3, True, False, 2, 1, h=0.5, integrator="rk2")
    y = graph.Dense(10, activation="softmax")(graph.GlobalAveragePooling2D()(y))
    with pytest.raises(_lib.AsrUnsupported, match="integrator"):
        analyze(graph.Model(x, y))


def test_analyze_general_layer_model():
    x = Input(shape=(32, 32, 3))
    y = graph.Conv2D(8, 3, padding="same", activation="relu", name="conv1")(x)
    for b in range(2):
        z = Conv2DAntisymmetric(3, gamma=0.1, antisymmetric=False, name=f"blk{b}")(y)
        z = graph.Activation("relu")(z)
        y = graph.add([z, y])
    y = graph.GlobalAveragePooling2D()(y)
    y = graph.Dense(10, activation="softmax")(y)
    p = analyze(graph.Model(x, y))
    assert p.param_kind == _lib.ASR_PARAM_GENERAL and not p.antisymmetric and p.L == 2 and p.h == 1.0
    assert p.subtract_mean is None


@pytest.mark.parametrize("kw", [dict(use_batch_norm=True), dict(use_max_pooling=[True])])
def test_analyze_rejects_unsupported(kw):
    with pytest.raises(_lib.AsrUnsupported):
        analyze(_single_block(L=2, **kw))


def test_analyze_multistage_plan():
    """num_stages > 2 (tfkeras_resnets.py:575-593): the He-style ResNet-32 lowers
    onto the multi-stage executor; its flat parameter order is the model's
    weight order and the C ABI's count (host function, no launch)."""
    import ctypes as ct
    from differential_equations_resnet_amd.lowering import StagesPlan
    from differential_equations_resnet_amd.runtime import StagesConfig
    fn = R.get_single_block_resnet_build_function(num_stages=4, blocks_per_stage=[10, 10, 10], h=0.5,
                                                  filters_per_block=[16, 32, 64], strides=[(1, 1), (2, 2), (2, 2)],
                                                  num_classes=10, subtract_mean=127.5, divide_by_stddev=127.5)
    m = fn(Input(shape=(32, 32, 3)))
    p = analyze(m)
    assert isinstance(p, StagesPlan) and p.stages == [(16, 10, 0), (32, 9, 2), (64, 9, 2)] and p.L == 28
    assert [t is None for t in p.transitions] == [True, False, False]
    assert p.transitions[1][0].name == "res3_0_branch2" and p.transitions[1][1].name == "res3_0_branch1"
    assert [v.name for v in p.weight_vars()] == [w.name for w in m.weights]
    spec = O.StagesSpec(stages=p.stages, h=0.5)
    assert [tuple(v.shape) for v in p.weight_vars()] == [tuple(s) for s in spec.param_shapes()]
    assert m.count_params() == spec.n_params()
    c = StagesConfig()
    c.N, c.H, c.W, c.Cin, c.num_classes, c.n_stages = 8, 32, 32, 3, 10, 3
    for i, (C, L, S) in enumerate(p.stages):
        c.C[i], c.L[i], c.stride[i] = C, L, S
    c.h, c.divide_by_stddev = 0.5, 1.0
    lib = _lib.load()
    assert lib.asr_stages_param_count(ct.byref(c)) == spec.n_params()
    assert lib.asr_stages_workspace_bytes(ct.byref(c)) > 0
    assert lib.asr_stages_check(ct.byref(c)) == _lib.ASR_OK
    c.dtype = _lib.ASR_BF16  # bf16: every stage with blocks on C {16,32,64} x W {32,16,8}
    assert lib.asr_stages_check(ct.byref(c)) == _lib.ASR_OK
    assert lib.asr_stages_param_count(ct.byref(c)) == spec.n_params()
    bf_ws = lib.asr_stages_workspace_bytes(ct.byref(c))
    c.dtype = _lib.ASR_F32
    assert 0 < bf_ws < lib.asr_stages_workspace_bytes(ct.byref(c))  # bf16 activations: a smaller workspace
    c.dtype = 7
    assert lib.asr_stages_check(ct.byref(c)) == _lib.ASR_E_ARG
    c.dtype, c.W = _lib.ASR_BF16, 16  # the last stage at W = 4
    assert lib.asr_stages_check(ct.byref(c)) == _lib.ASR_E_UNSUPPORTED and b"W=4" in lib.asr_last_error()
    c.dtype, c.W = _lib.ASR_F32, 32
    c.stride[0] = 2
    assert lib.asr_stages_check(ct.byref(c)) == _lib.ASR_E_ARG
    assert lib.asr_stages_param_count(ct.byref(c)) == -1
    # RK2 identity blocks are single-stage only
    fn = R.get_single_block_resnet_build_function(num_stages=3, blocks_per_stage=[2, 2], filters_per_block=[8, 16],
                                                  strides=[(1, 1), (2, 2)], num_classes=10, integrator="rk2")
    with pytest.raises(_lib.AsrUnsupported, match="rk2"):
        analyze(fn(Input(shape=(32, 32, 3))))


def test_analyze_rejects_per_channel_mean():
    fn = R.get_single_block_resnet_build_function(num_stages=2, blocks_per_stage=[2], filters_per_block=[8],
                                                  strides=[(1, 1)], num_classes=10, subtract_mean=[120, 115, 100])
    with pytest.raises(_lib.AsrUnsupported, match="per-channel"):
        analyze(fn(Input(shape=(32, 32, 3))))


def test_resnet50_graph_builds():
    m = R.build_resnet((64, 64, 3), num_classes=10, preset="resnet50")
    assert m.name == "resnet50_antisymmetric"
    assert m.get_layer("res2_0_branch2b") is not None
    with pytest.raises(_lib.AsrUnsupported):
        analyze(m)


def test_weight_files_round_trip(tmp_path):
    from differential_equations_resnet_amd.model_utils import double_load_weights, save_model_weights
    graph.set_seed(3)
    m = _single_block(C=8, L=2)
    p = tmp_path / "w.npz"
    m.save_weights(str(p))
    m2 = _single_block(C=8, L=2)
    m2.load_weights(str(p))
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)
    # depth doubling: 2 blocks -> 4 blocks, each saved block loaded twice
    q = tmp_path / "layers.npz"
    save_model_weights(m, str(q))
    m4 = _single_block(C=8, L=4)
    double_load_weights(m4, str(q))
    src = m.get_layer("res2_1_branch2").get_weights()
    for b in (2, 3):
        for a, c in zip(m4.get_layer(f"res2_{b}_branch2").get_weights(), src):
            np.testing.assert_array_equal(a, c)
    np.testing.assert_array_equal(m4.get_layer("fc").get_weights()[0], m.get_layer("fc").get_weights()[0])


def test_cifar10_loaders(tmp_path):
    from differential_equations_resnet_amd.dataset_utils import build_cifar10_dataset
    rng = np.random.default_rng(0)
    # binary distribution
    d = tmp_path / "bin"
    d.mkdir()
    recs = {}
    for f, n in [(f"data_batch_{i}", 10000) for i in range(1, 6)] + [("test_batch", 10000)]:
        r = rng.integers(0, 256, (n, 3073), dtype=np.uint8)
        r[:, 0] %= 10
        r.tofile(d / (f + ".bin"))
        recs[f] = r
    (d / "batches.meta.txt").write_text("airplane\nautomobile\n")
    xtr, ytr, xte, yte, names = build_cifar10_dataset(str(d))
    assert xtr.shape == (50000, 32, 32, 3) and xtr.dtype == np.uint8 and names[:2] == ["airplane", "automobile"]
    r1 = recs["data_batch_1"]
    np.testing.assert_array_equal(xtr[5], r1[5, 1:].reshape(3, 32, 32).transpose(1, 2, 0))
    assert ytr[5] == r1[5, 0] and yte.shape == (10000,)
    # python distribution (data-only unpickling), and a hostile file is refused
    d = tmp_path / "py"
    d.mkdir()
    for f in [f"data_batch_{i}" for i in range(1, 6)] + ["test_batch"]:
        with open(d / f, "wb") as fh:
            pickle.dump({b"data": rng.integers(0, 256, (10000, 3072), dtype=np.uint8),
                         b"labels": list(rng.integers(0, 10, 10000))}, fh)
    with open(d / "batches.meta", "wb") as fh:
        pickle.dump({b"label_names": [b"cat", b"dog"]}, fh)
    xtr, ytr, xte, yte, names = build_cifar10_dataset(str(d))
    assert xtr.shape == (50000, 32, 32, 3) and names == ["cat", "dog"]

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    with open(d / "test_batch", "wb") as fh:
        pickle.dump({b"data": Evil()}, fh)
    with pytest.raises(pickle.UnpicklingError):
        build_cifar10_dataset(str(d))


def test_array_dataset_stream_and_sharding():
    torch = pytest.importorskip("torch")
    from differential_equations_resnet_amd.dataset_utils import ArrayDataset
    n, B = 10, 4
    feats = np.arange(n, dtype=np.uint8).reshape(n, 1, 1, 1)
    labels = np.arange(n) % 3
    ds = ArrayDataset(feats, labels, B, seed=5, device=torch.device("cpu"))
    it = iter(ds)
    seen = [next(it)[0].flatten().tolist() for _ in range(5)]  # 20 images = 2 epochs
    flat = sum(seen, [])
    assert sorted(flat[:10]) == list(range(10)) and sorted(flat[10:20]) == list(range(10))
    x, y = next(iter(ds))
    assert y.shape == (B, 3) and float(y.sum()) == B
    # two ranks partition each global batch
    r0 = next(iter(ArrayDataset(feats, labels, 2, seed=9, rank=0, world_size=2, device=torch.device("cpu"))))[0]
    r1 = next(iter(ArrayDataset(feats, labels, 2, seed=9, rank=1, world_size=2, device=torch.device("cpu"))))[0]
    both = ArrayDataset(feats, labels, 4, seed=9, device=torch.device("cpu"))
    assert r0.flatten().tolist() + r1.flatten().tolist() == next(iter(both))[0].flatten().tolist()
