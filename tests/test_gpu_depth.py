"""The bench's own compositions at their own depth against the PLAIN fp64
oracle (oracle.net_forward / net_backward: the reference's network,
tfkeras_resnets.py:547-597, differentiated end to end as training.py:300
does), at small batches the oracle finishes in seconds:

  * C2 (BASELINE configs[1]): C=64, L=30 Euler blocks, h=8/30, bf16
    activations with fp32 accumulation — N=8 and N=16;
  * C5 (configs[4]): the same with RK2 (midpoint) blocks;
  * C3 (configs[2]): C=16, L=108, h=8/108 — the fused 108-block stack, N=4.

The executor runs its production kernel set (variant 0: the stacked
k_fwd3_stack / k_bwd3_stack at C=64, the fused deep16 stack at C=16), so
the bf16 error accumulated over all L blocks is measured against the
reference's math, not against a model of the executor's roundings.

Bars (the bf16 network bar), each stated where it is asserted:
  * loss within 1 % relative; probabilities within 2e-2 absolute;
  * relative L2 <= 2e-2 per gradient group (conv1 kernel / bias, each
    block's merged theta / bias, fc kernel / bias: the per-layer groups of
    the reference's gradient norms, training.py:385-409);
  * per tensor: max |err| <= TENSOR_TOL x the group's max |ref|, so that a
    zeroed channel (a handful of scalars among thousands, invisible to a
    group's relative L2) fails — see helpers.assert_grad_tensors_max.

Two initialisations: the bench's (bench.py: the reference init with the
block thetas x0.5 and the fc kernel x0.1, zero biases) and the reference
init with small random biases (the headline test's).
"""
import numpy as np
import pytest

from helpers import assert_grad_tensors_max, grad_groups, rel_l2
from oracle import asr_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GROUP_TOL = 2e-2
TENSOR_TOL = 1e-2   # per tensor, of the group's max |ref| (see helpers.assert_grad_tensors_max; measured <= 7.9e-3)


def _params(spec, init, seed):
    rng = np.random.default_rng(seed)
    if init == "bench":
        from differential_equations_resnet_amd.netparams import init_net_params
        flat = init_net_params(spec.C, spec.L, 3, 10, seed=seed).astype(np.float64)
        ps = O.unflatten(flat, spec.param_shapes())
        nt = len(spec.theta_shapes())
        for b in range(spec.L):
            for j in range(nt):
                ps[2 + b * (nt + 1) + j] = ps[2 + b * (nt + 1) + j] * 0.5
        ps[-2] = ps[-2] * 0.1
    else:
        ps = O.init_params(spec, rng, np.float64, bias_std=0.05)
        ps[-2] = ps[-2] * 0.1
    return [p.astype(np.float32).astype(np.float64) for p in ps]


def _run(C, L, N, integrator, init, seed, variant=0):
    from differential_equations_resnet_amd.runtime import NetExecutor
    h = 8.0 / L
    spec = O.NetSpec(C=C, L=L, h=h, integrator=integrator)
    params = _params(spec, init, seed)
    rng = np.random.default_rng(100 + seed)
    imgs = rng.integers(0, 256, (N, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10)[rng.integers(0, 10, N)]
    ex = NetExecutor(N, 32, 32, 3, C, L, 10, h, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                     dtype="bfloat16", input_u8=True, integrator=integrator, variant=variant)
    assert ex.variant == variant  # 0: the production composition the bench times
    flat = torch.from_numpy(O.flatten(params).astype(np.float32)).cuda()
    loss, grads = ex.forward_backward(flat, torch.from_numpy(imgs).cuda(),
                                      torch.from_numpy(onehot.astype(np.float32)).cuda(), want_probs=True)
    probs_gpu = ex.probs.cpu().numpy().astype(np.float64)
    probs, cache = O.net_forward(spec, params, imgs)
    want_loss = O.net_loss(probs, onehot)
    g_want = O.net_backward(spec, params, cache, onehot)
    g_got = O.unflatten(grads.cpu().numpy().astype(np.float64), [p.shape for p in params])
    return spec, float(loss.item()), want_loss, probs_gpu, probs, g_got, g_want


def _check(spec, loss, want_loss, probs_gpu, probs, g_got, g_want, tag):
    assert np.abs(g_want[0]).max() > 0, "saturated softmax: the stem gradient is zero, the comparison is vacuous"
    errs = {name: rel_l2(a, b) for (name, a), (_, b) in zip(grad_groups(spec, g_got), grad_groups(spec, g_want))}
    worst = max(errs, key=errs.get)
    dl = abs(loss - want_loss) / abs(want_loss)
    dp = float(np.abs(probs_gpu - probs).max())
    print(f"\n{tag}: loss {loss:.6f} vs {want_loss:.6f} (rel {dl:.2e}), probs {dp:.2e}, "
          f"worst group rel-L2 {errs[worst]:.3e} ({worst}), median {np.median(list(errs.values())):.3e}")
    tens = assert_grad_tensors_max(spec, g_got, g_want, TENSOR_TOL, report_only=True)
    print(f"{tag}: worst per-tensor max|err|/group max {tens[1]:.3e} ({tens[0]})")
    assert dl <= 1e-2, dl                 # loss within 1 %
    assert dp <= 2e-2, dp                 # probabilities within 2e-2 absolute
    bad = {k: v for k, v in errs.items() if not v <= GROUP_TOL}
    assert not bad, bad
    assert_grad_tensors_max(spec, g_got, g_want, TENSOR_TOL)


@pytest.mark.parametrize("N,init,seed", [(8, "bench", 0), (16, "bench", 1), (8, "ref", 2)])
def test_c2_full_depth_vs_oracle(N, init, seed):
    _check(*_run(64, 30, N, "euler", init, seed), tag=f"C2 L=30 N={N} {init}")


@pytest.mark.parametrize("N,init,seed", [(8, "bench", 3), (8, "ref", 4)])
def test_c5_rk2_full_depth_vs_oracle(N, init, seed):
    _check(*_run(64, 30, N, "rk2", init, seed), tag=f"C5 L=30 N={N} {init}")


@pytest.mark.parametrize("N,init,seed", [(4, "bench", 5), (4, "ref", 6)])
def test_c3_full_depth_vs_oracle(N, init, seed):
    _check(*_run(16, 108, N, "euler", init, seed), tag=f"C3 L=108 N={N} {init}")


def test_c3_nearest_rounded_weights_are_the_systematic_error():
    """ASR_VARIANT_W_BF16 (W rounded to nearest bf16 instead of the balanced
    pack, asr_theta.hip k_theta_to_w_pack_bal): on the reference-init case
    above the 108-block net's worst block gradient leaves the 2e-2 bar
    (measured 2.7e-2 at block 92; the CPU emulation, tools/bf16_depth_emulate.py,
    puts 2.6e-2 of it on the W rounding alone: every output channel carries the
    fixed sum of its row's rounding errors through every pixel and layer),
    while the balanced pack, the same bf16 W with each channel's error sum
    kept near zero, stays under it (emulated 6.8e-3).  Both within 1 % on the
    loss; the balanced error is the smaller."""
    from differential_equations_resnet_amd.runtime import ASR_VARIANT_W_BF16
    worst = {}
    for v in (0, ASR_VARIANT_W_BF16):
        spec, loss, want_loss, probs_gpu, probs, g_got, g_want = _run(16, 108, 4, "euler", "ref", 6, variant=v)
        assert abs(loss - want_loss) <= 1e-2 * abs(want_loss)
        worst[v] = max(rel_l2(a, b) for (_, a), (_, b) in zip(grad_groups(spec, g_got), grad_groups(spec, g_want)))
    print(f"\nC3 ref init, worst group rel-L2: balanced {worst[0]:.3e}, nearest {worst[ASR_VARIANT_W_BF16]:.3e}")
    assert worst[0] <= GROUP_TOL and worst[0] < worst[ASR_VARIANT_W_BF16]
