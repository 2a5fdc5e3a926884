"""GPU parity of the exact composition bench.py times (BASELINE.json
configs[1]: the C=64 Euler bf16 network) against the fp64 oracle, and the
reference-held conv KAT run through the C ABI itself.

The bf16 network runs with the production kernel set (variant 0, the
composition the bench line times): at C=64 the MFMA stem forward
(k_stem_fwd_mfma), ALL L blocks' forward in one k_fwd3_stack launch (two
4-wave workgroups per CU, whole images per workgroup, a ring of three LDS
tiles), ALL L blocks' backward in one k_bwd3_stack launch (one 12-wave
workgroup per CU: dgrad waves 0-3, pair-local wgrad waves 4-11, the stem's
relu' folded into block 0, pair-local weight-gradient slabs published
write-through with pass 1 of block l's reduction folded into block l-2's bands
behind the done[] counters, blocks 0-1 reduced after the launch), the
projection onto theta, and the MFMA stem weight gradient (k_stem_wgrad_mfma);
at C=16 the fused deep stack (k_fwd16_fused / k_bwd16_fused).  Every
workgroup walks 8 row bands per image and block, so the band pipeline, the
halo rows and the per-workgroup dW accumulation across bands are compared
with the oracle; N=192 also exercises the one-image-per-workgroup grid of
192 workgroups.  It is compared with
the fp64 oracle (oracle.net_forward / net_backward, a restatement of
tfkeras_resnets.py:547-597, training.py:295) on the same fp32 parameters and
uint8 images.

Tolerances: bf16 activations with fp32 accumulation against
fp64 — relative L2 error <= 2e-2 per gradient group (conv1 kernel, conv1
bias, each block's merged theta, each block's bias, fc kernel, fc bias: the
per-layer groups the reference's gradient norms use, training.py:385-409),
loss within 1 % relative, probabilities within 2e-2 absolute.
"""
import json
import os

import numpy as np
import pytest

from helpers import assert_grad_groups_rel_l2
from oracle import asr_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("C,N,L,h,seed", [(64, 8, 3, 8.0 / 30, 0), (64, 16, 4, 0.25, 1), (16, 8, 3, 8.0 / 30, 2),
                                          (64, 192, 2, 8.0 / 30, 3)])
def test_euler_bf16_network_matches_oracle(C, N, L, h, seed):
    from differential_equations_resnet_amd.runtime import NetExecutor
    spec = O.NetSpec(C=C, L=L, h=h)
    rng = np.random.default_rng(seed)
    params = [p.astype(np.float32).astype(np.float64) for p in O.init_params(spec, rng, np.float64, bias_std=0.05)]
    imgs = rng.integers(0, 256, (N, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10)[rng.integers(0, 10, N)]
    ex = NetExecutor(N, 32, 32, 3, C, L, 10, h, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                     dtype="bfloat16", input_u8=True)
    assert ex.variant == 0  # the production composition
    flat = torch.from_numpy(O.flatten(params).astype(np.float32)).cuda()
    x = torch.from_numpy(imgs).cuda()
    loss, grads = ex.forward_backward(flat, x, torch.from_numpy(onehot.astype(np.float32)).cuda(), want_probs=True)
    probs_gpu = ex.probs.cpu().numpy()
    probs, cache = O.net_forward(spec, params, imgs)
    want_loss = O.net_loss(probs, onehot)
    assert np.abs(probs_gpu - probs).max() < 2e-2
    assert abs(loss.item() - want_loss) <= 1e-2 * want_loss
    g_want = O.net_backward(spec, params, cache, onehot)
    g_got = O.unflatten(grads.cpu().numpy().astype(np.float64), [p.shape for p in params])
    assert_grad_groups_rel_l2(spec, g_got, g_want, 2e-2)


def test_conv_kat_through_c_abi():
    """antisymmetric_conv_kernel.ipynb cells 1-3 (:33-242): the printed 7x7
    image, 3x3 kernel and tf.nn.conv2d(SAME, NHWC) output.  Run through
    asr_conv_forward (ASR_MODE_CONV, fp32, C=1, plain HWIO kernel = the
    regular parametrisation): |err| < 1e-6, and the flipped kernel does not
    match (cross-correlation)."""
    from differential_equations_resnet_amd import runtime as rt
    rt.require_gpu()
    with open(os.path.join(GOLDEN, "kat_conv7x7.json")) as f:
        k = json.load(f)
    x = torch.tensor(k["image_hw"], dtype=torch.float32).view(1, 7, 7, 1).cuda().contiguous()
    w = torch.tensor(k["kernel_hw"], dtype=torch.float32).view(3, 3, 1, 1).cuda().contiguous()
    want = np.array(k["conv2d_same_hw"], np.float64)
    zero = torch.zeros(1, dtype=torch.float32).cuda()
    y = rt.conv_forward(rt.ASR_MODE_CONV, x, w, zero).cpu().numpy()[0, :, :, 0]
    assert np.abs(y - want).max() < 1e-6, np.abs(y - want).max()
    yf = rt.conv_forward(rt.ASR_MODE_CONV, x, torch.flip(w, (0, 1)).contiguous(), zero).cpu().numpy()[0, :, :, 0]
    assert np.abs(yf - want).max() > 0.1
