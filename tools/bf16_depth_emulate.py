"""Which bf16 rounding dominates the error of a deep bf16 Euler stack?

CPU-only emulation (numpy fp64 with bf16 roundings inserted where a kernel
stores or feeds bf16), compared with the plain fp64 oracle on the same
inputs, per gradient group (relative L2) -- used to choose the
precision fix for the C3 (L=108, C=16) failure in tests/test_gpu_depth.py.

Rounding points (each switchable):
  xs  the residual stream x_{l+1} = x_l + h relu(z) rounded to bf16 every block
  xc  the conv operand (bf16 copy of x_l fed to the MFMA)
  w   the assembled W in bf16: to nearest (w=1) or the executor's balanced
      pack (w='bal', helpers.w_bf16_balanced, asr_theta.hip)
  dz  the MFMA operand dz = h dy [z>0] in bf16
  dx  the chain gradient rounded to bf16 every `seg` blocks (deep16: 8)

usage: python tools/bf16_depth_emulate.py [C L N seed init]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/tests")
from helpers import bf16_round, grad_groups, rel_l2, w_bf16_balanced  # noqa: E402
from oracle import asr_oracle as O  # noqa: E402


def run(spec, params, imgs, onehot, xs=False, xc=False, w=False, dz=False, dx=False, seg=8):
    R = lambda on: (lambda a: bf16_round(a).astype(np.float64)) if on else (lambda a: a)  # noqa: E731
    rxs, rxc, rw, rdz, rdx = R(xs), R(xc), R(w), R(dz), R(dx)
    src, sign = O.param_map(spec.C)
    if w == "bal":
        rw = lambda a: w_bf16_balanced(a, src, sign).astype(np.float64)  # noqa: E731
    conv1_k, conv1_b, blocks, fc_k, fc_b = O.split_params(spec, params)
    x0 = O.normalize_input(imgs, spec)
    z1 = O.conv2d_same(x0, conv1_k) + conv1_b
    x = rxs(np.maximum(z1, 0))
    cache = []
    for theta, b in blocks:
        W = rw(O.assemble_from_map(O.flatten(theta), spec.C, src, sign, spec.gamma))
        xin = rxc(x)
        z = O.conv2d_same(xin, W) + b
        cache.append((xin, z, W))
        x = rxs(x + spec.h * np.maximum(z, 0))
    gap = x.mean(axis=(1, 2))
    probs = O.softmax(gap @ fc_k + fc_b)
    dlog = O.keras_cce_grad_logits(probs, onehot, 1.0 / len(onehot))
    g = np.broadcast_to((dlog @ fc_k.T)[:, None, None, :] / 1024.0, x.shape).copy()
    nth = int(sum(np.prod(s) for s in spec.theta_shapes()))
    back = []
    for li in range(spec.L - 1, -1, -1):
        xin, z, W = cache[li]
        d = rdz(spec.h * g * (z > 0))
        g = g - O.conv2d_same(d, W) + 2 * spec.gamma * d
        if li % seg == 0:
            g = rdx(g)
        back.append((O.unflatten(O.project_dW(O.conv2d_backprop_filter(xin, d), src, sign, nth),
                                 spec.theta_shapes()), d.sum(axis=(0, 1, 2))))
    back.reverse()
    dz1 = g * (z1 > 0)
    grads = [O.conv2d_backprop_filter(x0, dz1), dz1.sum(axis=(0, 1, 2))]
    for th, db in back:
        grads += th + [db]
    return probs, grads + [gap.T @ dlog, dlog.sum(0)]


def main():
    C, L, N, seed = (int(a) for a in (sys.argv[1:5] + ["16", "108", "4", "6"][len(sys.argv[1:5]):]))
    init = sys.argv[5] if len(sys.argv) > 5 else "ref"
    spec = O.NetSpec(C=C, L=L, h=8.0 / L)
    rng = np.random.default_rng(seed)
    params = O.init_params(spec, rng, np.float64, bias_std=0.05 if init == "ref" else 0.0)
    params[-2] = params[-2] * 0.1
    params = [p.astype(np.float32).astype(np.float64) for p in params]
    rng = np.random.default_rng(100 + seed)
    imgs = rng.integers(0, 256, (N, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10)[rng.integers(0, 10, N)]
    p0, g0 = run(spec, params, imgs, onehot)
    for name, kw in [("all (xs xc w dz dx/8)", dict(xs=1, xc=1, w=1, dz=1, dx=1)),
                     ("all, W balanced (the executor)", dict(xs=1, xc=1, w="bal", dz=1, dx=1)),
                     ("W balanced only", dict(w="bal")),
                     ("fp32 residual stream (xc w dz dx/8)", dict(xc=1, w=1, dz=1, dx=1)),
                     ("residual only (xs)", dict(xs=1)), ("conv operand only (xc)", dict(xc=1)),
                     ("W only", dict(w=1)), ("dz only", dict(dz=1)), ("dx/8 only", dict(dx=1)),
                     ("dx every block", dict(dx=1, seg=1))]:
        p, g = run(spec, params, imgs, onehot, **kw)
        errs = {k: rel_l2(a, b) for (k, a), (_, b) in zip(grad_groups(spec, g), grad_groups(spec, g0))}
        worst = max(errs, key=errs.get)
        print(f"{name:40s} probs {np.abs(p - p0).max():.2e}  worst group {errs[worst]:.3e} ({worst})  "
              f"median {np.median(list(errs.values())):.2e}")


if __name__ == "__main__":
    main()
