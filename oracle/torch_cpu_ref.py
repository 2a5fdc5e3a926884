"""Op-by-op restatement of the reference TF 1.12 training graph in PyTorch-CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used as the CPU baseline
("the reference CPU path") by bench.py's cpu_baseline leg and
as an independent second restatement in the CPU tests.

It reproduces the reference's per-step op structure, which is what makes the
reference slow:
  * the kernel of every Conv2DAntisymmetric3By3 is re-assembled on every step
    from its variables with the same per-output-channel slice / neg / concat /
    stack sequence as layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:104-141
    and :210-293 (autograd then differentiates through all of those ops);
  * tf.nn.conv2d(NHWC, SAME) is a channels-last oneDNN convolution;
  * bias add, relu, h*x and the residual add are separate ops
    (…3By3.py:168-169, models/tfkeras_resnets.py:89-92);
  * loss = mean Keras categorical cross-entropy on softmax probabilities
    (training/training.py:295), TF1 Adam with epsilon 1e-7 (training.py:300-301).
Everything is float32, like the reference (dtype=torch.float64 gives the
same graph in double precision: the full-size fp32 parity check of BASELINE
C1 in tests/test_gpu_fullsize.py).

RefNet(..., assembly="vectorised") replaces the per-step op-by-op assembly by
one gather W = sign * theta[src] (the closed form W = P - P* + gamma*I of
SURVEY §8a-4, through oracle.asr_oracle.param_map): the same math with the
framework overhead of ~C^2 tiny ops per layer removed, so the two CPU numbers
separate that overhead from the convolution arithmetic.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def _acs_kernel(a, b, c, d, gamma):
    """_get_anti_centrosymmetric_kernel (…3By3.py:210-275) -> [3,3,1,C]."""
    e = torch.full_like(a, gamma)
    row1 = torch.cat([a, b, c], dim=1)
    row2 = torch.cat([d, e, -d], dim=1)
    row3 = torch.cat([-c, -b, -a], dim=1)
    return torch.cat([row1, row2, row3], dim=0)


def _acs_transpose(t):
    """_get_anti_centrosymmetric_transpose (…3By3.py:277-293)."""
    a, b, c = -t[0, 0, :], -t[0, 1, :], -t[0, 2, :]
    d, e, f = -t[1, 0, :], -t[1, 1, :], -t[1, 2, :]
    g, h, i = -t[2, 0, :], -t[2, 1, :], -t[2, 2, :]
    row1 = torch.stack([i, h, g], dim=0)
    row2 = torch.stack([f, e, d], dim=0)
    row3 = torch.stack([c, b, a], dim=0)
    return torch.stack([row1, row2, row3], dim=0)


def assemble_kernel(a, b, c, d, indeps, gamma):
    """The build loop of …3By3.py:104-141, executed every step like TF does."""
    C = a.shape[-1]
    acs = _acs_kernel(a, b, c, d, gamma)
    singles, transposes = [], []
    for o in range(C):
        nind = C - o - 1
        if nind > 0:
            ind = indeps[o]
            act = _acs_transpose(ind)
            single = torch.cat([acs[:, :, :, o], ind], dim=-1)
        else:
            single = acs[:, :, :, o]
        for i in range(o):
            ct = transposes[-(i + 1)][:, :, i].unsqueeze(-1)
            single = torch.cat([ct, single], dim=-1)
        singles.append(single)
        if nind > 0:
            transposes.append(act)
    return torch.stack(singles, dim=-1)  # HWIO


def conv2d_nhwc_same(x, w_hwio):
    """tf.nn.conv2d(x, W, [1,1,1,1], 'SAME', NHWC) on channels-last memory."""
    xn = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory (channels_last)
    w = w_hwio.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)
    y = F.conv2d(xn, w, padding=1)
    return y.permute(0, 2, 3, 1)


class RefNet:
    """antisymmetric single-block ResNet (tfkeras_resnets.py:547-597) in float32."""

    def __init__(self, params_np, C, L, h, gamma=0.0, num_classes=10, mean=127.5, std=127.5, assembly="reference",
                 dtype=torch.float32):
        if assembly not in ("reference", "vectorised"):
            raise ValueError(assembly)
        self.C, self.L, self.h, self.gamma, self.K = C, L, h, gamma, num_classes
        self.assembly = assembly
        if assembly == "vectorised":
            from .asr_oracle import param_map
            src, sign = param_map(C)
            self._src = torch.from_numpy(np.maximum(src, 0))
            self._sign = torch.from_numpy(sign.astype(np.float32)).to(dtype)
            self._is_gamma = torch.from_numpy(src < 0)
        self.mean, self.std = mean, std
        self.dtype = dtype
        self.params = [torch.tensor(np.asarray(p), dtype=dtype, requires_grad=True) for p in params_np]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    def _split(self):
        p = self.params
        nt = 4 + self.C - 1
        blocks, i = [], 2
        for _ in range(self.L):
            blocks.append((p[i:i + nt], p[i + nt]))
            i += nt + 1
        return p[0], p[1], blocks, p[i], p[i + 1]

    def forward(self, images_u8):
        c1k, c1b, blocks, fck, fcb = self._split()
        x = torch.as_tensor(images_u8).to(self.dtype)
        x = x - self.mean
        x = x / self.std
        x = conv2d_nhwc_same(x.contiguous(), c1k) + c1b
        x = torch.relu(x)
        for theta, b in blocks:
            if self.assembly == "vectorised":
                flat = torch.cat([t.reshape(-1) for t in theta])
                W = torch.where(self._is_gamma, torch.full((), self.gamma, dtype=self.dtype), self._sign * flat[self._src])
                W = W.view(3, 3, self.C, self.C)
            else:
                a, bb, c, d = theta[:4]
                W = assemble_kernel(a, bb, c, d, theta[4:], self.gamma)
            z = conv2d_nhwc_same(x, W)
            z = z + b
            r = torch.relu(z)
            if self.h != 1.0:
                r = self.h * r
            x = r + x
        gap = x.mean(dim=(1, 2))
        logits = gap @ fck + fcb
        return torch.softmax(logits, dim=-1)

    @staticmethod
    def keras_cce(probs, onehot):
        out = probs / probs.sum(dim=-1, keepdim=True)
        out = torch.clamp(out, 1e-7, 1.0 - 1e-7)
        return -(onehot * torch.log(out)).sum(dim=-1)

    def loss_and_grads(self, images_u8, onehot):
        """(probs, batch-mean loss, gradients in Keras weight order) without
        an optimizer step."""
        probs = self.forward(images_u8)
        loss = self.keras_cce(probs, torch.as_tensor(onehot, dtype=self.dtype)).mean()
        for p in self.params:
            p.grad = None
        loss.backward()
        return (probs.detach().numpy(), float(loss.detach()), [p.grad.detach().numpy().copy() for p in self.params])

    def train_step(self, images_u8, onehot, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7):
        probs = self.forward(images_u8)
        loss = self.keras_cce(probs, torch.as_tensor(onehot, dtype=self.dtype)).mean()
        for p in self.params:
            p.grad = None
        loss.backward()
        self.t += 1
        lr_t = lr * math.sqrt(1 - beta2 ** self.t) / (1 - beta1 ** self.t)
        with torch.no_grad():
            for p, m, v in zip(self.params, self.m, self.v):
                g = p.grad
                m.mul_(beta1).add_((1 - beta1) * g)
                v.mul_(beta2).add_((1 - beta2) * g * g)
                p.sub_(lr_t * m / (v.sqrt() + eps))
        return float(loss.detach())
