"""CPU oracle for the antisymmetric-ResNet Euler-step hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package
(`differential_equations_resnet_amd`) imports, links or executes anything in
this directory.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may use it, and only as the checker (or, for
`cpu_baseline`, as the timed CPU restatement of the reference).

Contents
--------
asr_oracle.py      numpy (fp64 by default) restatement of the reference's
                   operator (`layers/tfkeras_layer_Conv2DAntisymmetric3By3.py`,
                   `layers/tfkeras_layer_Conv2DAntisymmetric.py`), identity
                   block (`models/tfkeras_resnets.py:28-94`), network
                   (`models/tfkeras_resnets.py:511-604`), loss and TF1 Adam
                   (`training/training.py:283-304`).
torch_cpu_ref.py   op-by-op restatement of the reference TF graph in PyTorch-CPU
                   (per-step slice/neg/concat kernel assembly, separate
                   bias/relu/mul/add ops, autograd).  This is the
                   "reference CPU path" timed by bench.py's cpu_baseline leg.
make_golden.py     regenerates tests/golden/*.npz from asr_oracle.py.

Pinning: see DESIGN.md "Oracle".  The conv primitive and the kernel assembly
are pinned by the reference notebooks' printed known-answer values
(tests/golden/kat_*.json); block/backward/network values are pinned only by
this restatement (parity for those is "pinned by restatement + finite
differences", not by reference-produced numbers, because TensorFlow 1.12 is
not importable here).
"""
