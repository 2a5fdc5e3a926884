"""MI355X-native antisymmetric-ResNet (Euler-step ODE blocks) hot path.

Host-side mirror of pierluigiferrari/differential_equations_resnet's plugin
surface (layers/, models/tfkeras_resnets.py) over libasr.so, a C-ABI library
of hand-written gfx950 HIP kernels (include/asr.h).
"""
__version__ = "0.1.0"
