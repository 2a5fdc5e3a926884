"""development: event-timed C=64 forward / backward launches (eager and HIP
graph) at the bench shape, to compare with rocprofv3 kernel durations."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402

lib = _lib.load()
dev = rt.require_gpu()
N, H, W, C = 512, 32, 32, 64
g = torch.Generator(device=dev).manual_seed(7)
x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
dy = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
y, dx = torch.empty_like(x), torch.empty_like(x)
pm = rt.param_map(C)
scale = float(os.environ.get("EV_SCALE", "0.05"))
w = rt.theta_to_w(torch.randn(pm.n_theta, device=dev, generator=g) * scale, C, pm, 0.0, rt.ASR_BF16)
bias = torch.zeros(C, device=dev)
mask = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
wsb = int(lib.asr_conv_backward_workspace_bytes(N, H, W, C, rt.ASR_BF16))
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
_, tdst = pm.device(dev)


def cs():
    return torch.cuda.current_stream().cuda_stream


def fwd():
    _lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                    0.2667, N, H, W, C, 1, cs()))


def bwd():
    _lib.check(lib.asr_conv_backward(0, dy.data_ptr(), x.data_ptr(), mask.data_ptr(), w.data_ptr(), tdst.data_ptr(),
                                     pm.n_theta, 0.2667, 0.0, N, H, W, C, 1, dx.data_ptr(), None, None, None,
                                     ws.data_ptr(), wsb, cs()))


def ev(fn, reps, graph):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if graph:
        gr = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            fn()
        torch.cuda.current_stream().wait_stream(st)
        with torch.cuda.graph(gr):
            for _ in range(reps):
                fn()
        gr.replay()
        torch.cuda.synchronize()
        e0.record()
        gr.replay()
        e1.record()
    else:
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for _ in range(20):
    fwd()
    bwd()
torch.cuda.synchronize()
for name, fn in (("fwd", fwd), ("bwd", bwd)):
    for reps in (10, 50):
        print(f"{name} reps={reps}: eager {ev(fn, reps, False):.1f} us  graph {ev(fn, reps, True):.1f} us  "
              f"eager again {ev(fn, reps, False):.1f} us", flush=True)
