"""Build libasr.so (the HIP/gfx950 hot path + C ABI) in-tree with hipcc.

The shared library is written next to this file so it travels with the
repository snapshot to the GPU box; nothing is installed anywhere.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libasr.so")
SOURCES = ["asr_theta.hip", "asr_block_mfma.hip", "asr_conv_f32.hip", "asr_stem_head.hip", "asr_api.hip", "asr_dist.hip", "asr_deep16.hip", "asr_stages.hip"]
HEADERS = ["asr_common.h", "asr_device.h", os.path.join("..", "..", "include", "asr.h")]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain (ROCm) is required to build libasr.so")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    """Compile every HIP source for gfx950 (one object per source, in
    parallel) and link them into one shared library."""
    if not force and not _stale():
        return LIB
    cc = hipcc()
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
             "-Wno-unused-variable", "-Wno-unused-but-set-variable"]
    jobs = jobs or max(1, min(len(SOURCES), os.cpu_count() or 1, 8))
    with tempfile.TemporaryDirectory(prefix="asr_build_") as tmpdir:
        def compile_one(src):
            obj = os.path.join(tmpdir, os.path.splitext(src)[0] + ".o")
            cmd = [cc] + flags + ["-c", "-o", obj, os.path.join(CSRC, src)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            res = subprocess.run(cmd, capture_output=True, text=True)
            if res.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n" + res.stdout + res.stderr)
            return obj
        with ThreadPoolExecutor(jobs) as pool:
            objs = list(pool.map(compile_one, SOURCES))
        tmp = LIB + ".tmp"
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError("linking libasr.so failed:\n" + res.stdout + res.stderr)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
