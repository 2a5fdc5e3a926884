"""Do two git revisions compile the product kernels to the same gfx950
instruction streams?  (A refactor claimed neutral must: round 4's switch
cleanup 6c75dab compiles every stack kernel bit-identically to f540cc2, the
measured tree before it.)  Labels are renumbered, comments and directives
dropped.  usage: python tools/isa_equiv.py REV_A REV_B [source.hip ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = "differential_equations_resnet_amd/csrc"


def kernels(asm):
    out = {}
    for f in re.split(r'\n(?=_Z[\w]+:|[A-Za-z_]\w*:\s+; @)', asm):
        name = f.split(':', 1)[0]
        if not name.startswith('_Z') or 's_endpgm' not in f:
            continue  # (data symbols and the metadata that follows them)
        body = [re.sub(r'\.LBB\d+_\d+', 'L', l.strip()) for l in f.split('\n')[1:]]
        # (the trailing __hip_cuid_<hash of the source file> symbol is not code)
        out[name] = [l for l in body if l and not l.startswith((';', '.', '__hip_cuid_'))]
    return out


def compile_rev(rev, src, d):
    dst = os.path.join(d, rev)
    os.makedirs(dst, exist_ok=True)
    tar = subprocess.run(["git", "-C", ROOT, "archive", rev, CSRC, "include"], check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", dst], input=tar, check=True)
    out = os.path.join(dst, src + ".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-w", "-o", out, os.path.join(dst, CSRC, src)], check=True)
    return kernels(open(out).read())


if __name__ == "__main__":
    a, b = sys.argv[1], sys.argv[2]
    srcs = sys.argv[3:] or ["asr_block_mfma.hip"]
    with tempfile.TemporaryDirectory() as d:
        for src in srcs:
            ka, kb = compile_rev(a, src, d), compile_rev(b, src, d)
            for k in sorted(set(ka) | set(kb)):
                tag = "same" if ka.get(k) == kb.get(k) else "DIFF"
                print(f"{tag} {src} {k[:90]}")
