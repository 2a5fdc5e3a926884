"""Audit: registers written by inline-asm global loads (the untracked loads
of asr_device.h: gload128_untracked / gload32_untracked) must not be read or
written by any instruction until an s_waitcnt vmcnt retires the load.  Walks
the control-flow graph of each function from every such load (fall-through
and branch targets, loop back-edges included), counting the vector-memory
ops issued after the load on each path (vmcnt retires in issue order, so
s_waitcnt vmcnt(k) retires it once k or more younger ops were issued); a
barrier_vm's s_barrier also ends the walk: barrier_vm = vm_wait(n) (a
switch of counted waits) + one asm barrier, so every path into that barrier
passed a wait whose count is the stores issued since (kept by the source:
the protocol that guards the LDS-DMA'd tiles, checked by the GPU parity
tests).  Any instruction on a path before that which mentions one of
the registers is a finding: the compiler copied, spilled or reused them.  Used by tests/test_isa.py; as a script it scans one .s file."""
import re
import sys

VMEM = ("global_", "buffer_", "flat_", "scratch_")
LOAD_RE = re.compile(r"^(global_load_dword\w*)\s+v\[?(\d+)(?::(\d+))?\]?")


def _regs(text):
    out = set()
    for mm in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        if mm.group(3):
            out.add(int(mm.group(3)))
        else:
            out.update(range(int(mm.group(1)), int(mm.group(2)) + 1))
    return out


def _parse(func_text):
    """instructions as (op, text, in_asm) and label -> index"""
    ins, labels, in_asm = [], {}, False
    for l in func_text.split("\n"):
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not t or t.startswith(";"):
            continue
        if t.endswith(":") or re.match(r"^[.\w]+:\s*(;.*)?$", t):
            labels[t.split(":")[0]] = len(ins)
            continue
        if t.startswith("."):
            continue
        body = t.split(";")[0].strip()
        ins.append((body.split(None, 1)[0], body, in_asm))
    return ins, labels


def audit(src):
    funcs = re.split(r"\n(?=_Z[\w]+:|[A-Za-z_]\w*:\s+; @)", src)
    bad, findings = 0, []
    for f in funcs:
        name = f.split(":", 1)[0][:60]
        ins, labels = _parse(f)
        for i, (op, body, in_asm) in enumerate(ins):
            m = LOAD_RE.match(body) if in_asm else None
            if not m or "lds" in op:
                continue
            lo = int(m.group(2))
            regs = set(range(lo, int(m.group(3) or lo) + 1))
            seen = set()
            stack = [(i + 1, 0)]
            while stack:
                k, younger = stack.pop()
                if k >= len(ins) or (k, younger) in seen:
                    continue
                seen.add((k, younger))
                op2, body2, _ = ins[k]
                w = re.search(r"s_waitcnt.*vmcnt\((\d+)\)", body2)
                if w and younger >= int(w.group(1)):
                    continue  # retired on this path
                if op2 == "s_barrier" and ins[k][2]:
                    continue  # barrier_vm: its counted wait precedes this barrier on every path
                if not w and _regs(body2.split(None, 1)[1] if " " in body2 else "") & regs:
                    bad += 1
                    findings.append(f"{name}: '{body[:50]}' result touched by '{body2[:60]}' before a retiring wait")
                    continue
                if op2 == "s_endpgm":
                    continue
                y = min(younger + (1 if op2.startswith(VMEM) else 0), 64)
                if op2 == "s_branch" or op2.startswith("s_cbranch"):
                    tgt = body2.split()[-1]
                    if tgt in labels:
                        stack.append((labels[tgt], y))
                    if op2 == "s_branch":
                        continue
                stack.append((k + 1, y))
    return bad, findings


if __name__ == "__main__":
    n, found = audit(open(sys.argv[1]).read())
    for line in found[:40]:
        print(line)
    print("suspicious uses:", n)
