"""Audit: registers written by inline-asm global loads (the untracked loads
of asr_device.h: gload128_untracked / gload32_untracked) must not be read or
written by any instruction until an s_waitcnt vmcnt retires the load.  Walks
the control-flow graph of each function from every such load (fall-through
and branch targets, loop back-edges included), counting the vector-memory
ops issued after the load on each path (vmcnt retires in issue order, so a
compiler s_waitcnt vmcnt(k) retires it once k or more younger ops were
issued).  The kernels' own counted waits (vm_wait / barrier_vm: asm
s_waitcnt whose count is the ops the source issued since, the protocol that
guards the LDS-DMA'd tiles and is checked by the GPU parity tests) end the
walk as well; the audit proves that every path reaches one of them before
anything touches the registers.  Guards of the structurized switch inside
vm_wait are tracked (see _flags_after), so paths that skip every case are
not taken.  Any instruction on a path before that which mentions one of
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


# The backend structurizes a switch into guarded blocks whose guards are SGPR
# flags (s_mov_b64 s[a:b], -1 / 0; s_and(n2)_b64 vcc, exec, s[a:b];
# s_cbranch_vcc(n)z): tracking those constants keeps the walk off paths that
# skip every case of a counted-wait switch, which cannot execute.
def _flags_after(flags, op, body):
    d = dict(flags)
    args = [a.strip() for a in body.split(None, 1)[1].split(",")] if " " in body else []
    dst = args[0] if args else ""
    if op in ("s_and_b64", "s_andn2_b64") and dst == "vcc" and len(args) == 3 and args[1] == "exec":
        v = d.get(args[2])
        d.pop("vcc", None)
        if v is not None:
            d["vcc"] = (v != 0) if op == "s_and_b64" else (v == 0)
        return frozenset(d.items())
    if op.startswith("v_cmp") or dst == "vcc" or dst.startswith("vcc"):
        d.pop("vcc", None)
    if op.startswith("s_") and dst.startswith("s["):
        lo, hi = (int(t) for t in re.match(r"s\[(\d+):(\d+)\]", dst).groups())
        for key in [key for key in d if key.startswith("s[")]:
            a0, a1 = (int(t) for t in re.match(r"s\[(\d+):(\d+)\]", key).groups())
            if not (a1 < lo or a0 > hi):
                d.pop(key)
        if op == "s_mov_b64" and len(args) == 2 and args[1] in ("-1", "0"):
            d[dst] = int(args[1])
    elif op.startswith("s_") and re.match(r"s(\d+)$", dst):
        r = int(dst[1:])
        for key in [key for key in d if key.startswith("s[")]:
            a0, a1 = (int(t) for t in re.match(r"s\[(\d+):(\d+)\]", key).groups())
            if a0 <= r <= a1:
                d.pop(key)
    return frozenset(d.items())


def _branch_known(flags, op):
    """True / False when the branch direction follows from a known vcc, else None."""
    v = dict(flags).get("vcc")
    if v is None:
        return None
    if op == "s_cbranch_vccz":
        return not v
    if op == "s_cbranch_vccnz":
        return bool(v)
    return None


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
            stack = [(i + 1, 0, frozenset())]
            while stack:
                k, younger, flags = stack.pop()
                if k >= len(ins) or (k, younger, flags) in seen:
                    continue
                seen.add((k, younger, flags))
                op2, body2, _ = ins[k]
                w = re.search(r"s_waitcnt.*vmcnt\((\d+)\)", body2)
                if w and (younger >= int(w.group(1)) or ins[k][2]):
                    continue  # retired on this path, or a counted asm wait (vm_wait / barrier_vm)
                if not w and _regs(body2.split(None, 1)[1] if " " in body2 else "") & regs:
                    bad += 1
                    findings.append(f"{name}: '{body[:50]}' result touched by '{body2[:60]}' before a retiring wait")
                    continue
                if op2 == "s_endpgm":
                    continue
                y = min(younger + (1 if op2.startswith(VMEM) else 0), 64)
                fl = _flags_after(flags, op2, body2)
                if op2 == "s_branch" or op2.startswith("s_cbranch"):
                    tgt = body2.split()[-1]
                    taken = _branch_known(flags, op2)
                    if tgt in labels and taken is not False:
                        stack.append((labels[tgt], y, fl))
                    if op2 == "s_branch" or taken is True:
                        continue
                stack.append((k + 1, y, fl))
    return bad, findings


if __name__ == "__main__":
    n, found = audit(open(sys.argv[1]).read())
    for line in found[:40]:
        print(line)
    print("suspicious uses:", n)
