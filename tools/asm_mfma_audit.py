"""Audit: every register an MFMA writes (its D operand) must not be read or
written by any later instruction before the MFMA result's wait states have
passed, on EVERY control-flow path from the MFMA (branch targets included).

gfx950 does not interlock an MFMA result against a following VALU / VMEM /
DS / SALU access: the compiler must put enough independent instructions or
`s_nop`s in between (cdna_hip_programming.md §5.7 item 2: "an MFMA's D -> any
reader or writer except the next MFMA taking it whole as C (accumulate
chain: 0)").  hipcc's hazard recognizer does this, but in round 4 a rotated
loop in a persistent-band `k_conv32` (fp32 `v_mfma_f32_16x16x4_f32`) reached
its epilogue by a branch straight from the last MFMA, and the epilogue read
the accumulator's 4th register after only `s_nop 2` (3 states; the
straight-line requirement is 10): output channels 4g+3 came out wrong
(DESIGN.md §3e).  This audit walks the control-flow graph of the device
assembly from each MFMA and reports any access that comes too early.

Counting follows the hazard recognizer: each instruction is one wait state,
`s_nop N` is N+1, labels and directives none.  The per-opcode requirement
(`REQUIRED`) is the number of states hipcc itself inserts between the MFMA
and a dependent VALU read on a straight line; tests/test_isa.py re-derives it
from probe kernels, so the table follows the toolchain.  Used by
tests/test_isa.py on every product source; as a script it scans one device .s
file and prints the findings."""
import re
import sys

# wait states between an MFMA and the first access of its D registers, gfx950,
# as hipcc (ROCm 7.2) inserts them on a straight line (probe: tests/test_isa.py)
REQUIRED = {
    "v_mfma_f32_16x16x32_bf16": 8,
    "v_mfma_f32_16x16x4_f32": 10,
}
DEFAULT_REQUIRED = 20  # unknown MFMA opcodes: the largest gfx950 requirement (16-pass XDL)

_REG = re.compile(r'\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b')


def _regs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(1):
            out.update((m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def _operands(body):
    parts = body.split(None, 1)
    if len(parts) < 2:
        return []
    return [p.strip() for p in parts[1].split(',')]


def _parse(lines):
    """(instructions, label -> instruction index): an instruction is
    (line number, opcode, operand list, operand text); labels point at the
    next instruction."""
    insts, labels = [], {}
    for i, l in enumerate(lines):
        t = l.strip()
        if not t or t.startswith(';'):
            continue
        if re.match(r'^[.\w$]+:', t):
            labels[t.split(':', 1)[0]] = len(insts)
            continue
        if t.startswith('.'):
            continue
        body = t.split(';')[0].strip()
        if not body:
            continue
        op = body.split(None, 1)[0]
        insts.append((i, op, _operands(body), body))
    return insts, labels


def _states(op, ops):
    if op == 's_nop':
        try:
            return int(ops[0], 0) + 1
        except (ValueError, IndexError):
            return 1
    return 1


def audit(src, required=None):
    """(number of early accesses, their descriptions) in device assembly text."""
    req_table = dict(REQUIRED)
    if required:
        req_table.update(required)
    funcs = re.split(r'\n(?=_Z[\w]+:|[A-Za-z_]\w*:\s+; @)', src)
    bad, findings = 0, []
    for f in funcs:
        name = f.split(':', 1)[0][:70]
        insts, labels = _parse(f.split('\n'))
        for k, (ln, op, ops, body) in enumerate(insts):
            if not op.startswith('v_mfma') or len(ops) < 4:
                continue
            dst = _regs(ops[0])
            if not dst:
                continue
            need = req_table.get(op, DEFAULT_REQUIRED)
            seen = set()
            stack = [(k + 1, 0, ())]
            while stack:
                j, cnt, path = stack.pop()
                while True:
                    if cnt >= need or j >= len(insts):
                        break
                    if (j, cnt) in seen:
                        break
                    seen.add((j, cnt))
                    ln2, op2, ops2, body2 = insts[j]
                    if op2.startswith('v_mfma') and len(ops2) >= 4 and _regs(ops2[3]) == dst \
                            and not (_regs(ops2[1]) | _regs(ops2[2])) & dst:
                        break  # accumulation chain: the next MFMA takes D whole as C (0 states)
                    if _regs(','.join(ops2)) & dst:
                        bad += 1
                        via = f" via {'/'.join(path)}" if path else ""
                        findings.append(f"{name}: line {ln}: '{body[:60]}' -> line {ln2}: '{body2[:60]}' "
                                        f"after {cnt} of {need} wait states{via}")
                        break
                    cnt += _states(op2, ops2)
                    if op2 in ('s_endpgm', 's_setpc_b64'):
                        break
                    if op2 == 's_branch' or op2.startswith('s_cbranch'):
                        tgt = ops2[0] if ops2 else ''
                        if tgt in labels:
                            stack.append((labels[tgt], cnt, path + (tgt,)))
                        if op2 == 's_branch':
                            break
                    j += 1
    return bad, findings


if __name__ == "__main__":
    n, found = audit(open(sys.argv[1]).read())
    for line in found[:40]:
        print(line)
    print("early MFMA-result accesses:", n)
