"""Audit: results of inline-asm LDS reads (lds_rd64/128/u8, ds_read128) must
not be read by any instruction before an s_waitcnt lgkmcnt that retires them
(hipcc treats an asm output as available at once; a copy or spill made before
the wait reads garbage).  Models lgkmcnt as an in-order queue of DS/SMEM ops
along the control flow (branch targets merge the queues of every path to
them).  Used by tests/test_isa.py on every product source; as a script it
scans one device .s file and prints suspicious uses."""
import re
import sys


def _merge(a, b):
    """lgkm queues of two control-flow paths, youngest ends aligned, register
    sets united (None = unreachable)."""
    if a is None:
        return None if b is None else list(b)
    if b is None:
        return list(a)
    n = max(len(a), len(b))
    out = []
    for k in range(n, 0, -1):
        x = a[-k] if k <= len(a) else None
        y = b[-k] if k <= len(b) else None
        out.append((x or set()) | (y or set()) if (x or y) else None)
    return out


def audit(src):
    """(number of suspicious uses, their descriptions) in device assembly text.
    The pending-read state follows the control flow: every branch carries its
    queue to its target label, a label merges the fall-through queue with the
    queues of the branches to it (two passes, so loop back edges count)."""
    funcs = re.split(r'\n(?=_Z[\w]+:|[A-Za-z_]\w*:\s+; @)', src)
    bad, findings = 0, []
    for f in funcs:
        name = f.split(':', 1)[0][:60]
        lines = f.split('\n')
        at_label = {}  # label -> merged queue of the branches to it
        for final in (False, True):
            queue = []  # regs (or None) of each outstanding lgkm op, oldest first; None: unreachable
            in_asm = False
            for i, l in enumerate(lines):
                t = l.strip()
                if t.startswith(';;#ASMSTART'):
                    in_asm = True
                    continue
                if t.startswith(';;#ASMEND'):
                    in_asm = False
                    continue
                if t.endswith(':') and not t.startswith(';') or re.match(r'^\.?\w+:\s+;', t):
                    lab = t.split(':', 1)[0]
                    queue = _merge(queue, at_label.get(lab))
                    if queue is None:
                        queue = []
                    continue
                if queue is None:
                    continue  # unreachable until the next label
                m = re.search(r's_waitcnt.*lgkmcnt\((\d+)\)', t)
                if m:
                    n = int(m.group(1))
                    queue = queue[len(queue) - n:] if n < len(queue) else queue
                    if n == 0:
                        queue = []
                    continue
                op = t.split(None, 1)[0] if t and not t.startswith(';') else ''
                if not op or op.startswith('.'):
                    continue
                if op.startswith('s_cbranch') or op == 's_branch':
                    tgt = t.split(None, 1)[1].split(';')[0].strip()
                    at_label[tgt] = _merge(at_label.get(tgt), queue)
                    if op == 's_branch':
                        queue = None
                    continue
                if op in ('s_endpgm', 's_setpc_b64'):
                    queue = None
                    continue
                used = set()
                body = t.split(';')[0].strip()
                if ' ' in body:
                    args = body.split(None, 1)[1].split(',')
                    is_store = op.startswith(('ds_write', 'global_store', 'buffer_store', 'scratch_store'))
                    srcs = ','.join(args if is_store else args[1:])
                    for mm in re.finditer(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b', srcs):
                        if mm.group(3):
                            used.add(int(mm.group(3)))
                        else:
                            used.update(range(int(mm.group(1)), int(mm.group(2)) + 1))
                pend = set()
                for regs in queue:
                    if regs:
                        pend |= regs
                hit = used & pend
                if hit and final:
                    bad += 1
                    findings.append(f"{name}: line {i}: '{t[:70]}' reads v{sorted(hit)[:4]} before its asm LDS read "
                                    f"retired")
                if op.startswith('ds_') or op.startswith('s_load') or op.startswith('s_buffer_load'):
                    regs = None
                    if in_asm and op.startswith('ds_read'):
                        mm = re.match(r'ds_read\w*\s+v\[?(\d+)(?::(\d+))?\]?', t)
                        if mm:
                            lo = int(mm.group(1))
                            hi = int(mm.group(2) or lo)
                            regs = set(range(lo, hi + 1))
                    queue.append(regs)
    return bad, findings


if __name__ == "__main__":
    n, found = audit(open(sys.argv[1]).read())
    for line in found[:40]:
        print(line)
    print("suspicious uses:", n)
