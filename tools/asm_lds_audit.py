"""Audit: results of inline-asm LDS reads (lds_rd64/128/u8, ds_read128) must
not be read by any instruction before an s_waitcnt lgkmcnt that retires them
(hipcc treats an asm output as available at once; a copy or spill made before
the wait reads garbage).  Models lgkmcnt as an in-order queue of DS/SMEM ops
within a basic block (control flow resets it: conservative for straight-line
code).  Used by tests/test_isa.py on every product source; as a script it
scans one device .s file and prints suspicious uses."""
import re
import sys


def audit(src):
    """(number of suspicious uses, their descriptions) in device assembly text."""
    funcs = re.split(r'\n(?=_Z[\w]+:|[A-Za-z_]\w*:\s+; @)', src)
    bad, findings = 0, []
    for f in funcs:
        name = f.split(':', 1)[0][:60]
        lines = f.split('\n')
        queue = []  # regs (or None) of each outstanding lgkm op, oldest first
        in_asm = False
        for i, l in enumerate(lines):
            t = l.strip()
            if t.startswith(';;#ASMSTART'):
                in_asm = True
                continue
            if t.startswith(';;#ASMEND'):
                in_asm = False
                continue
            m = re.search(r's_waitcnt.*lgkmcnt\((\d+)\)', t)
            if m:
                n = int(m.group(1))
                queue = queue[len(queue) - n:] if n < len(queue) else queue
                if n == 0:
                    queue = []
                continue
            if t.endswith(':') and not t.startswith(';'):
                queue = []  # label: unknown predecessors
                continue
            op = t.split(None, 1)[0] if t and not t.startswith(';') else ''
            if not op or op.startswith('.'):
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
            if hit:
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
