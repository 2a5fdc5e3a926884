"""LDS bank-conflict model for the tile layouts used by the HIP kernels.

Model (MI355X_MICROARCH.md §LDS): per instruction, lanes are serviced in fixed
groups; within a group the cost is max over banks of the number of distinct
dword addresses on that bank.  Used offline to pick the swizzle functions in
csrc/asr_tile.h (not part of the product).
"""
import itertools

G_B128 = [[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],
          [4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
G_B128 += [[l + 32 for l in g] for g in G_B128]
G_HALF = [list(range(32)), list(range(32, 64))]


def cost(addrs, nbytes, groups, mod):
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            for d in range(nbytes // 4):
                dw = a // 4 + d
                banks.setdefault(dw % mod, set()).add(dw)
        tot = max(tot, max((len(v) for v in banks.values()), default=0))
    return tot


def tile_off(row, col, q, W, NQ, swz):
    return ((row * (W + 2) + col) * NQ + (q ^ swz(row, col))) * 16


def check(C, W, swz, verbose=False):
    NQ = C // 8
    worst = {}
    # (a) B-frag ds_read_b128 for fwd/dgrad: pixel tile pt, tap kx, chunk block
    for pt in range(W // 16):
        for ky in range(3):
            for kx in range(3):
                for cb in range(max(1, C // 32)):
                    addrs = []
                    for l in range(64):
                        col = 16 * pt + (l & 15) + kx
                        if C >= 32:
                            q = 4 * cb + (l >> 4); r = ky
                        else:  # C=16: lanes>=32 read the next tap
                            q = (l >> 4) & 1; t = ky * 3 + kx + (l >> 5)
                            r, col = t // 3, 16 * pt + (l & 15) + t % 3
                        addrs.append(tile_off(r, col, q, W, NQ, swz))
                    worst['bfrag'] = max(worst.get('bfrag', 0), cost(addrs, 16, G_B128, 64))
    # (b) tr_b16 reads for wgrad A (x tile, shifted) and B (dz tile)
    for sx in range(3):
        for it in range(C // 16):
            for half in range(2):
                for kb in range(W // 32 if W >= 32 else 1):
                    addrs = []
                    for l in range(64):
                        g, w = l >> 4, l & 15
                        q, p = w >> 2, w & 3
                        pix = 32 * kb + 8 * g + q + 4 * half
                        col = pix + sx
                        chunk = 2 * it + (p >> 1)
                        addrs.append(tile_off(1, col, chunk, W, NQ, swz) + 8 * (p & 1))
                    worst['tr'] = max(worst.get('tr', 0), cost(addrs, 8, G_HALF, 64))
    # (c) staging ds_write_b128: thread t writes chunk index t (q fastest)
    for base in range(0, 4 * (W + 2) * NQ, 64):
        addrs = []
        for l in range(64):
            idx = base + l
            q = idx % NQ; pc = idx // NQ; col = pc % (W + 2); row = pc // (W + 2)
            addrs.append(tile_off(row, col, q, W, NQ, swz))
        worst['stage_w'] = max(worst.get('stage_w', 0), cost(addrs, 16, [list(range(i, i + 8)) for i in range(0, 64, 8)], 32))
    # (d) epilogue residual ds_read_b64: px = 16pt + (l&15), ch = 16 ot + 4(l>>4)
    for pt in range(W // 16):
        for ot in range(C // 16):
            addrs = []
            for l in range(64):
                px = 16 * pt + (l & 15); ch = 16 * ot + 4 * (l >> 4)
                addrs.append(tile_off(1, px + 1, ch // 8, W, NQ, swz) + 8 * ((ch // 4) & 1))
            worst['epi'] = max(worst.get('epi', 0), cost(addrs, 8, G_HALF, 64))
    return worst


if __name__ == '__main__':
    cands = {
        'none': lambda NQ: (lambda r, c: 0),
        'c>>1': lambda NQ: (lambda r, c: (c >> 1) % NQ),
        'c': lambda NQ: (lambda r, c: c % NQ),
        'c>>2': lambda NQ: (lambda r, c: (c >> 2) % NQ),
        'c^c>>3': lambda NQ: (lambda r, c: (c ^ (c >> 3)) % NQ),
        'c>>1^c>>4': lambda NQ: (lambda r, c: ((c >> 1) ^ (c >> 4)) % NQ),
        '(c>>1)^(c>>3)': lambda NQ: (lambda r, c: ((c >> 1) ^ (c >> 3)) % NQ),
    }
    for C in (16, 32, 64):
        for name, f in cands.items():
            print(C, name, check(C, 32, f(C // 8)))
