"""LDS bank-conflict model of the LC kernel's PCM staging (MI355X_MICROARCH.md LDS table: ds_write_b32
2 x 32 lanes, bank (a/4) mod 32; ds_read_b128 4 x 16 lanes, bank (a/4) mod 64).  Writes: lane u
stores frame position long_pos(u, o), o = 0..15; reads: lane u loads words 4u + 256j .. +3.  Prints
the extra cycles (writes, reads) per frame for the identity layout and the best XOR swizzles of
word bits 2..4 (stage_idx in jaad_lc.hip)."""
import itertools, numpy as np
def lane_pos(u): return (u >> 3) | ((((u & 1) << 2) | (u & 2) | ((u >> 2) & 1)) << 3)
def long_pos(u, o):
    s, h = o >> 1, o & 1; k = lane_pos(u) + 64 * s
    if s < 4: return 512 + 2*k if h else 511 - 2*k
    return 1535 - 2*k if h else 2*k - 512
W32 = [range(0,32), range(32,64)]
R128 = [[*range(0,4),*range(12,16),*range(20,28)],[*range(4,12),*range(16,20),*range(28,32)],
        [*range(32,36),*range(44,48),*range(52,60)],[*range(36,44),*range(48,52),*range(60,64)]]
def cyc(addrs, width, groups, nb):
    t = 0
    for g in groups:
        banks = {}
        for l in g:
            for w in range(width):
                a = addrs[l] + w; banks.setdefault(a % nb, set()).add(a)
        t += max(len(v) for v in banks.values())
    return t
def ev(sw):
    wr = sum(cyc([sw(long_pos(u, o)) for u in range(64)], 1, W32, 32) - 2 for o in range(16))
    rd = sum(cyc([sw(4*u + 256*j) for u in range(64)], 4, R128, 64) - 4 for j in range(4))
    return wr, rd
print("identity", ev(lambda p: p))
best = []
for a, b in itertools.product(range(5, 10), range(5, 10)):
  for sh in (2,):
    f = lambda p, a=a, b=b: p ^ ((((p >> a) & 1) | (((p >> b) & 1) << 1) | 0) << 2)
    best.append((sum(ev(f)), 'x2', a, b))
for a, b, c in itertools.product(range(5, 11), repeat=3):
    f = lambda p, a=a, b=b, c=c: p ^ ((((p >> a) & 1) | (((p >> b) & 1) << 1) | (((p >> c) & 1) << 2)) << 2)
    best.append((sum(ev(f)), 'x3', a, b, c))
best.sort(); print(best[:8])
print("stage_idx (bits 5,6 -> 2,3):", ev(lambda p: p ^ (((p >> 5) & 3) << 2)))
