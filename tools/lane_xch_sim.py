import numpy as np
def bitrev(x, n):
    return int(format(x, f"0{n}b")[::-1], 2)
u = np.arange(64)
# pass-1 layout: register s holds e = 8*bitrev6(u) + bitrev3(s)
c = [np.array([8 * bitrev(int(l), 6) + bitrev(s, 3) for l in u]) for s in range(8)]
def dpp_ror(src, n):  # lane i reads lane (i - n) mod 16 within its row
    return np.array([src[(i & ~15) | ((i - n) & 15)] for i in range(64)])
def qp(src, x):
    return np.array([src[i ^ x] for i in range(64)])
def bankmask(mask):
    return np.array([(mask >> ((i & 15) >> 2)) & 1 for i in range(64)], bool)
def xch(a, b, L):
    if L == 5:
        return np.concatenate([a[:32], b[:32]]), np.concatenate([a[32:], b[32:]])
    if L == 4:
        ra = a.copy(); rb = b.copy()
        for r in (0, 2):
            ra[(r + 1) * 16:(r + 2) * 16] = b[r * 16:(r + 1) * 16]
            rb[r * 16:(r + 1) * 16] = a[(r + 1) * 16:(r + 2) * 16]
        return ra, rb
    if L == 3:
        na = np.where(bankmask(0xC), dpp_ror(b, 8), a); nb = np.where(bankmask(0x3), dpp_ror(a, 8), b); return na, nb
    if L == 2:
        na = np.where(bankmask(0xA), dpp_ror(b, 4), a); nb = np.where(bankmask(0x5), dpp_ror(a, 12), b); return na, nb
    x = 1 << L
    hi = (u >> L) & 1
    return np.where(hi == 1, qp(b, x), a), np.where(hi == 1, b, qp(a, x))
def xbit(c, I, L):
    c = list(c)
    for s in range(8):
        if (s >> I) & 1: continue
        c[s], c[s | 1 << I] = xch(c[s], c[s | 1 << I], L)
    return c
c = xbit(c, 0, 5); c = xbit(c, 1, 4); c = xbit(c, 2, 3)
for s in range(8):
    assert all(((c[s] >> 3) & 7) == s), s
    assert all((c[s] & 7) == (u >> 3)), s
c = xbit(c, 0, 2); c = xbit(c, 1, 1); c = xbit(c, 2, 0)
sig = (u >> 3) | (np.array([bitrev(int(l) & 7, 3) for l in u]) << 3)
for s in range(8):
    assert all(c[s] == sig + 64 * s), (s, c[s][:8], sig[:8])
print("ok")
