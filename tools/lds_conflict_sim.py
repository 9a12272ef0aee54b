#!/usr/bin/env python3
"""Model of the LDS bank conflicts of k_mergek's in-LDS merge levels (runsk.hip):
512 lanes x 18 outputs, pointer-swap chains and lifting co-rank probes over one
pair of sorted runs, ds_read_b32 banking (two groups of 32 lanes, bank = word
% 32, identical words broadcast; MI355X_MICROARCH.md LDS table).  Prints the
mean extra cycles per wave instruction for the chains and the co-rank probes,
for the plain layout and two bank-spreading layouts, and the chain conflicts
against the B run's bank offset.  Measurement only (python3 tools/lds_conflict_sim.py)."""
import numpy as np
rng = np.random.default_rng(1)
NT, IT = 512, 18
def conflicts(addrs):
    # addrs: array (64,) word addresses for one wave instruction; ds_read_b32: groups of 32 lanes, bank=a%32
    tot = 0
    for g in range(2):
        a = addrs[32*g:32*(g+1)]
        a = a[a >= 0]
        u = np.unique(a)  # identical addresses broadcast
        banks = np.bincount(u % 32, minlength=32)
        tot += banks.max() - 1 if len(u) else 0
    return tot
def sim(LA, LB, layout=lambda p: p):
    A = np.sort(rng.integers(0, 2**32, LA)); B = np.sort(rng.integers(0, 2**32, LB))
    A0, B0 = 4, 4 + LA + IT + 1
    L = LA + LB
    d = np.arange(NT) * IT
    # co-rank per lane (exact)
    M = np.concatenate([np.zeros(LA, int), np.ones(LB, int)])[np.argsort(np.concatenate([A, B]), kind='stable')]
    nA = np.concatenate([[0], np.cumsum(M == 0)])
    chain_conf = []; co_conf = []
    # chain: each step, lane reads next element of side taken
    for w in range(NT // 64):
        lanes = np.arange(64*w, 64*w+64)
        dd = d[lanes]
        valid = dd < L
        ia = np.where(valid, nA[np.minimum(dd, L)], -1)
        ib = np.where(valid, dd - ia, -1)
        for k in range(IT):
            o = np.minimum(dd + k, L - 1)
            takeA = M[o] == 0
            # after taking, read next of that side
            pa = ia + 1; pb = ib + 1
            addr = np.where(takeA, A0 + layout(pa), B0 + layout(pb))
            addr = np.where(valid & (dd + k < L), addr, -1)
            chain_conf.append(conflicts(addr))
            ia = np.where(takeA, ia + 1, ia); ib = np.where(takeA, ib, ib + 1)
        # co-rank binary search probes (lifting, steps 2^j <= min(LA,LB))
        maxr = min(LA, LB); step = 1 << int(np.log2(maxr))
        lo = np.maximum(dd - LB, 0); hi = np.minimum(dd, LA); base = lo.copy()
        while step >= 1:
            i = base + step; ic = np.minimum(i, hi)
            addrA = A0 - 1 + layout(ic); addrB = B0 + layout(dd - ic)
            m = valid
            co_conf.append(conflicts(np.where(m, addrA, -1))); co_conf.append(conflicts(np.where(m, addrB, -1)))
            ok = (i <= hi) & (np.r_[A, 0][np.maximum(ic - 1, 0)] <= np.r_[B, 2**33][np.minimum(dd - ic, LB)])
            base = np.where(ok, i, base); step //= 2
    return np.mean(chain_conf), np.mean(co_conf), len(co_conf) / (NT // 64)
for LA, LB in [(900, 900), (1800, 1800), (3600, 3600)]:
    print(LA, LB, "plain", sim(LA, LB))
    print(LA, LB, "pad32", sim(LA, LB, lambda p: p + (p >> 5)))
    print(LA, LB, "xor", sim(LA, LB, lambda p: p ^ ((p >> 5) & 31)))
print("---- B offset sweep")
def sim_off(LA, LB, off):
    global rng
    rng = np.random.default_rng(7)
    A = np.sort(rng.integers(0, 2**32, LA)); B = np.sort(rng.integers(0, 2**32, LB))
    A0 = 4
    B0 = A0 + LA + IT + 1
    B0 += (off - B0) % 32
    L = LA + LB; d = np.arange(NT) * IT
    M = np.concatenate([np.zeros(LA, int), np.ones(LB, int)])[np.argsort(np.concatenate([A, B]), kind='stable')]
    nA = np.concatenate([[0], np.cumsum(M == 0)])
    cc = []
    for w in range(NT // 64):
        lanes = np.arange(64*w, 64*w+64); dd = d[lanes]; valid = dd < L
        ia = np.where(valid, nA[np.minimum(dd, L)], -1); ib = np.where(valid, dd - ia, -1)
        for k in range(IT):
            o = np.minimum(dd + k, L - 1); takeA = M[o] == 0
            addr = np.where(takeA, A0 + ia + 1, B0 + ib + 1)
            addr = np.where(valid & (dd + k < L), addr, -1)
            cc.append(conflicts(addr))
            ia = np.where(takeA, ia + 1, ia); ib = np.where(takeA, ib, ib + 1)
    return np.mean(cc)
for LA in (900, 1800, 3600):
    print(LA, [round(sim_off(LA, LA, off), 2) for off in range(0, 32, 2)])
