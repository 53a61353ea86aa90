"""Host simulation of K1's wavelet-tree statistics (namazu_amd/csrc/replayable_wt.hip), step for step, against
per-event decisions. A design check for the plan layout and the descents -- not the product, not the oracle.

usage: python tools/wt_sim.py [trials]
"""
import random
import sys


def bitlen(x):
    return x.bit_length()


def build(cm, e, chi, bb=5):
    """cm, e, chi per position (C order); rank blocks of 2^bb ranks. Returns the image as Python lists."""
    n = len(cm)
    keys = sorted(((cm[i] << 32) | ((0xFFFF - e[i]) << 16) | i) for i in range(n))
    cm_r = [k >> 32 for k in keys] + [0xFFFFFFFF]
    e_r = [0xFFFF - ((k >> 16) & 0xFFFF) for k in keys]
    S = [0] * n
    for j, k in enumerate(keys):
        S[k & 0xFFFF] = j
    K = bitlen(n)
    lb = K - bb if K > bb else 0  # levels above the 2^bb-rank blocks
    nw = n // 32 + 1
    lv = []
    cur = S
    for l in range(lb):
        k = K - l
        h = 1 << (k - 1)
        wb = [0] * nw
        for j in range(n):
            if cur[j] & h:
                wb[j >> 5] |= 1 << (j & 31)
        cum = [0] * nw
        acc = 0
        for w in range(nw):
            cum[w] = acc
            acc += bin(wb[w]).count("1")
        lv.append([(wb[w], cum[w]) for w in range(nw)])
        nxt = [None] * n
        for j in range(n):
            v = cur[j]
            s0 = v & ~(2 * h - 1)
            r1 = cum[j >> 5] + bin(wb[j >> 5] & ((1 << (j & 31)) - 1)).count("1") - (s0 >> 1)
            nxt[(s0 + h + r1) if (v & h) else (j - r1)] = v
        assert None not in nxt
        cur = nxt
    # level lb: the node of a block b holds ranks [BW b, BW b + BW) in position order; mk[b][o] = the set of
    # those ranks (bit r mod BW) among the node's first o entries
    BW = 1 << bb
    nb = (n >> bb) + 1
    mk = []
    for b in range(nb):
        row = [0]
        acc = 0
        for j in range(BW):
            p = BW * b + j
            if p < n:
                assert cur[p] >> bb == b
                acc |= 1 << (cur[p] & (BW - 1))
            row.append(acc)
        mk.append(row)
    return dict(n=n, K=K, lb=lb, nw=nw, lv=lv, mk=mk, cm=cm_r, e=e_r, chi=list(chi) + [0xFFFFFFFF],
                bb=bb)


def ones(lvl, s, p):
    w = lvl[p >> 5]
    return w[1] + bin(w[0] & ((1 << (p & 31)) - 1)).count("1") - (s >> 1)


def query(img, d, RA, RB, Hm, Hm2, m):
    """returns (W, keyA or None, keyB or None) following wt_seed_class after the searches."""
    n, lb, lv, mk, cm, ev = img["n"], img["lb"], img["lv"], img["mk"], img["cm"], img["e"]
    K = img["K"]
    NONE = None
    oA = oB = d
    cA = cB = 0
    lA = lB = NONE
    sA = qA = sB = qB = 0
    for l in range(lb):
        h = 1 << (K - l - 1)
        msk = ~(2 * h - 1)
        lvl = lv[l]
        s = RA & msk
        o = ones(lvl, s, s + oA)
        z = oA - o
        if RA & h:
            if z:
                lA, sA, qA = l + 1, s, z
            oA = o
        else:
            cA += o
            oA = z
        s = RB & msk
        o = ones(lvl, s, s + oB)
        z = oB - o
        if RB & h:
            if min(n - s, h) > z:
                lB, sB, qB = l + 1, s, z
            oB = o
        else:
            cB += o
            oB = z
    # the rank block of R: its first o entries are the node's prefix elements
    bb = img["bb"]
    BW = 1 << bb
    F = (1 << BW) - 1
    mA = mk[RA >> bb][oA]
    mB = mk[RB >> bb][oB]
    rA, rB = RA & (BW - 1), RB & (BW - 1)
    cA += bin(mA >> rA).count("1")
    cB += bin(mB >> rB).count("1")
    W = cA + (n - RB) - cB
    belA = mA & ((1 << rA) - 1)
    belB = (~mB & F) & ((1 << rB) - 1)
    hasA, hasB = d > 0, d < n
    hitA, hitB = belA != 0, belB != 0
    wrapA = hasA and not hitA and lA is NONE
    wrapB = hasB and not hitB and lB is NONE
    # a part with nothing below its bound: its largest rank overall, by the same descent from the root
    if wrapA:
        lA, sA, qA = 0, 0, d
    if wrapB:
        lB, sB, qB = 0, 0, d
    dA = hasA and not hitA  # descend from the tracked level
    dB = hasB and not hitB
    lA = lA if dA else lb
    lB = lB if dB else lb
    # the kernel does not track the node start: it rebuilds it from the level (R & ~(2^(K - l + 1) - 1))
    if dA:
        assert sA == RA & ~((2 << (K - lA)) - 1)
        sA = RA & ~((2 << (K - lA)) - 1)
    if dB:
        assert sB == RB & ~((2 << (K - lB)) - 1)
        sB = RB & ~((2 << (K - lB)) - 1)
    for l in range(min(lA, lB), lb):
        h = 1 << (K - l - 1)
        lvl = lv[l]
        if l >= lA:
            o = ones(lvl, sA, sA + qA)
            if o:
                sA += h
                qA = o
        if l >= lB:
            o = ones(lvl, sB, sB + qB)
            size = min(n - sB, 2 * h)
            if size > h + o:
                sB += h
                qB = o
            else:
                qB -= o
    def top(x):
        return x.bit_length() - 1
    pA = pB = None
    if not hasA:
        pass
    elif hitA:
        pA = (RA & ~(BW - 1)) + top(belA)
    else:
        v = mk[sA >> bb][qA]
        assert v
        pA = sA + top(v)
    if not hasB:
        pass
    elif hitB:
        pB = (RB & ~(BW - 1)) + top(belB)
    else:
        size = min(n - sB, BW)
        v = (~mk[sB >> bb][qB] & F) & (F >> (BW - size))
        assert v
        pB = sB + top(v)
    kA = kB = None
    if hasA:
        t = (Hm + cm[pA] - (m if wrapA else 0)) % (1 << 32)
        kA = (t << 32) | (0xFFFFFFFF - ev[pA])
    if hasB:
        t = (Hm2 + cm[pB] - (m if wrapB else 0)) % (1 << 32)
        kB = (t << 32) | (0xFFFFFFFF - ev[pB])
    return W, kA, kB


def brute(cm, e, d, Hm, Hm2, m):
    W = 0
    best = None
    for i in range(len(cm)):
        b = Hm if i < d else Hm2
        s = b + cm[i]
        wrap = s >= m
        t = s - m if wrap else s
        W += wrap
        k = (t << 32) | (0xFFFFFFFF - e[i])
        best = k if best is None or k > best else best
    return W, best


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rng = random.Random(7)
    for t in range(trials):
        n = rng.choice([9, 10, 15, 16, 31, 32, 33, 63, 64, 65, 96, 100, 127, 128, 129, 200, 255, 256, 257, 511, 512, 700,
                        1024, 2079])
        m = rng.choice([1, 2, 3, 7, 100, 1000, 10 ** 8, (1 << 30) - 1, (1 << 31) + 5, (1 << 32) - 1])
        dup = rng.random() < 0.3
        vals = [rng.randrange(m) for _ in range(max(1, n // 8 if dup else n))]
        cm = [rng.choice(vals) for _ in range(n)]
        e = rng.sample(range(4096), n)
        img = build(cm, e, [0] * n, bb=rng.choice([5, 6, 7]))
        for _ in range(30):
            d = rng.choice([0, n, rng.randrange(n + 1)])
            Hm = rng.randrange(m)
            Hm2 = rng.randrange(m)
            XA, XB = m - Hm, m - Hm2
            RA = sum(1 for x in cm if x < XA)
            RB = sum(1 for x in cm if x < XB)
            W, kA, kB = query(img, d, RA, RB, Hm, Hm2, m)
            bW, bk = brute(cm, e, d, Hm, Hm2, m)
            k = max(x for x in (kA, kB) if x is not None)
            assert W == bW, (n, m, d, W, bW)
            assert k == bk, (n, m, d, hex(k), hex(bk))
    print("ok", trials)


if __name__ == "__main__":
    main()


def query_quantile(img, d, RA, RB, Hm, Hm2, m):
    """As query(), with the predecessors by a count-guided descent from the root (no branch-off tracking in the
    count descent): the part's predecessor of R is its (#elements below R)-th smallest, or its largest when none is
    below R (it wraps)."""
    n, lb, lv, mk, cm, ev, K, bb = img["n"], img["lb"], img["lv"], img["mk"], img["cm"], img["e"], img["K"], img["bb"]
    BW = 1 << bb
    F = (1 << BW) - 1
    oA = oB = d
    cA = cB = 0
    for l in range(lb):
        h = 1 << (K - l - 1)
        msk = ~(2 * h - 1)
        s = RA & msk
        o = ones(lv[l], s, s + oA)
        if RA & h:
            oA = o
        else:
            cA += o
            oA = oA - o
        s = RB & msk
        o = ones(lv[l], s, s + oB)
        if RB & h:
            oB = o
        else:
            cB += o
            oB = oB - o
    mA = mk[RA >> bb][oA]
    mB = mk[RB >> bb][oB]
    cA += bin(mA >> (RA & (BW - 1))).count("1")
    cB += bin(mB >> (RB & (BW - 1))).count("1")
    W = cA + (n - RB) - cB

    def top(x):
        return x.bit_length() - 1

    def below(x):  # bits [0, x) of a block mask, x may pass the block
        return F if x >= BW else (1 << max(x, 0)) - 1

    kA = kB = None
    if d > 0:
        lt = d - cA
        wrap = lt == 0
        k = d - 1 if wrap else lt - 1
        s, q = 0, d
        for l in range(lb):
            h = 1 << (K - l - 1)
            o = ones(lv[l], s, s + q)
            z = q - o
            if k < z:
                q = z
            else:
                k -= z
                s += h
                q = o
        v = mk[s >> bb][q] & (F if wrap else below(RA - s))
        pA = s + top(v)
        t = (Hm + cm[pA] - (m if wrap else 0)) % (1 << 32)
        kA = (t << 32) | (0xFFFFFFFF - ev[pA])
    if d < n:
        lt = RB - (d - cB)
        wrap = lt == 0
        k = n - d - 1 if wrap else lt - 1
        s, q = 0, d
        for l in range(lb):
            h = 1 << (K - l - 1)
            o = ones(lv[l], s, s + q)
            zl = min(n - s, h)
            zs = zl - (q - o)  # zeros of the node from entry q on
            if k < zs:
                q = q - o
            else:
                k -= zs
                s += h
                q = o
        v = (~mk[s >> bb][q] & F) & (F >> (BW - min(n - s, BW))) & (F if wrap else below(RB - s))
        pB = s + top(v)
        t = (Hm2 + cm[pB] - (m if wrap else 0)) % (1 << 32)
        kB = (t << 32) | (0xFFFFFFFF - ev[pB])
    return W, kA, kB
