# lab (host only): lane-steps of the LDS walk's fixed groups against refilling finished slots, on the
# element counts of generator values (C3: 1 KiB; mixdec: U[64, 4096] in the tier-2 buckets).  DESIGN 4.2.
import numpy as np, sys
sys.path.insert(0, '/root/repo')
from bitalosdb_amd import synth
from oracle import oracle as O
def elems(s):
    p = 0
    while s[p] >= 0x80: p += 1
    p += 1; e = 0
    while p < len(s):
        t = s[p]; ty = t & 3
        if ty == 0:
            x = t >> 2
            if x < 60: ln = x + 1; p += 1
            else: nb = x - 59; ln = int.from_bytes(s[p+1:p+1+nb], 'little') + 1; p += 1 + nb
            p += ln
        else: p += 1 + ty if ty < 3 else 5
        e += 1
    return e
def gen(kind, n):
    if kind == 'c3':
        v = synth.dict_values_gpu(n, 1024, device="cpu", seed=0xC3).numpy()
        return np.array([elems(O.snappy_encode(r.tobytes())) for r in v])
    rng = np.random.default_rng(5); lens = rng.integers(64, 4097, n)
    v = synth.dict_values_gpu(n, 4096, device="cpu", seed=0xC4).numpy()
    e = np.array([elems(O.snappy_encode(r[:L].tobytes())) for r, L in zip(v, lens)])
    return e, lens
def groups(e, B):
    m = len(e)//B*B
    return e[:m].reshape(-1, B).max(1).sum(), m
def refill(e, B, K, ov):
    # B slots; walk until >= K slots done (or none left to refill and all done), then refill; ov = steps per pause
    it = iter(e); rem = np.zeros(B, int); act = np.zeros(B, bool); steps = 0; pauses = 0; nblk = 0
    for b in range(B):
        x = next(it, None)
        if x is not None: rem[b] = x; act[b] = True; nblk += 1
    exhausted = False
    while act.any():
        need = K if not exhausted else act.sum()
        # steps until `need` more slots finish... simulate step by step
        done_now = 0
        while True:
            r = rem[act]
            k = min(need, len(r))
            t = np.sort(r)[k-1]
            steps += t; rem[act] -= t
            fin = act & (rem <= 0)
            break
        act &= ~fin
        if exhausted: continue
        pauses += 1
        for b in np.nonzero(fin)[0]:
            x = next(it, None)
            if x is None: exhausted = True; break
            rem[b] = x; act[b] = True; nblk += 1
    return steps + pauses * ov, nblk
def report(name, e, B):
    g, m = groups(e, B)
    ideal = e[:m].sum() / B
    print("%s B=%d: groups %.0f steps (ideal %.0f, waste %.1f%%)" % (name, B, g, ideal, 100*(1-ideal/g)))
    for K in (B//4, B//3, B//2):
        for ov in (1.0, 2.0, 4.0):
            s, nb = refill(e[:m], B, K, ov)
            print("   refill K=%d ov=%.0f: %.0f steps -> %.1f%% of groups" % (K, ov, s, 100*s/g))
e = gen('c3', 6000); report('c3 tier1', e, 18)
e2, lens = gen('mix', 6000)
for lo, hi, B in ((1024, 1792, 13), (1792, 2560, 9), (2560, 3328, 7), (3328, 5000, 6)):
    m = (lens > lo) & (lens <= hi); report('mix %d-%d' % (lo, hi), e2[m], B)
