import numpy as np, torch
from bitalosdb_amd import synth
rng = np.random.default_rng(1)
v = synth.dict_values_gpu(400, 4096, device="cpu").numpy()
F = [0]; skip = 32; off = 0
for k in range(300):
    step = skip >> 5; off += step; skip += step; F.append(off)
F = np.array(F[:64])
def hashes(val, s):
    pos = s + F
    pos = pos[pos + 4 <= len(val)]
    u = (val[pos].astype(np.uint32) | (val[pos+1].astype(np.uint32) << 8) | (val[pos+2].astype(np.uint32) << 16) | (val[pos+3].astype(np.uint32) << 24))
    h = ((u * np.uint32(0x1e35a7bd)) & 0xffffffff) >> np.uint32(32 - 12)  # shift for 4 KiB blocks: table 4096 entries
    return h.astype(np.int64)
def conflict_cycles(dw, nb):
    # cycles beyond 1 = max over banks of distinct dwords in that bank, minus 1
    banks = {}
    for d in set(dw.tolist()):
        banks.setdefault(d % nb, 0); banks[d % nb] += 1
    return max(banks.values()) - 1
for nb in (32, 64):
    res = {"u16": [], "u16_xor": [], "u32": []}
    for i in range(400):
        val = v[i]
        for s in rng.integers(1, 3900, 8):
            h = hashes(val, int(s))
            res["u16"].append(conflict_cycles(h >> 1, nb))
            hx = h ^ ((h >> 6) & 0x3f)
            res["u16_xor"].append(conflict_cycles(hx >> 1, nb))
            res["u32"].append(conflict_cycles(h, nb))
    print(nb, {k: round(float(np.mean(x)), 2) for k, x in res.items()})
