"""CPU check of the LDS snappy element walk (k_snappy_lds, bhg_snappy_dec.hip):
the device function `snappy_walk_lds` is extracted from the product source,
compiled for the host with clang, and run on an LDS-shaped byte array laid out
as the kernel lays out an in-place slot (output from the slot start, stream
staged at the slot end).  Every result must be the restated golang/snappy
decode (oracle, parity pinned by pyarrow interop in test_oracle_snappy.py),
SNAPPY_CORRUPT exactly where the restatement rejects, or a hand-over to the
global-memory pass (2) -- never wrong bytes.  No GPU involved; the GPU run of
the same code is tests/test_gpu_decode.py."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "bitalosdb_amd", "csrc", "bhg_snappy_dec.hip")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
SLOT = 1088   # kSlSlot (bhg_snappy_dec.hip): tier 1, values <= 1 KiB
SLOT2 = 4160  # kSlSlot2: tier 2, values <= 4 KiB


@pytest.fixture(scope="module")
def walk(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("no clang++")
    s = open(SRC).read()
    # the walk is a template on G (lanes per block).  On the host one call is the whole group, in
    # the lanes' lockstep order: an element's parallel 16-B ops go in rounds of G, each round's G
    # reads before its G writes (one ds_read, then one ds_write instruction, on the GPU).  (A literal
    # in an in-place slot reads its stream just above the output it writes, so ops in another
    # order would read bytes a previous op overwrote.)
    i0 = s.index("template <int G>\n__device__ __forceinline__ uint32_t snappy_walk_lds(")
    i1 = s.index("\n}\n", i0) + 3  # the end of the function
    body = s[i0:i1].replace("__device__ __forceinline__ ", "")
    par = ("            for (uint32_t t = 16 * g; t < n; t += 16 * G)\n"
           "                *reinterpret_cast<u32x4_lds_u *>(lds + o + t) = *reinterpret_cast<const u32x4_lds_u *>(lds + a + t);\n")
    assert body.count(par) == 1
    body = body.replace(par, (
        "            for (uint32_t t0 = 0; t0 < n; t0 += 16 * G) {\n"
        "                u32x4 tmp[G];\n"
        "                for (uint32_t gg = 0; gg < G; gg++)\n"
        "                    if (t0 + 16 * gg < n) tmp[gg] = *reinterpret_cast<const u32x4_lds_u *>(lds + a + t0 + 16 * gg);\n"
        "                for (uint32_t gg = 0; gg < G; gg++)\n"
        "                    if (t0 + 16 * gg < n) *reinterpret_cast<u32x4_lds_u *>(lds + o + t0 + 16 * gg) = tmp[gg];\n"
        "            }\n"))
    for gl in (1, 2, 4):
        body += ('extern "C" uint32_t snappy_walk_lds_%d(uint8_t *lds, uint32_t sp, uint32_t se, uint32_t op, '
                 'uint32_t dlen) { return snappy_walk_lds<%d>(lds, sp, se, op, dlen, 0); }\n' % (gl, gl))
    hdr = ("#include <stdint.h>\n"
           "#define __builtin_amdgcn_s_waitcnt(x) ((void)0)\n"   # a wait-count hint on the GPU
           "typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));\n"
           "typedef uint64_t u64_lds_u __attribute__((aligned(1), may_alias));\n"
           "typedef u32x4 u32x4_lds_u __attribute__((aligned(1), may_alias));\n")
    d = tmp_path_factory.mktemp("walk")
    cpp, so = d / "walk.cpp", d / "walk.so"
    cpp.write_text(hdr + body)
    subprocess.check_call([CLANG, "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(so), str(cpp)])
    lib = ctypes.CDLL(str(so))
    for gl in (1, 2, 4):
        f = getattr(lib, "snappy_walk_lds_%d" % gl)
        f.restype = ctypes.c_uint32
        f.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 4
    return lib


@pytest.fixture(params=[1, 2, 4])
def lanes(request):
    return request.param


def run_slot(walk, stream, dlen, slot=SLOT, lanes=1):
    """Stage `stream` as k_snappy_lds does and walk it; returns (code, output bytes)."""
    clen = len(stream)
    pos = (slot - 8 - ((clen + 15) & ~15)) & ~15
    lds = np.zeros(2 * slot + 64, dtype=np.uint8)   # the slot, then a neighbour slot and the pad
    lds[pos:pos + clen] = np.frombuffer(stream, dtype=np.uint8)
    hdr = 0
    while hdr < 5 and lds[pos + hdr] >= 0x80:
        hdr += 1
    hdr += 1
    r = getattr(walk, "snappy_walk_lds_%d" % lanes)(lds.ctypes.data, pos + hdr, pos + clen, 0, dlen)
    return r, lds[:dlen].tobytes()


def uvarint(x):
    out = bytearray()
    while x >= 0x80:
        out.append(x & 0x7f | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def values(rng, k):
    for i in range(k):
        n = rng.choice([1, 4, 15, 16, 17, 63, 64, 65, 100, 500, 1000, 1024])
        kind = i % 5
        if kind == 0:
            yield bytes(rng.getrandbits(8) for _ in range(n))              # literals only
        elif kind == 1:
            yield bytes(rng.choice(b"ab") for _ in range(n))              # short-offset copies
        elif kind == 2:
            yield (b"0123456789abcdefXYZ" * 60)[:n]                       # period 19
        else:                                                             # 16-B words, the C3 shape
            words = [bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(8)]
            yield b"".join(rng.choice(words) if rng.random() > 0.25 else
                           bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(64))[:n]


def test_walk_matches_restated_decode(walk, lanes):
    rng = random.Random(5)
    codes = {0: 0, 1: 0, 2: 0}
    for v in values(rng, 1500):
        st = O.snappy_encode(v)
        if len(st) + 24 > SLOT or len(v) > 1024:
            continue                       # not staged: the kernel sends it to k_snappy_rt
        r, out = run_slot(walk, st, len(v), lanes=lanes)
        codes[r] += 1
        assert r != 1
        if r == 0:
            assert out == v
    assert codes[0] > 1000


def test_walk_tier2_slots(walk, lanes):
    """The same walk in tier 2's 4,160-B slots: values of 1-4 KiB (dict-like tokens, runs,
    incompressible) decode to the restated bytes or are handed over, never wrong."""
    rng = random.Random(9)
    dic = bytes(rng.getrandbits(8) for _ in range(4096))
    codes = {0: 0, 1: 0, 2: 0}
    for i in range(300):
        n = rng.choice([1025, 1500, 2048, 3000, 4000, 4096])
        k = i % 3
        if k == 0:
            v = bytearray()
            while len(v) < n:
                a = rng.randrange(0, 4000)
                v += dic[a:a + rng.randrange(4, 65)] if rng.random() > 0.2 else bytes(
                    rng.getrandbits(8) for _ in range(rng.randrange(4, 65)))
            v = bytes(v[:n])
        elif k == 1:
            v = bytes(rng.getrandbits(8) for _ in range(n))
        else:
            v = (b"abc" * 2000)[:n]
        st = O.snappy_encode(v)
        if len(st) + 24 > SLOT2:
            continue
        r, out = run_slot(walk, st, len(v), SLOT2, lanes)
        codes[r] += 1
        assert r != 1
        if r == 0:
            assert out == v
    assert codes[0] > 250


def test_walk_hands_over_when_output_overtakes_stream(walk, lanes):
    body = bytes([0]) + b"x"
    body += (bytes([(64 - 1) << 2 | 2]) + (1).to_bytes(2, "little")) * 10
    body += bytes([(59 - 1) << 2 | 2]) + (1).to_bytes(2, "little")
    body += (bytes([2]) + (7).to_bytes(2, "little")) * 324      # 324 one-byte copies, 3 B of stream each
    st = uvarint(1024) + body
    assert O.snappy_decode(st) is not None
    r, _ = run_slot(walk, st, 1024, lanes=lanes)
    assert r == 2


def test_walk_rejects_what_the_restatement_rejects(walk, lanes):
    rng = random.Random(6)
    good = O.snappy_encode(b"".join(bytes([rng.getrandbits(8)]) * 9 for _ in range(100)))
    cases = [
        good[:-1],                                       # truncated
        uvarint(5) + bytes([0]) + b"a" + bytes([1, 0]),  # copy-1 with offset 0
        uvarint(5) + bytes([0, 1]),                      # short output
        uvarint(8) + bytes([60 << 2]),                   # truncated literal length
        uvarint(4) + bytes([3 << 2]) + b"abc" + bytes([1 << 2 | 1, 9]),   # offset past the output
        uvarint(2) + bytes([2 << 2]) + b"abc",           # literal past dlen
    ]
    walked = 0
    for st in cases:
        with pytest.raises(O.SnappyCorrupt):
            O.snappy_decode(st)
        try:
            dl, _ = O.snappy_decoded_len(st)
        except O.SnappyCorrupt:
            continue                       # rejected by the header pass before any walk
        if dl > 1024:
            continue
        r, _ = run_slot(walk, st, dl, lanes=lanes)
        assert r in (1, 2), st
        walked += 1
    assert walked >= 4


def test_walk_long_literal_length_bytes(walk, lanes):
    """Literal lengths in 1-4 extra bytes (tags 60-63; golang/snappy writes 1-2 of them, any decoder
    must take all four), including 4-byte lengths past the output (rejected), decode as the
    restatement does."""
    body = b"abcdefghijklmnopqrstuvwxyz0123456789"
    cases = []
    for nb in (1, 2, 3, 4):
        n = len(body)
        cases.append(uvarint(n) + bytes([(59 + nb) << 2]) + (n - 1).to_bytes(nb, "little") + body)
    cases.append(uvarint(8) + bytes([63 << 2]) + (0xFFFFFFFF).to_bytes(4, "little") + b"abcdefgh")
    cases.append(uvarint(8) + bytes([63 << 2]) + (1 << 24).to_bytes(4, "little") + b"abcdefgh")
    for st in cases:
        try:
            want = O.snappy_decode(st)
        except O.SnappyCorrupt:
            want = None
        dl, _ = O.snappy_decoded_len(st)
        r, out = run_slot(walk, st, dl, lanes=lanes)
        if want is None:
            assert r in (1, 2), st
        else:
            assert r == 0 and out == want, st
