"""CPU check of the snappy tag walk and its op replay (bhg_snappy_parse.h,
used by k_snappy_front and k_snappy_mat): the product header is compiled for
the host with clang, a harness stages a stream the way the front pass does
(at an arbitrary 16-B arena offset), walks it into 16-byte copy ops, then
replays the ops as the materialiser does (16-B reads from the stream or the
output, 20-B writes at the cursor, in program order).  Every result must be the restated golang/snappy decode
(oracle, pinned by pyarrow interop in test_oracle_snappy.py), SNAPPY_CORRUPT
exactly where the restatement rejects, or a hand-over to the global-memory
pass -- never wrong bytes.  No GPU involved; the GPU run of the same code is
tests/test_gpu_decode.py."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "bitalosdb_amd", "csrc", "bhg_snappy_parse.h")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"

HARNESS = r"""
#include <stdint.h>
#include <string.h>
#include <vector>
%s
using namespace bhg;
// 0 ok (out holds dlen bytes), 1 corrupt, 3 hand over (op cap)
extern "C" int walk_replay(const uint8_t *stream, uint32_t clen, uint32_t hdr, uint32_t dlen, uint32_t arena_off,
                           uint8_t *out, uint32_t *nops_out) {
    std::vector<uint8_t> arena_v(arena_off + clen + 64 + 32, 0xA5);
    uint8_t *arena = arena_v.data() + (16 - ((uintptr_t)arena_v.data() & 15));
    memcpy(arena + arena_off, stream, clen);
    std::vector<uint32_t> ops(kSnapOpCap + 8, 0xdead);
    SnapParse S;
    S.s = arena_off + hdr; S.se = arena_off + clen; S.sb = arena_off;
    S.d = 0; S.dlen = dlen; S.nops = 0; S.res = 0;
    S.t8 = snap_ld8(arena, S.s);
    if (S.s < S.se)
        while (snap_parse_step(arena, S, [&](uint32_t q, uint32_t op, bool on) { if (on && q < kSnapOpCap) ops[q] = op; })) {}
    const uint32_t r = S.res ? S.res : (S.d == S.dlen ? 0u : 1u);
    *nops_out = S.nops;
    if (r) return (int)r;
    if (S.nops > kSnapOpCap) return 3;
    // replay as k_snappy_mat does: 16-B reads from the stream (literal) or the output (copy), 20-B writes
    std::vector<uint8_t> outb(kSnapMaxOut + 64, 0x5A), strm(clen + 32, 0);
    memcpy(strm.data(), stream, clen);
    uint32_t d = 0;
    for (uint32_t k = 0; k < S.nops; k++) {
        const uint32_t op = ops[k], src = op & 0x7ffu, len = ((op >> 11) & 15u) + 1u, lit = op >> 15;
        uint8_t t[20];
        memcpy(t, (lit ? strm.data() : outb.data()) + src, 16);
        memset(t + 16, 0xEE, 4);
        memcpy(outb.data() + d, t, 20);
        d += len;
    }
    if (d != dlen) return 9;
    memcpy(out, outb.data(), dlen);
    return 0;
}
"""


@pytest.fixture(scope="module")
def walk(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("no clang++")
    body = open(HDR).read().replace("__device__ __forceinline__ ", "static inline ")
    d = tmp_path_factory.mktemp("walk")
    cpp, so = d / "walk.cpp", d / "walk.so"
    cpp.write_text(HARNESS % body)
    subprocess.check_call([CLANG, "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(so), str(cpp)])
    lib = ctypes.CDLL(str(so))
    lib.walk_replay.restype = ctypes.c_int
    lib.walk_replay.argtypes = [ctypes.c_char_p] + [ctypes.c_uint32] * 4 + [ctypes.c_void_p, ctypes.c_void_p]
    return lib


def run(walk, stream, arena_off=37):
    dlen, hdr = O.snappy_decoded_len(stream)
    out = np.zeros(max(dlen, 1), dtype=np.uint8)
    nops = ctypes.c_uint32()
    r = walk.walk_replay(stream, len(stream), hdr, dlen, arena_off, out.ctypes.data, ctypes.byref(nops))
    return r, out[:dlen].tobytes(), nops.value


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
        kind = i % 6
        if kind == 0:
            yield bytes(rng.getrandbits(8) for _ in range(n))              # literals only
        elif kind == 1:
            yield bytes(rng.choice(b"ab") for _ in range(n))              # short-offset copies
        elif kind == 2:
            yield (b"0123456789abcdefXYZ" * 60)[:n]                       # period 19
        elif kind == 3:
            p = rng.randrange(1, 16)                                      # every short period
            unit = bytes(rng.getrandbits(8) for _ in range(p))
            yield (unit * (n // p + 1))[:n]
        else:                                                             # 16-B words, the C3 shape
            words = [bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(8)]
            yield b"".join(rng.choice(words) if rng.random() > 0.25 else
                           bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(64))[:n]


def test_walk_replay_matches_restated_decode(walk):
    rng = random.Random(5)
    codes = {0: 0, 1: 0, 3: 0}
    for j, v in enumerate(values(rng, 2400)):
        st = O.snappy_encode(v)
        if len(st) > 2047 or len(v) > 1024:
            continue                       # not eligible: the front pass sends it to k_snappy_rt
        r, out, nops = run(walk, st, arena_off=16 * (j % 50))
        codes[r] += 1
        assert r in (0, 3), (r, v[:32])
        if r == 0:
            assert out == v
            assert nops >= (len(v) + 15) // 16
    assert codes[0] > 1900


def test_short_period_ops_double(walk):
    """A run with period 1 (16 copies of 64 B, offset 1): ops of 1, 2, 4, 8, then 16 bytes per
    copy -- 8 per copy, not 64."""
    v = b"x" * 1024
    st = O.snappy_encode(v)
    r, out, nops = run(walk, st)
    assert r == 0 and out == v
    assert nops <= 16 * 8 + 1


def test_walk_takes_streams_that_outrun_their_input(walk):
    """700 B of RLE copies first, then 324 one-byte copies (3 stream bytes each):
    the output outgrows the stream -- no in-place constraint any more (the
    materialiser keeps only the output in LDS), so the op path takes it."""
    body = bytes([0]) + b"x"
    body += (bytes([(64 - 1) << 2 | 2]) + (1).to_bytes(2, "little")) * 10
    body += bytes([(59 - 1) << 2 | 2]) + (1).to_bytes(2, "little")
    body += (bytes([2]) + (7).to_bytes(2, "little")) * 324      # 324 one-byte copies, 3 B of stream each
    st = uvarint(1024) + body
    want = O.snappy_decode(st)
    r, out, nops = run(walk, st)
    assert (r == 0 and out == want) or r == 3


def test_walk_rejects_what_the_restatement_rejects(walk):
    rng = random.Random(6)
    good = O.snappy_encode(b"".join(bytes([rng.getrandbits(8)]) * 9 for _ in range(100)))
    cases = [
        good[:-1],                                       # truncated
        uvarint(5) + bytes([0]) + b"a" + bytes([1, 0]),  # copy-1 with offset 0
        uvarint(5) + bytes([0, 1]),                      # short output
        uvarint(8) + bytes([60 << 2]),                   # truncated literal length
        uvarint(4) + bytes([3 << 2]) + b"abc" + bytes([1 << 2 | 1, 9]),   # offset past the output
        uvarint(2) + bytes([2 << 2]) + b"abc",           # literal past dlen
        uvarint(70) + bytes([0]) + b"a" + bytes([(64 - 1) << 2 | 2, 1, 0]) + bytes([1 << 2 | 1, 200]),  # offset > d
    ]
    walked = 0
    for st in cases:
        with pytest.raises(O.SnappyCorrupt):
            O.snappy_decode(st)
        try:
            dl, _ = O.snappy_decoded_len(st)
        except O.SnappyCorrupt:
            continue                       # rejected by decodedLen before any walk
        if dl > 1024:
            continue
        r, _, _ = run(walk, st)
        assert r == 1, st
        walked += 1
    assert walked >= 5
