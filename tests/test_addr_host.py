"""CPU check of the wave-uniform 64-bit address helpers (readlane_u64 /
readfirstlane_u64 in bitalosdb_amd/csrc/bhg_device.h) that every kernel uses
to broadcast a block's stream / output address from its lane.

The functions are extracted from the product header and compiled for the host
with clang, with the two builtins replaced by host stand-ins that return `int`
exactly as the gfx950 builtins do.  An address whose low word has bit 31 set
must come back unchanged (round 2's fault: the int sign-extended into the high
word).  The GPU side of the same case is
tests/test_gpu_decode.py::test_snappy_addresses_with_bit31_set."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "bitalosdb_amd", "csrc", "bhg_device.h")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.fixture(scope="module")
def helpers(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("no clang++")
    s = open(HDR).read()
    i0 = s.index("__device__ __forceinline__ uint64_t readlane_u64(")
    i1 = s.index("// Wave-wide inclusive scans through DPP")
    body = s[i0:i1].replace("__device__ __forceinline__ ", 'extern "C" ')
    # every lane holds the same value, so lane l's register is the argument itself; the
    # stand-ins return it as `int`, as the gfx950 builtins do
    pre = ("#include <stdint.h>\n"
           "static int host_readlane(int v, int l) { (void)l; return v; }\n"
           "static int host_readfirstlane(int v) { return v; }\n"
           "#define __builtin_amdgcn_readlane(v, l) host_readlane((v), (l))\n"
           "#define __builtin_amdgcn_readfirstlane(v) host_readfirstlane((v))\n")
    d = tmp_path_factory.mktemp("addr")
    cpp, so = d / "addr.cpp", d / "addr.so"
    cpp.write_text(pre + body)
    subprocess.check_call([CLANG, "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(so), str(cpp)])
    lib = ctypes.CDLL(str(so))
    lib.readlane_u64.restype = ctypes.c_uint64
    lib.readlane_u64.argtypes = [ctypes.c_uint64, ctypes.c_int]
    lib.readfirstlane_u64.restype = ctypes.c_uint64
    lib.readfirstlane_u64.argtypes = [ctypes.c_uint64]
    return lib


@pytest.mark.parametrize("addr", [0x7F00_8000_0000, 0x7F00_FFFF_FFF0, 0x7F00_7FFF_FFFF, 0x8000_0000,
                                  0xFFFF_FFFF_FFFF_FFFF, 0x1_8000_0010, 0x8000_0000_8000_0000, 0])
def test_readlane_u64_keeps_bit31(helpers, addr):
    assert helpers.readlane_u64(addr, 17) == addr
    assert helpers.readfirstlane_u64(addr) == addr


def test_naive_composition_would_sign_extend():
    """What the helpers prevent: (uint64_t)(int)lo | (uint64_t)hi << 32 with bit 31 of lo set."""
    lo, hi = 0x8000_0010, 0x7F00
    naive = ((lo - (1 << 32)) & 0xFFFF_FFFF_FFFF_FFFF) | (hi << 32)
    assert naive != (hi << 32 | lo)
