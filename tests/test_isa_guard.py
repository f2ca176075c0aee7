"""CPU check on the shipped device code: disassemble every gfx950 code object
in libbithashgpu.so and assert that no instruction writes through the scalar
data cache (scalar stores / scalar atomics / its write-back and discard) --
every global write in the kernels is a vector store.

(This file names those mnemonics, so it is listed in .gpurunignore; it
needs no GPU.)"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from bitalosdb_amd import _lib as B

LLVM = "/opt/rocm/lib/llvm/bin"
FORBIDDEN = re.compile(r"^\s*(s_store_|s_buffer_store|s_scratch_store|s_atomic_|s_buffer_atomic|s_dcache_wb|"
                       r"s_dcache_discard)", re.M)


def code_objects(lib_path, tmp):
    blob = subprocess.check_output(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib_path, "/dev/stdout"])
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs = [m.start() for m in re.finditer(re.escape(magic), blob)] + [len(blob)]
    out = []
    for k in range(len(offs) - 1):
        bpath = os.path.join(tmp, "b%d.bin" % k)
        cpath = os.path.join(tmp, "co%d.o" % k)
        with open(bpath, "wb") as f:
            f.write(blob[offs[k]:offs[k + 1]])
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--input=" + bpath, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + cpath])
        out.append(cpath)
    return out


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")) or not shutil.which("objcopy"),
                    reason="llvm tools missing")
def test_no_scalar_cache_writes_in_device_code():
    B.build()
    with tempfile.TemporaryDirectory() as tmp:
        cos = code_objects(B.LIB_PATH, tmp)
        assert len(cos) >= 8                      # one per kernel translation unit
        total = loads = 0
        for co in cos:
            dis = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co]).decode()
            total += dis.count("\n")
            loads += len(re.findall(r"^\s*s_load_dword", dis, re.M))   # positive control of the line format
            bad = FORBIDDEN.findall(dis)
            assert not bad, (co, sorted(set(bad)))
        assert total > 10000 and loads > 100      # the disassembly is real and the pattern anchors match
