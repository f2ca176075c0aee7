"""The C-ABI from a plain-C host program (tests/c_client/abi_client.c, built by
__graft_entry__.build() with gcc against include/bithashgpu.h and libbithashgpu.so only):
the calling pattern of the cgo binding in INTEGRATION.md, without Python or torch in the
process.  The program checks device and host-path decode, encode and the long-range
checksum against the C restatement (oracle/, the checker)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLIENT = os.path.join(ROOT, "tests", "c_client", "abi_client")


def _run(timeout):
    if not os.path.exists(CLIENT):
        pytest.fail("tests/c_client/abi_client is not built (run __graft_entry__.build())")
    return subprocess.run([CLIENT], capture_output=True, text=True, timeout=timeout)


def test_c_client_without_gpu_reports_no_context():
    """No GPU: bhg_create fails, the program says so and exits 2 (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = _run(60)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "no device context" in r.stderr


@pytest.mark.gpu
def test_c_client_on_gpu():
    r = _run(240)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "abi_client ok" in r.stdout
    assert "decode codec 1" in r.stdout and "encode:" in r.stdout and "crc_long" in r.stdout
