"""CPU-side checks of the C-ABI library: it builds, loads, and exports every
symbol include/bithashgpu.h declares (no compute calls without a GPU)."""
import os
import re
import subprocess

import pytest

from bitalosdb_amd import _lib as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "bithashgpu.h")).read()
    return sorted(set(re.findall(r"\b(bhg_[a-z0-9_]+)\s*\(", txt)))


def test_library_builds_and_loads():
    B.build()
    assert os.path.exists(B.LIB_PATH)
    L = B.lib()
    assert L.bhg_abi_version() == B.ABI_VERSION == 3


def test_exports_match_header():
    B.build()
    syms = header_symbols()
    assert set(syms) == set(B.EXPORTS)
    out = subprocess.check_output(["nm", "-D", "--defined-only", B.LIB_PATH]).decode()
    exported = set(re.findall(r"\bT (bhg_[a-z0-9_]+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_no_torch_types_in_header():
    txt = open(os.path.join(ROOT, "include", "bithashgpu.h")).read()
    code = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)       # declarations only, comments stripped
    code = re.sub(r"//[^\n]*", "", code)
    for bad in ("torch", "at::", "hipStream_t", "Tensor", "#include <hip"):
        assert bad not in code


def test_struct_layouts():
    assert B.HANDLE_DT.itemsize == 16
    assert B.DESC_DT.itemsize == 40
    assert B.DESC_DT.fields["trailer"][1] == 16
    assert B.DESC_DT.fields["status"][1] == 36


def test_scan_scratch_is_bounded():
    """the table scan's scratch was ~0.9 MiB per table with no cap.  Tables are now
    scanned 256 at a time through one scratch area: the size stops growing at 256 tables."""
    L = B.lib()
    s1, s256, s10k = (L.bhg_scan_scratch_bytes(n) for n in (1, 256, 10000))
    assert s1 < (2 << 20)
    assert s256 < (256 << 20)
    assert s10k - s256 < (1 << 20)  # only the u64 scan's per-table words still grow


def test_no_device_means_no_context():
    # this container has no GPU: the library must refuse, not fall back to a CPU path
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = B.lib()
    assert L.bhg_device_count() == 0
    assert not L.bhg_create(0, 0)


def test_no_selectable_kernel_variants():
    """The shipped library has one kernel per job: no environment switch can
    select an exploration or diagnostic kernel (those live in scripts/lab)."""
    B.build()
    blob = open(B.LIB_PATH, "rb").read()
    for env in (b"BHG_DECODE_VARIANT", b"BHG_SNAPPY_VARIANT", b"BHG_LANE_WGS_PER_CU", b"BHG_HOST_NOPIPE"):
        assert env not in blob, env
    syms = subprocess.check_output(["nm", "-C", B.LIB_PATH]).decode()
    for k in ("k_diag", "k_decode_lane", "k_decode_coop", "k_decode_lanebuf", "k_snappy_wave", "k_decode_tile2"):
        assert k not in syms, k
    assert not re.search(rb"BHG_[A-Z_]*VARIANT", blob)


def _src_default(fname, knob):
    src = open(os.path.join(os.path.dirname(B.LIB_PATH), "..", "csrc", fname)).read()
    m = re.search(r"constexpr (?:int|uint32_t) %s = (\d+);" % knob, src)
    assert m, (fname, knob)
    return int(m.group(1))


def test_shipped_library_has_default_knobs():
    """The .so holds exactly the kernel instantiations the sources' tuning constants select
    (no compile-time knobs remain; a stale or lab-built object would ship a different one)."""
    B.build()
    blob = open(B.LIB_PATH, "rb").read()
    pf = _src_default("bhg_decode_tile.hip", "kTilePf")
    nch = _src_default("bhg_decode_tile.hip", "kTileNch")
    bpw = _src_default("bhg_snappy_dec.hip", "kSlBpw")
    slot = _src_default("bhg_snappy_dec.hip", "kSlSlot")
    want = {  # <WPB, NCH, PF, NB = 2, LONG>: the C2 kernel and its long-record-batch twin
        rb"_ZN3bhg13k_decode_tileI": {b"_ZN3bhg13k_decode_tileILi8ELi%dELi%dELi2ELi%dEE" % (nch, pf, lg)
                                      for lg in (0, 1)},
    }
    # the snappy LDS tiers: tier 1 in batch order, and one multi-role launch for the lists, with
    # kG1 / kG2 lanes per block
    g1 = _src_default("bhg_snappy_dec.hip", "kG1")
    g2 = _src_default("bhg_snappy_dec.hip", "kG2")
    nat = set(re.findall(rb"_ZN3bhg16k_snappy_lds_natI[A-Za-z0-9]+?EE", blob))
    multi = set(re.findall(rb"_ZN3bhg18k_snappy_lds_multiI[A-Za-z0-9]+?EE", blob))
    assert nat == {b"_ZN3bhg16k_snappy_lds_natILi%dEE" % g1}, nat
    assert multi == {b"_ZN3bhg18k_snappy_lds_multiILi%dELi%dEE" % (g1, g2)}, multi
    assert not re.search(rb"_ZN3bhg12k_snappy_ldsI", blob)
    assert _src_default("bhg_snappy_dec.hip", "kSlBpw") == 18 and slot == 1088
    for prefix, names in want.items():
        found = set(re.findall(re.escape(prefix) + rb"[A-Za-z0-9]+?EE", blob))
        assert found == names, (prefix, found, names)
    enc = set(re.findall(rb"_ZN3bhg12k_snappy_encI[A-Za-z0-9]+?EE", blob))
    assert enc == {b"_ZN3bhg12k_snappy_encILi2048ELi1ELi4EE", b"_ZN3bhg12k_snappy_encILi4096ELi3ELi3EE"}, enc
