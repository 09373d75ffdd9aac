"""The shipped library's wave-tile kernels keep their prefetch registers out of the register
allocator's hands (tools/kcheck.py; VERDICT r4 item 6: the PD = 6 k = 8 instance spilled its
prefetch AGPRs to scratch right behind the loads and produced an all-NaN W)."""
import os
import shutil

import pytest

from tools import kcheck

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cnmf_amd", "libcnmf_hip.so")


@pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(os.path.join(kcheck.LLVM, "llvm-objdump"))),
                    reason="library or LLVM tools missing")
def test_shipped_library_prefetch_registers_untouched():
    dis = kcheck.disassemble(LIB)
    ks = [(n, b) for n, b in kcheck.kernels(dis) if kcheck.FAMILIES.search(n)]
    assert len(ks) >= 20  # every wave-tile family is in the product library
    for name, body in ks:
        nreg, bad, big = kcheck.check_kernel(body)
        assert nreg > 0 or "bfw" in name or "als" in name or "mf8" in name, name
        assert not bad and not big, (name, bad[:3], big)


def test_the_pd6_failure_pattern_is_flagged():
    """The round-4 PD = 6 instance: every prefetch load followed by a scratch store of its register."""
    body = ["global_load_dwordx4 a[0:3], v[6:7], off nt",
            "scratch_store_dwordx4 off, a[0:3], off offset:16",
            "s_waitcnt vmcnt(26)",
            "ds_write_b128 v2, a[0:3]"]
    nreg, bad, big = kcheck.check_kernel(body)
    assert nreg == 4 and bad == ["scratch_store_dwordx4 off, a[0:3], off offset:16"] and not big
    # a copy of a prefetch register into a VGPR before its wait is the same hazard
    nreg, bad, _ = kcheck.check_kernel(["global_load_dwordx4 a[8:11], v[6:7], off nt",
                                        "v_accvgpr_read_b32 v5, a9", "s_waitcnt vmcnt(0)"])
    assert bad == ["v_accvgpr_read_b32 v5, a9"]
    # clean: loads, counted waits and the staging stores only
    _, bad, big = kcheck.check_kernel(["global_load_dwordx4 a[8:11], v[6:7], off nt", "s_waitcnt vmcnt(20)",
                                       "ds_write_b128 v2, a[8:11] offset:1024", "v_add_f32 v1, v2, v3"])
    assert not bad and not big
    assert kcheck.check_kernel(["s_waitcnt vmcnt(70)"])[2] == [70]


@pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(os.path.join(kcheck.LLVM, "llvm-readelf"))),
                    reason="library or LLVM tools missing")
def test_shipped_wave_tile_kernels_within_spill_budget():
    """Round 6: the code object's metadata — no wave-tile kernel spills VGPRs past its family's budget
    (0; the constrained ALS's TOL form 2, outside its streaming loop)."""
    sp = kcheck.spills(kcheck.disassemble(LIB))
    fam = {n: kcheck.FAMILIES.search(n).group(1) for n in sp if kcheck.FAMILIES.search(n)}
    assert len(fam) >= 20
    over = {n: sp[n] for n, f in fam.items() if sp[n] > kcheck.SPILL_BUDGET.get(f, 0)}
    assert not over, over


def test_spill_notes_parse():
    text = ("0000 <k>:\n\tv_add_f32 v1, v2, v3\n" + kcheck.NOTES_MARK + "\n"
            "  - .agpr_count:     0\n    .name:           _Z18wmu_iter_wt_kernelX\n    .vgpr_spill_count: 3\n"
            "  - .agpr_count:     4\n    .name:           other\n    .vgpr_spill_count: 0\n")
    assert kcheck.spills(text) == {"_Z18wmu_iter_wt_kernelX": 3, "other": 0}
    assert [n for n, _ in kcheck.kernels(text)] == ["k"]
