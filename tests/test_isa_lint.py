"""The codegen guard of the device ExtendLoopFast (DESIGN.md "A compiler fault
found on the way"): ROCm 7.2 once emitted a vector store whose address
registers overlapped its data in k_pass_fill<PlanPass> (elf_device.inc), and
the source pins the loaded values with an empty asm barrier.  This compiles
every HIP source to gfx950 assembly (hipcc cross-compiles without a GPU) and
fails if any vector store's address and data registers overlap again, so a
rebuild that brings the pattern back fails the CPU suite."""
import os
import shutil
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not on PATH")
def test_no_address_data_overlapping_store():
    import isa_store_lint
    res = isa_store_lint.lint_all(jobs=min(8, os.cpu_count() or 1))
    assert "block_build.hip" in res and "similar_aligner.hip" in res  # (elf_device.inc is in block_build)
    bad = {k: v for k, v in res.items() if v}
    assert not bad, "vector stores with address registers overlapping their data: %r" % bad
