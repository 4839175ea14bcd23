"""CPU tier: no inline-asm block in any gfx950 kernel reads a VGPR an MFMA wrote too
few wait states earlier (the hazard recognizer cannot see into inline asm; the
hardware does not interlock).  Root cause of round 2's stem_fwd_kernel NaN at
__launch_bounds__(256, 2) — see scripts/check_mfma_asm_hazards.py."""
import glob
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not available")
@pytest.mark.parametrize("src", sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip"))
                                       + glob.glob(os.path.join(ROOT, "csrc", "comm", "*.hip"))),
                         ids=os.path.basename)
def test_no_inline_asm_reads_fresh_mfma_results(src):
    import check_mfma_asm_hazards as H
    probs = H.check_file(src)
    assert not probs, probs[:5]


def test_checker_flags_the_round2_stem_pattern():
    """The checker itself: an inline-asm read right after an MFMA into VGPRs is flagged."""
    import check_mfma_asm_hazards as H
    asm = "\n".join([
        "k:",
        "\tv_mfma_f32_16x16x32_bf16 v[16:19], v[0:3], v[4:7], v[16:19]",
        "\t;;#ASMSTART",
        "\tv_cvt_pk_bf16_f32 v20, v16, v17",
        "\t;;#ASMEND",
        "\ts_nop 7",
        "\ts_nop 3",
        "\t;;#ASMSTART",
        "\tv_cvt_pk_bf16_f32 v21, v18, v19",
        "\t;;#ASMEND",
    ])
    probs = H.scan_asm(asm)
    assert {p[3] for p in probs} == {16, 17}
