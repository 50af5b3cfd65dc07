"""CPU: static audit of the gfx950 ISA of every kernel that uses inline-asm memory operations
(tools/isa_audit.py): no VGPR written by an asm load is touched before a vmcnt wait retires the
load, no compiler instruction uses M0, no spills.  hipcc cross-compiles here (no GPU needed).
The audit also has to find round 1's actual defect in a minimal reproduction, so a passing
audit is evidence, not an analyser that sees nothing."""
import os
import shutil
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_audit  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(isa_audit.HIPCC), reason="hipcc not installed")


@pytest.mark.parametrize("src", ["scorer.hip", "head.hip"])
def test_kernels_have_no_asm_register_hazards(src):
    findings, _ = isa_audit.audit_file(os.path.join(isa_audit.CSRC, src))
    assert not findings, "\n".join(findings[:20])


def test_scorer_audit_tracks_the_stored_p_loads():
    findings, n = isa_audit.audit_file(os.path.join(isa_audit.CSRC, "scorer.hip"), only="score_ddp_kernel")
    assert not findings
    assert n >= 4 * 16  # four instantiations, each with its prologue and per-stage P loads


# Round 1's defect, reduced to its ISA (score_ddp_kernel<32>, scorer.hip at f175cd5): the loop
# latch compares the trip counter in v[80:81], the destination of the asm P load the stage before
# issued, on the path where that load is still in flight (the loop ended after stage t).
_ROUND1_LATCH = """
_Zkernel:
\tglobal_load_dwordx4 v[16:19], v101, s[2:3] offset:0
\ts_waitcnt vmcnt(0)
\ts_branch .LBB0_3
.LBB0_2:
\ts_add_u32 s8, s8, 5
\tv_mov_b64_e32 v[80:81], s[4:5]
\tv_cmp_ge_u64_e32 vcc, s[8:9], v[80:81]
\ts_cbranch_vccnz .LBB0_12
.LBB0_3:
;;#ASMSTART
\tglobal_load_dwordx4 v[80:83], v101, s[28:29] offset:32
;;#ASMEND
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[104:107], v[16:19], v[0:15]
\ts_waitcnt vmcnt(4)
\ts_cbranch_vccnz .LBB0_5
;;#ASMSTART
\ts_waitcnt vmcnt(0)
;;#ASMEND
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[104:107], v[80:83], v[0:15]
.LBB0_5:
\ts_branch .LBB0_2
.LBB0_12:
;;#ASMSTART
\ts_waitcnt vmcnt(0)
;;#ASMEND
\ts_endpgm
.Lfunc_end0:
"""


def test_audit_detects_round1_latch_hazard():
    findings, n = isa_audit.audit_asm_text(_ROUND1_LATCH)
    assert n == 1
    assert any("v_mov_b64_e32 v[80:81]" in f for f in findings), findings
    assert any("v_cmp_ge_u64_e32" in f for f in findings), findings
    # with the latch's compare in a free register the same code is clean
    fixed = _ROUND1_LATCH.replace("v[80:81], s[4:5]", "v[90:91], s[4:5]").replace("s[8:9], v[80:81]", "s[8:9], v[90:91]")
    assert isa_audit.audit_asm_text(fixed)[0] == []
