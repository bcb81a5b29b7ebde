"""The gfx950 store-data hazard checked on the SHIPPED library, not remembered.

Round 4 found torn drained values: a `buffer_store_dwordx4`'s data VGPR rewritten two wait states
after issue (the wait the compiler inserts on gfx940+), before the store had read it. Every drain of
the library keeps its store data live until the next barrier (`keep_vgprs`), waits for its stores
(`store_fence`) or holds the data through 16 wait states in one asm statement (`store_guard*`).
tools/store_hazard.py disassembles the gfx950 code object inside libfemasm.so and finds every
12/16-byte vector store whose data VGPRs an instruction writes within 16 wait states with no
`s_waitcnt vmcnt(0)` / `s_barrier` in between; compiler spill stores, rocPRIM's kernels and the
HBM probe kernels are reported but exempt (see the tool's header). Runs in the CPU suite and, as
the same check of the library the GPU tests load, in the GPU suite."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import store_hazard as SH  # noqa: E402

SO = os.path.join(ROOT, "fem-libraries_amd", "femasm", "lib", "libfemasm.so")


def _need_tools():
    if not os.path.exists(SO):
        pytest.skip("libfemasm.so not built (run __graft_entry__.build())")
    if not os.path.exists(os.path.join(SH.LLVM, "llvm-objdump")) or shutil.which("c++filt") is None:
        pytest.skip("ROCm llvm tools missing")


FAKE = """
0000000000001000 <_Z5k_badv>:
\tbuffer_store_dwordx4 v[96:99], v105, s[40:43], 0 offen nt  // 000000001000: 0
\ts_nop 1  // 0
\tv_add_u32_e32 v97, 8, v105  // 0
\ts_endpgm  // 0
0000000000002000 <_Z6k_goodv>:
\tglobal_store_dwordx4 v[2:3], v[4:7], off nt  // 0
\ts_nop 7  // 0
\ts_nop 7  // 0
\tv_mov_b32_e32 v4, 0  // 0
\tglobal_store_dwordx4 v[2:3], v[8:11], off  // 0
\ts_waitcnt vmcnt(0)  // 0
\tv_mov_b32_e32 v8, 0  // 0
\tglobal_store_dwordx4 v[2:3], v[12:15], off  // 0
\tds_write_b64 v12, v[20:21]  // 0
\tglobal_load_dwordx2 v[30:31], v[2:3], off  // 0
\ts_endpgm  // 0
0000000000003000 <_Z6k_fillv>:
\tglobal_store_dwordx3 v[2:3], v[4:6], off  // 0
\tds_read_b64 v[5:6], v1  // 0
\ts_endpgm  // 0
"""


# control flow (addresses as llvm-objdump prints them): a writer behind a TAKEN branch is a site; a
# writer past an unconditional branch (never executed next) is not; a loop's back edge brings the loop
# head's writers after a store at the bottom of the loop
FAKE_CF = """
0000000000001000 <_Z6k_takenv>:
\tbuffer_store_dwordx4 v[10:13], v1, s[4:7], 0 offen  // 000000001000: E07C0000 80010A01
\ts_cbranch_scc1 2  // 000000001008: BF850002
\tv_mov_b32_e32 v40, 0  // 00000000100C: 7E500280
\ts_endpgm  // 000000001010: BF810000
\tv_mov_b32_e32 v41, 0  // 000000001014: 7E520280
\tv_mov_b32_e32 v11, 0  // 000000001018: 7E160280
\ts_endpgm  // 00000000101C: BF810000
0000000000002000 <_Z7k_skipsv>:
\tbuffer_store_dwordx4 v[10:13], v1, s[4:7], 0 offen  // 000000002000: E07C0000 80010A01
\ts_branch 1  // 000000002008: BF820001
\tv_mov_b32_e32 v12, 0  // 00000000200C: 7E180280
\ts_nop 7  // 000000002010: BF800007
\ts_nop 7  // 000000002014: BF800007
\tv_mov_b32_e32 v12, 0  // 000000002018: 7E180280
\ts_endpgm  // 00000000201C: BF810000
0000000000003000 <_Z6k_loopv>:
\tv_mov_b32_e32 v20, 0  // 000000003000: 7E280280
\tv_add_u32_e32 v1, 16, v1  // 000000003004: 68020290
\tbuffer_store_dwordx4 v[20:23], v1, s[4:7], 0 offen  // 000000003008: E07C0000 80011401
\ts_cbranch_vccnz 65531  // 000000003010: BF87FFFB
\ts_endpgm  // 000000003014: BF810000
"""


def test_checker_follows_branches():
    sites = {s[0]: s for s in SH.check(FAKE_CF)}
    assert "_Z6k_takenv" in sites and sites["_Z6k_takenv"][2].startswith("v_mov_b32_e32 v11")
    assert sites["_Z6k_takenv"][3] == 3  # branch (1), v41 (2), v11 (3) on the taken path
    assert "_Z7k_skipsv" not in sites  # the first v12 write is jumped over; the second is 16 wait states on
    assert "_Z6k_loopv" in sites and sites["_Z6k_loopv"][2].startswith("v_mov_b32_e32 v20")


def test_checker_finds_known_patterns():
    """The checker itself: a write 3 wait states after the store is a site; 16 wait states of
    s_nop, a vmcnt(0) wait, an LDS write's address operand and an unrelated load are not; an LDS
    read INTO the data registers is."""
    sites = SH.check(FAKE)
    fns = [s[0] for s in sites]
    assert fns.count("_Z5k_badv") == 1 and sites[0][3] == 3
    assert "_Z6k_goodv" not in fns
    assert fns.count("_Z6k_fillv") == 1


def test_shipped_library_has_no_store_data_hazard():
    _need_tools()
    text = SH.disassemble(SO)
    assert "k_gather_lin" in text and "k_gather_neo" in text, "the hot kernels are in the checked code object"
    bad = [s for s in SH.check(text) if not SH.exempt(s[0], s[1])]
    names = SH.demangle([s[0] for s in bad]) if bad else []
    assert not bad, "store-data hazard sites:\n" + "\n".join(f"{n[:100]}: {s[1]} / {s[2]} at {s[3]}"
                                                             for s, n in zip(bad, names))


@pytest.mark.gpu
def test_shipped_library_has_no_store_data_hazard_gpu_suite():
    """The same check in the GPU suite: the library the GPU tests load."""
    test_shipped_library_has_no_store_data_hazard()
