"""Static in-flight-load hazard check of the built HIP extension (tools/vmcnt_check.py).

The round-2 GPU fault of sepconv_ws ids 9/10 came from inline-asm loads whose
destination registers the compiler re-allocated (as the next load's address) while
the load was still in flight. The checker models the in-order vmcnt queue over every
kernel's control-flow graph; this test requires it to find NO such hazard in any
kernel of kdl/_C, and checks the checker itself on the exact instruction pattern
that faulted. CPU only: it reads the gfx950 code object, it runs nothing.
"""
import importlib.util
import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
spec = importlib.util.spec_from_file_location("vmcnt_check", ROOT / "tools" / "vmcnt_check.py")
vc = importlib.util.module_from_spec(spec)
sys.modules["vmcnt_check"] = vc          # dataclasses resolve their module by name
spec.loader.exec_module(vc)


def _kernel(lines):
    k = vc.Kernel("k")
    for i, (op, args) in enumerate(lines):
        addr = 0x1000 + 8 * i
        k.insns.append(vc.Insn(addr, op, " " + args, f"{op} {args} // {addr:012X}: 00"))
    return k


def test_checker_flags_the_round2_fault_pattern():
    # global_load_dwordx4 v[4:7] is in flight while v[6:7] is recomputed and used as the
    # next load's address (sepconv_ws ABL=2 prologue, round 2)
    k = _kernel([("global_load_dwordx4", "v[4:7], v[4:5], off"),
                 ("v_lshl_add_u64", "v[6:7], v[58:59], 0, s[8:9]"),
                 ("global_load_dwordx4", "v[12:15], v[6:7], off"),
                 ("s_waitcnt", "vmcnt(0)"),
                 ("s_endpgm", "")])
    hz = vc.check_kernel(k, {"k": 0x1000})
    assert len(hz) == 2 and "v6,v7" in hz[0]


def test_checker_accepts_counted_waits_and_in_order_waw():
    k = _kernel([("global_load_dwordx4", "v[0:3], v[40:41], off"),
                 ("global_load_dwordx4", "v[4:7], v[42:43], off"),
                 ("global_load_dwordx4", "v[4:7], v[44:45], off"),     # WAW: loads return in order
                 ("s_waitcnt", "vmcnt(2)"),                            # retires the first load only
                 ("v_mfma_f32_16x16x32_bf16", "a[0:3], v[0:3], v[8:11], a[0:3]"),
                 ("s_waitcnt", "vmcnt(0)"),
                 ("v_mov_b32_e32", "v4, 0"),
                 ("s_endpgm", "")])
    assert vc.check_kernel(k, {"k": 0x1000}) == []
    # ... but one wait too few leaves v[4:7] pending at the mov
    k.insns[5] = vc.Insn(k.insns[5].addr, "s_waitcnt", " vmcnt(1)", "s_waitcnt vmcnt(1) // 0")
    assert len(vc.check_kernel(k, {"k": 0x1000})) == 1


def test_checker_follows_loop_back_edges():
    # a load issued at the bottom of a loop body is still pending at the top of the next trip
    k = _kernel([("s_mov_b32", "s0, 4"),
                 ("v_add_u32_e32", "v1, v2, v3"),                       # loop head: touches v1
                 ("global_load_dword", "v1, v[8:9], off"),
                 ("s_sub_u32", "s0, s0, 1"),
                 ("s_cbranch_scc1", "-4 <k+0x8>"),
                 ("s_waitcnt", "vmcnt(0)"),
                 ("s_endpgm", "")])
    hz = vc.check_kernel(k, {"k": 0x1000})
    assert len(hz) == 1 and "v_add_u32" in hz[0]


def test_built_extension_has_no_inflight_register_hazards():
    so = next((ROOT / "kdl").glob("_C*.so"), None)
    if so is None or not shutil.which(str(vc.LLVM / "llvm-objdump")):
        pytest.skip("kdl/_C not built or ROCm llvm tools missing")
    n, hz = vc.check(so)
    assert n > 300, f"only {n} kernels disassembled"
    assert not hz, "\n".join(hz[:20])
