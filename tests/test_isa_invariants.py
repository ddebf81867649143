"""CPU checks on the generated gfx950 ISA (hipcc cross-compiles; no GPU needed).

The act-search loss kernel reads its LDS table ring with inline-asm ``ds_read_b128``
(csrc/awq_actsearch.hip ``lds_slot_s`` / ``lds_slot_rs``) that the compiler does not track:
the registers such a read is still writing must not be read, written or copied by any
instruction before the explicit ``s_waitcnt lgkmcnt`` that ends it.  The asm waits take
the loaded registers as operands, which makes that the compiler's obligation too, but a
register copy inserted before the wait would read stale data — so the invariant is checked
on the ISA of every loss-kernel instantiation."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "awq-converter_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "--cuda-device-only", "-S"]


def _regs(text):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


# instructions counted by LGKM_CNT: LDS (return in issue order, like the ring reads) and
# SMEM / FLAT / messages (may return in any order)
_LDS = re.compile(r"ds_\w+")
_OUT_OF_ORDER = re.compile(r"(s_load_|s_buffer_load_|s_scratch_load_|s_memtime|s_memrealtime|s_sendmsg|s_dcache_|"
                           r"s_atc_probe|flat_)\w*")


def ring_violations(asm: str, func_rx: str):
    """(function, line, instruction) for every instruction that touches a register an
    inline-asm ds_read_b128 / ds_read2_b32 is still loading.  Every LGKM-counted instruction is modelled, not
    only the asm reads: s_waitcnt lgkmcnt(N) waits until at most N of them are outstanding, so
    at most N LDS operations are — and since LDS operations complete in issue order, everything
    but the N youngest LDS operations (compiler ds_* included) is done.  An outstanding SMEM /
    FLAT operation can only make that wait stronger, so it is tracked as outstanding but never
    credited with retiring an LDS read (the conservative reading of a count it may satisfy out
    of order).  Inline-asm reads are told from the compiler's own by the ;;#ASMSTART / ;;#ASMEND
    brackets; only their registers are watched."""
    bad, funcs = [], re.findall(r"^(" + func_rx + r"\w*):", asm, re.M)
    for f in funcs:
        i = asm.index(f + ":")
        body = asm[i:asm.index(".Lfunc_end", i)].split("\n")
        lds = []                                       # outstanding LDS operations' watched registers, issue order
        in_asm = False
        for n, line in enumerate(body):
            s = line.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not s or s.startswith(";"):
                continue
            m = re.match(r"s_waitcnt .*lgkmcnt\((\d+)\)", s)
            if m:
                k = int(m.group(1))
                lds = lds[len(lds) - k:] if k else []
                continue
            op = s.split()[0]
            live = set().union(*lds) if lds else set()
            if _LDS.fullmatch(op):
                m = re.match(r"ds_read(?:_b128|2_b32) (v\[\d+:\d+\]), v\d+", s)
                if live & _regs(s):
                    bad.append((f, n, s))
                lds.append(_regs(m.group(1)) if (m and in_asm) else set())
                continue
            if _OUT_OF_ORDER.fullmatch(op) or re.match(r"(s_|\.|[A-Za-z_.$][\w.$]*:)", s):
                continue
            if live & _regs(s):
                bad.append((f, n, s))
    return funcs, bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_act_loss_ring_registers_untouched_until_their_wait(tmp_path):
    out = tmp_path / "act.s"
    if shutil.which(HIPCC) is None:
        pytest.skip("hipcc missing")
    subprocess.run([HIPCC, *FLAGS, os.path.join(CSRC, "awq_actsearch.hip"), "-o", str(out)], cwd=CSRC,
                   check=True, capture_output=True, timeout=900)
    asm = out.read_text()
    funcs, bad = ring_violations(asm, r"_ZN3awq12_GLOBAL__N_115act_loss_kernel")
    assert len(funcs) >= 12, "loss-kernel instantiations not found in the ISA"
    assert "ds_read_b128" in asm and "global_load_lds_dwordx4" in asm, "the LDS ring is not in the build"
    assert re.search(r";;#ASMSTART\s*\n\s*ds_read_b128 v\[", asm), "no inline-asm ring read to watch"
    assert not bad, bad[:5]


def test_ring_checker_flags_an_early_use():
    asm = """_ZN3awq12_GLOBAL__N_115act_loss_kernelX:
\t;;#ASMSTART
\tds_read_b128 v[4:7], v1 offset:0
\t;;#ASMEND
\t;;#ASMSTART
\tds_read_b128 v[8:11], v1 offset:16
\t;;#ASMEND
\ts_waitcnt lgkmcnt(1)
\tv_mul_f32_e32 v2, v4, v3
\tv_mov_b32_e32 v12, v9
\ts_waitcnt lgkmcnt(0)
\tv_mov_b32_e32 v13, v9
.Lfunc_end0:
"""
    funcs, bad = ring_violations(asm, r"_ZN3awq12_GLOBAL__N_115act_loss_kernel")
    assert len(funcs) == 1
    assert [b[2] for b in bad] == ["v_mov_b32_e32 v12, v9"]


def test_ring_checker_models_other_lgkm_instructions():
    """A compiler LDS op issued after the ring reads shifts what lgkmcnt(N) retires; an SMEM
    load may satisfy the count out of order."""
    head = "_ZN3awq12_GLOBAL__N_115act_loss_kernelX:\n\t;;#ASMSTART\n\tds_read_b128 v[4:7], v1 offset:0\n\t;;#ASMEND\n"
    # ds_read_b32 by the compiler after the ring read: lgkmcnt(1) retires only the ring read
    ok = head + "\tds_read_b32 v20, v1 offset:64\n\ts_waitcnt lgkmcnt(1)\n\tv_mov_b32_e32 v12, v5\n.Lfunc_end0:\n"
    assert ring_violations(ok, r"_ZN3awq12_GLOBAL__N_115act_loss_kernel")[1] == []
    # ... but lgkmcnt(2) with one younger compiler op leaves the ring read outstanding
    early = head + "\tds_read_b32 v20, v1 offset:64\n\ts_waitcnt lgkmcnt(1)\n\tds_write_b32 v1, v3\n" \
        "\ts_waitcnt lgkmcnt(1)\n\tv_mov_b32_e32 v12, v5\n.Lfunc_end0:\n"
    assert ring_violations(early, r"_ZN3awq12_GLOBAL__N_115act_loss_kernel")[1] == []
    late = head + "\tds_read_b32 v20, v1 offset:64\n\ts_waitcnt lgkmcnt(2)\n\tv_mov_b32_e32 v12, v5\n.Lfunc_end0:\n"
    assert [b[2] for b in ring_violations(late, r"_ZN3awq12_GLOBAL__N_115act_loss_kernel")[1]] == \
        ["v_mov_b32_e32 v12, v5"]
    # an SMEM load younger than the ring read may retire first and satisfy lgkmcnt(1): the ring
    # read can still be in flight
    smem = head + "\ts_load_dword s4, s[0:1], 0x0\n\ts_waitcnt lgkmcnt(1)\n\tv_mov_b32_e32 v12, v5\n.Lfunc_end0:\n"
    assert [b[2] for b in ring_violations(smem, r"_ZN3awq12_GLOBAL__N_115act_loss_kernel")[1]] == \
        ["v_mov_b32_e32 v12, v5"]
    # ... while with two ring reads outstanding, lgkmcnt(1) leaves at most one LDS read in flight
    two = head.replace(";;#ASMEND\n", ";;#ASMEND\n\t;;#ASMSTART\n\tds_read_b128 v[8:11], v1 offset:16\n\t;;#ASMEND\n", 1)
    ok2 = two + "\ts_load_dword s4, s[0:1], 0x0\n\ts_waitcnt lgkmcnt(1)\n\tv_mov_b32_e32 v12, v5\n.Lfunc_end0:\n"
    assert ring_violations(ok2, r"_ZN3awq12_GLOBAL__N_115act_loss_kernel")[1] == []
