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


def ring_violations(asm: str, func_rx: str):
    """(function, line, instruction) for every instruction that touches a register an
    inline ds_read_b128 is still loading (lgkmcnt(N) retires all but the N youngest reads:
    LDS reads complete in order)."""
    bad, funcs = [], re.findall(r"^(" + func_rx + r"\w*):", asm, re.M)
    for f in funcs:
        i = asm.index(f + ":")
        body = asm[i:asm.index(".Lfunc_end", i)].split("\n")
        pending = []                                   # [(issue order, registers)]
        for n, line in enumerate(body):
            s = line.strip()
            if not s or s.startswith(";"):
                continue
            m = re.match(r"ds_read_b128 (v\[\d+:\d+\]), v\d+", s)
            if m:
                pending.append(_regs(m.group(1)))
                continue
            m = re.match(r"s_waitcnt .*lgkmcnt\((\d+)\)", s)
            if m:
                k = int(m.group(1))
                pending = pending[len(pending) - k:] if k else []
                continue
            if re.match(r"(s_|\.|[A-Za-z_.$][\w.$]*:)", s):
                continue
            live = set().union(*pending) if pending else set()
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
    assert not bad, bad[:5]


def test_ring_checker_flags_an_early_use():
    asm = """_ZN3awq12_GLOBAL__N_115act_loss_kernelX:
\tds_read_b128 v[4:7], v1 offset:0
\tds_read_b128 v[8:11], v1 offset:16
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
