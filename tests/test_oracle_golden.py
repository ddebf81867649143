"""Pin the CPU oracle (oracle/) against the reference's own outputs (tests/golden/).

The fixtures were produced by importing the reference awq.py in the build
container (tests/golden/make_golden.py).  Every case must match bit for bit
(int32 tensor_q/zero_points, fp16 scales, fp32 dequantize) — NaN payloads and signs
included: the NaN-origin fixtures (make_golden.py --nan, golden_nan.*) pin the bits of NaN
scales for every input dtype, group size, NaN origin and the small-tensor path.
"""
import pytest
import torch

import golden_io as gio
from oracle import awq_oracle as orc


@pytest.mark.parametrize("case", gio.ok_cases(), ids=lambda c: c["name"])
def test_oracle_matches_reference_case(case):
    x = gio.case_input(case)
    p = case["params"]
    res = orc.quantize(x, bits=p["bits"], group_size=p["group_size"], symmetric=p["symmetric"],
                       per_channel=p.get("per_channel", True))
    T = gio.tensors()
    name = case["name"]
    assert torch.equal(res["tensor_q"], T[name + ".tensor_q"]), "tensor_q"
    assert torch.equal(res["zero_points"], T[name + ".zero_points"]), "zero_points"
    assert gio.same_bits(res["scales"], T[name + ".scales"]), "scales"
    if "out_shapes" in case:
        assert list(res["scales"].shape) == case["out_shapes"]["scales"]
    if name + ".dq" in T:
        dq = orc.dequantize(res)
        assert gio.same_bits(dq, T[name + ".dq"]), "dequantize"
    elif case.get("dequantize") == "IndexError":
        with pytest.raises(IndexError):
            orc.dequantize(res)


@pytest.mark.parametrize("case", gio.nan_cases(), ids=lambda c: c["name"])
def test_oracle_matches_reference_nan_case(case):
    x = gio.nan_case_input(case)
    p = case["params"]
    res = orc.quantize(x, bits=p["bits"], group_size=p["group_size"], symmetric=p["symmetric"],
                       per_channel=p["per_channel"])
    T = gio.nan_tensors()
    name = case["name"]
    assert torch.equal(res["tensor_q"], T[name + ".tensor_q"]), "tensor_q"
    assert torch.equal(res["zero_points"], T[name + ".zero_points"]), "zero_points"
    assert gio.same_bits(res["scales"], T[name + ".scales"]), "scales"
    if name + ".dq" in T:
        assert gio.same_bits(orc.dequantize(res), T[name + ".dq"]), "dequantize"


def test_nan_fixtures_cover_every_origin():
    """The NaN-origin fixtures hold NaN scales of every kind the rule distinguishes."""
    T = gio.nan_tensors()
    seen = set()
    for c in gio.nan_cases():
        s = T[c["name"] + ".scales"].reshape(-1).view(torch.int16)
        seen |= {int(v) & 0xFFFF for v in s.tolist() if (int(v) & 0x7FFF) > 0x7C00}
    assert {0x7E00, 0xFE00, 0x7FFF, 0xFFFF, 0x7E90, 0xFE90} <= seen, sorted(map(hex, seen))


@pytest.mark.parametrize("rec", gio.manifest()["hashed"], ids=lambda r: r["name"])
def test_oracle_matches_reference_hashed(rec):
    x = gio.hashed_input(rec)
    assert gio.sha(x) == rec["sha_x"], "input regeneration drifted"
    p = rec["params"]
    res = orc.quantize(x, bits=p["bits"], group_size=p["group_size"], symmetric=p["symmetric"])
    assert gio.sha(res["tensor_q"]) == rec["sha_tensor_q"]
    assert gio.sha(res["scales"]) == rec["sha_scales"]
    assert gio.sha(res["zero_points"]) == rec["sha_zero_points"]
    if rec.get("sha_dq"):
        assert gio.sha(orc.dequantize(res)) == rec["sha_dq"]


def test_exhaustive_bf16_reciprocal_identity():
    """The bf16 fast path's x*RN(1/s) == x/s identity, over all 1.35e9 (x, s) pairs."""
    import os
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.dirname(orc.__file__), "verify_recip"], check=True)
    out = subprocess.run([os.path.join(os.path.dirname(orc.__file__), "verify_recip"), "bf16"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout


def test_f16_markstein_division_exhaustive():
    """The fp16 fast path's corrected quotient fma(fma(-s, x*r, x), r, x*r) == RN(x/s) after
    fp16 rounding, over all 2.0e9 (x, positive finite s) pairs."""
    import os
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.dirname(orc.__file__), "verify_recip"], check=True)
    out = subprocess.run([os.path.join(os.path.dirname(orc.__file__), "verify_recip"), "f16m"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout


def test_f16_plain_product_small_scales_exhaustive():
    """The fp16 fast path's plain quotient RN(x * RN(1/s)) == RN(x/s) for every fp16 x and
    every positive fp16 scale s < 14 (1.2e9 pairs); 14 is the first scale where it fails."""
    import os
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.dirname(orc.__file__), "verify_recip"], check=True)
    out = subprocess.run([os.path.join(os.path.dirname(orc.__file__), "verify_recip"), "f16s"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout and "first_failing_scale=14" in out.stdout


def test_search_alpha_markstein_exhaustive():
    """The clip search's alpha_i = RN((n - i) / n) from RN(1/n) and one Markstein correction ==
    the IEEE quotient for every n <= 65536 and i < n (2.1e9 pairs): the streaming kernel forms
    it without a division per candidate (awq_fast.hip search_alpha)."""
    import os
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.dirname(orc.__file__), "verify_recip"], check=True)
    out = subprocess.run([os.path.join(os.path.dirname(orc.__file__), "verify_recip"), "alpha"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "pairs=2147516416 mismatches=0" in out.stdout


def _verify_recip(arg):
    import os
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.dirname(orc.__file__), "verify_recip"], check=True)
    return subprocess.run([os.path.join(os.path.dirname(orc.__file__), "verify_recip"), arg],
                          capture_output=True, text=True, timeout=600)


def test_search_packed_fp16_steps_exhaustive():
    """The clip search's packed-fp16 chains (awq_fast.hip chunk_err_f16p / chunk_err_bf16h):
    rint + clamp as RN_f16(u + 1024 - qmin) clamped to [1024, 1024 + qmax - qmin] equals
    clamp(rint(u)) for every fp16 and bf16 u, 4 / 8 bit, sym / asym; and the fp16 quotient must
    stay double-rounded (RN_f16(RN_f32(x r))): one rounding straight to fp16 misses pairs."""
    out = _verify_recip("chain16")
    assert out.returncode == 0, out.stdout + out.stderr
    assert "cases=515088 mismatches=0" in out.stdout
    fused = _verify_recip("f16f")
    assert fused.returncode == 1 and "mismatches=890" in fused.stdout, fused.stdout


def test_f16_scale_by_reciprocal_exhaustive():
    """The fp16 group scale without the IEEE division (awq_quant.h FmtF16::scale, act
    HwFmt<F16>::scale): RN_f16(d * RN(1/qr)) == RN_f16(d / qr) for every non-negative fp16 d
    (inf included) and qr = 2^bits - 1, bits 2..8."""
    out = _verify_recip("f16scale")
    assert out.returncode == 0, out.stdout + out.stderr
    assert "cases=222215 mismatches=0" in out.stdout
