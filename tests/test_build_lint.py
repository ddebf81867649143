"""Lint of the build recipes the repository ships (CPU only).

The GPU pool refuses any run whose uploaded sources hold a hipcc statement that
would instrument device code: GPU AddressSanitizer is unavailable there.  A
hipcc statement carrying ``-fsanitize=`` is accepted only when

* every ``-fsanitize=`` token directly follows ``-Xarch_host``, or
* the statement has ``-fno-gpu-sanitize`` and no ``-Xarch_`` option at all.

Makefile variables are followed one level: a variable holding ``-fsanitize=``
is checked as part of every hipcc statement that expands it, and is exempt
when only gcc/g++ statements use it.  Round 3 lost its driver GPU run to one
non-conforming link line (``tests/native/Makefile``); this test keeps that
from recurring.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_HIPCC = re.compile(r"(hipcc|HIPCC|amdclang\+\+|clang\+\+)")
_GCC = re.compile(r"(^|\s|/)(gcc|g\+\+|cc|CC)(\s|$)")
_VAR_DEF = re.compile(r"^\s*([A-Za-z_][A-Za-z0-9_]*)\s*(\?=|:=|\+=|=)(.*)$")


def _tracked_recipes():
    try:
        out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True,
                             text=True, timeout=60, check=True).stdout.split()
    except (OSError, subprocess.SubprocessError):
        out = []
        for d, _, files in os.walk(ROOT):
            if ".git" in d or "gpurun_out" in d:
                continue
            out += [os.path.relpath(os.path.join(d, f), ROOT) for f in files]
    return [f for f in out
            if os.path.basename(f) == "Makefile" or f.endswith((".mk", ".sh"))]


def _logical_lines(text):
    """Join backslash continuations; return (first_line_no, statement)."""
    lines, buf, start = [], "", None
    for i, raw in enumerate(text.splitlines(), 1):
        line = raw.split("#", 1)[0] if not raw.lstrip().startswith("\t") else raw
        if start is None:
            start = i
        if line.rstrip().endswith("\\"):
            buf += line.rstrip()[:-1] + " "
            continue
        buf += line
        lines.append((start, buf))
        buf, start = "", None
    if buf:
        lines.append((start, buf))
    return lines


def _conforms(stmt):
    toks = stmt.split()
    san = [i for i, t in enumerate(toks) if t.startswith("-fsanitize=")]
    if not san:
        return True
    if all(i > 0 and toks[i - 1] == "-Xarch_host" for i in san):
        return True
    return "-fno-gpu-sanitize" in toks and not any(t.startswith("-Xarch_") for t in toks)


def violations(text):
    stmts = _logical_lines(text)
    defs = {}
    for no, s in stmts:
        m = _VAR_DEF.match(s)
        if m and not s.startswith("\t"):
            defs.setdefault(m.group(1), []).append((no, m.group(3)))
    bad = []
    san_vars = {v for v, ds in defs.items() if any("-fsanitize=" in d for _, d in ds)}
    for no, s in stmts:
        if _VAR_DEF.match(s) and not s.startswith("\t"):
            continue
        used = [v for v in san_vars if re.search(r"\$[({]%s[)}]" % v, s) or
                re.search(r"\$%s\b" % v, s)]
        if "-fsanitize=" not in s and not used:
            continue
        if not _HIPCC.search(s):
            continue          # gcc / g++ host-only statement
        expanded = s
        for v in used:
            expanded += " " + " ".join(d for _, d in defs[v])
        if not _conforms(expanded):
            bad.append((no, s.strip()[:160]))
    # A sanitizer variable no statement expands is still a hazard if it is a hipcc line.
    for v in san_vars:
        for no, d in defs[v]:
            if _HIPCC.search(d) and not _conforms(d):
                bad.append((no, d.strip()[:160]))
    return bad


def test_lint_catches_round3_link_line():
    bad = ("OUT := x\n"
           "all:\n"
           "\t$(HIPCC) --offload-arch=gfx950 -fsanitize=address,undefined -o $@ a.o\n")
    assert violations(bad)
    var = ("SAN := -fsanitize=address\n"
           "t:\n\t$(HIPCC) $(SAN) -c a.hip\n")
    assert violations(var)


def test_lint_accepts_conforming_forms():
    ok = ("H := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -fno-gpu-sanitize\n"
          "G := -fsanitize=address,undefined\n"
          "t:\n\t$(HIPCC) $(H) -c a.hip\n"
          "\tgcc $(G) -o x x.c\n"
          "\t$(HIPCC) --offload-arch=gfx950 -fsanitize=address -fno-gpu-sanitize -o y y.o\n")
    assert violations(ok) == []


@pytest.mark.parametrize("path", _tracked_recipes())
def test_tracked_recipe_has_no_device_sanitizer(path):
    with open(os.path.join(ROOT, path), errors="replace") as f:
        bad = violations(f.read())
    assert not bad, f"{path}: hipcc statement instruments device code: {bad}"
