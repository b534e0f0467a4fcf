"""The ctypes ABI of the kernel library, checked without a GPU.

ctypes passes surplus arguments with default conversions (a Python int becomes a 32-bit C
int), so a call or a declaration that disagrees with the C signature truncates pointers and
faults on the device.  Three views must agree for every entry point: the ``extern "C"``
definition in ``csrc/*.hip``, the argtypes table in ``ops/_lib.py`` and every call site."""

import ast
import re
from pathlib import Path

from sparse_coding__amd.ops import _lib

ROOT = Path(__file__).resolve().parents[1] / "sparse_coding__amd"


def _c_arities():
    out = {}
    for f in (ROOT / "ops" / "csrc").rglob("*.hip"):
        text = f.read_text()
        for m in re.finditer(r"^int\s+(sc_\w+)\s*\(", text, re.M):
            depth, i = 1, m.end()
            while depth:
                depth += {"(": 1, ")": -1}.get(text[i], 0)
                i += 1
            params = text[m.end(): i - 1].strip()
            out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def _declared():
    req, opt = _lib.signatures()
    return {**req, **opt}


def test_argtypes_match_c_definitions():
    c = _c_arities()
    decl = _declared()
    missing = sorted(set(decl) - set(c))
    assert not missing, f"declared but not defined in csrc: {missing}"
    bad = {n: (len(a), c[n]) for n, a in decl.items() if len(a) != c[n]}
    assert not bad, f"argtypes count != C parameter count (declared, C): {bad}"


def test_call_sites_match_argtypes():
    decl = _declared()
    bad = []
    for f in ROOT.rglob("*.py"):
        tree = ast.parse(f.read_text())
        for node in ast.walk(tree):
            if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)):
                continue
            name = node.func.attr
            if name not in decl or any(isinstance(a, ast.Starred) for a in node.args) or node.keywords:
                continue
            if len(node.args) != len(decl[name]):
                bad.append(f"{f.relative_to(ROOT)}:{node.lineno} {name}: {len(node.args)} args, "
                           f"declared {len(decl[name])}")
    assert not bad, "\n".join(bad)
