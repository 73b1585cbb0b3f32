"""rust/hec-sys (the Rust side of the drop-in) cannot be
compiled here (no Rust toolchain), so its extern block is checked against
include/hec.h as text: the same set of functions, each with the same number of
parameters, and the status-code constants equal to hec.h's enum."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_decls():
    src = open(os.path.join(ROOT, "include", "hec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(hec_\w+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def _rust_decls():
    src = open(os.path.join(ROOT, "rust", "hec-sys", "src", "lib.rs")).read()
    block = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (hec_\w+)\((.*?)\)", block, flags=re.S):
        args = m.group(2).strip().rstrip(",")
        out[m.group(1)] = 0 if not args else args.count(",") + 1
    return out


def test_extern_block_matches_header():
    c, r = _c_decls(), _rust_decls()
    assert len(c) > 60
    assert set(r) == set(c), (sorted(set(c) - set(r)), sorted(set(r) - set(c)))
    for name in c:
        assert r[name] == c[name], (name, c[name], r[name])


def test_status_constants_match_header():
    hdr = open(os.path.join(ROOT, "include", "hec.h")).read()
    codes = dict((k, int(v)) for k, v in re.findall(r"\b(HEC_(?:OK|ERR_\w+))\s*=\s*(\d+)", hdr))
    src = open(os.path.join(ROOT, "rust", "hec-sys", "src", "lib.rs")).read()
    consts = dict((k, int(v)) for k, v in re.findall(r"pub const (HEC_\w+): c_int = (\d+);", src))
    assert consts
    for k, v in consts.items():
        assert codes[k] == v, k
