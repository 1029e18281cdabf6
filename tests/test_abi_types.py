"""The C-ABI boundary checked by type, not only by name (CPU only).

* INTEGRATION.md §2's Rust `extern "C"` block (the binding a ciruela
  maintainer adds; reference call sites src/client/sync/uploads.rs:49-59,
  src/block_id.rs:37) is translated to C prototypes and compiled in one
  translation unit after include/ciruela_blockhash.h: a parameter of another
  width, signedness or constness, a missing or extra parameter, or another
  return type is a conflicting redeclaration, so the compile fails.
* ciruela_amd/_native.py's ctypes table (the binding the tests go through)
  is checked against the header's parsed prototypes: the same arity, the
  same integer width and signedness per scalar, a pointer wherever the
  header has one (and a pointee of the same width when typed), the same
  return type.
Either drift is undefined behaviour across an FFI boundary and would pass a
check by names alone.
"""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

from ciruela_amd import _native

HEADER = os.path.join(ROOT, "include", "ciruela_blockhash.h")

# ---- Rust -> C -------------------------------------------------------------

_RUST_SCALARS = {
    "u8": "uint8_t", "u16": "uint16_t", "u32": "uint32_t", "u64": "uint64_t",
    "i32": "int32_t", "i64": "int64_t", "usize": "size_t", "isize": "ptrdiff_t",
    "c_int": "int", "c_uint": "unsigned", "c_char": "char", "c_void": "void",
    "f64": "double", "CirCtx": "cir_ctx", "CirIndexes": "cir_indexes", "CirBlocks": "cir_blocks",
}
_WRITE_FN = 'extern "C" fn(*mut c_void, *const u8, usize) -> c_int'


def rust_type_to_c(t):
    t = " ".join(t.split())
    if t == _WRITE_FN:
        return "cir_write_fn"
    if t == "HipStream":
        return "void*"
    m = re.fullmatch(r"\*(const|mut) (.+)", t)
    if m:
        inner = rust_type_to_c(m.group(2))
        # `*const T` -> `const T*`; a pointer's own constness sits after the *
        if inner.endswith("*"):
            return inner + (" const*" if m.group(1) == "const" else "*")
        return ("const " if m.group(1) == "const" else "") + inner + "*"
    if t in _RUST_SCALARS:
        return _RUST_SCALARS[t]
    raise ValueError("no C type for Rust type %r" % t)


def _split_args(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out if a.strip()]


def rust_extern_fns():
    """[(name, [(arg, rust type)], rust return type or None)] of the block."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    block = re.sub(r"//[^\n]*", "", block)
    fns = []
    for m in re.finditer(r"pub fn (cir_[a-z0-9_]+)\((.*?)\)\s*(->\s*([^;]+))?;", block, re.S):
        # the writer's fn type contains parentheses: re-find the real end of
        # the parameter list from the name on
        start = m.start(2)
        depth, i = 1, start
        while depth:
            depth += {"(": 1, ")": -1}.get(block[i], 0)
            i += 1
        params = block[start:i - 1]
        rest = block[i:block.index(";", i)]
        ret = rest.split("->", 1)[1].strip() if "->" in rest else None
        args = []
        for a in _split_args(params):
            name, ty = a.split(":", 1)
            args.append((name.strip(), ty.strip()))
        fns.append((m.group(1), args, ret))
    return fns


def rust_as_c_prototypes():
    lines = []
    for name, args, ret in rust_extern_fns():
        cargs = ", ".join("%s %s" % (rust_type_to_c(t), a) for a, t in args) or "void"
        lines.append("%s %s(%s);" % (rust_type_to_c(ret) if ret else "void", name, cargs))
    return lines


def test_rust_types_translate():
    assert rust_type_to_c("*mut *mut CirCtx") == "cir_ctx**"
    assert rust_type_to_c("*const *const c_char") == "const char* const*"
    assert rust_type_to_c("*const u8") == "const uint8_t*"
    assert rust_type_to_c("*mut u8") == "uint8_t*"
    assert rust_type_to_c(_WRITE_FN) == "cir_write_fn"


@pytest.mark.skipif(not shutil.which("gcc"), reason="no C compiler")
def test_rust_extern_block_compiles_against_the_header(tmp_path):
    protos = rust_as_c_prototypes()
    assert len(protos) >= 40
    src = tmp_path / "rust_block.c"
    src.write_text("#include <stddef.h>\n#include <stdint.h>\n#include \"ciruela_blockhash.h\"\n"
                   "/* INTEGRATION.md's Rust extern block, as C */\n" + "\n".join(protos) + "\n")
    # (-Wno-array-parameter: `uint8_t out[32]` and `uint8_t* out` are the same
    # parameter type; gcc only warns about the spelling)
    p = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Werror",
                        "-Wno-array-parameter", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-4000:]


@pytest.mark.skipif(not shutil.which("gcc"), reason="no C compiler")
def test_a_drifted_rust_signature_is_caught(tmp_path):
    """The check has teeth: one flipped constness, one widened scalar and one
    dropped parameter each fail the compile."""
    protos = rust_as_c_prototypes()
    one = next(p for p in protos if " cir_hash_blocks_dev(" in p)
    drifts = [one.replace("uint8_t* d_out", "const uint8_t* d_out"),
              one.replace("size_t nblk", "uint32_t nblk"),
              one.replace(", void* stream", "")]
    for d in drifts:
        assert d != one
        src = tmp_path / "drift.c"
        src.write_text("#include \"ciruela_blockhash.h\"\n" + d + "\n")
        p = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Werror",
                            "-I", os.path.join(ROOT, "include"), str(src)],
                           capture_output=True, text=True)
        assert p.returncode != 0, d


# ---- header -> ctypes ------------------------------------------------------

def header_prototypes():
    """{name: (return C type, [param C types])} of every cir_* function."""
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#[^\n]*", "", text)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_ \*]*?)\b(cir_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;",
                         text, re.S):
        ret, name, params = " ".join(m.group(1).split()), m.group(2), " ".join(m.group(3).split())
        if name == "cir_write_fn" or ret.startswith("typedef"):
            continue
        ptypes = []
        if params and params != "void":
            for prm in params.split(","):
                prm = prm.strip()
                arr = re.search(r"\[[^\]]*\]$", prm)
                if arr:  # `T out[N]` is `T* out` in a parameter list
                    prm = prm[:arr.start()].strip()
                    prm = re.sub(r"\s*\b\w+$", "", prm) + "*"
                else:
                    prm = re.sub(r"\s*\b\w+$", "", prm)  # drop the parameter name
                ptypes.append(" ".join(prm.replace("*", " * ").split()).replace(" *", "*"))
        protos[name] = (ret, ptypes)
    return protos


_SCALAR_CTYPES = {
    "int": ctypes.c_int, "uint32_t": ctypes.c_uint32, "uint64_t": ctypes.c_uint64,
    "size_t": ctypes.c_size_t,
}


def _compatible(ctype_decl, ctype):
    """Is the ctypes type `ctype` a faithful stand-in for the C type?"""
    c = ctype_decl.replace("const ", "").strip()
    if c == "void":
        return ctype is None
    if c.endswith("*") or c == "cir_write_fn":
        if ctype in (ctypes.c_void_p, ctypes.c_char_p) or \
                (isinstance(ctype, type) and issubclass(ctype, ctypes._CFuncPtr)):
            return True
        if isinstance(ctype, type) and issubclass(ctype, ctypes._Pointer):
            pointee = c[:-1].strip()
            if pointee in _SCALAR_CTYPES:
                want = _SCALAR_CTYPES[pointee]
                return ctypes.sizeof(ctype._type_) == ctypes.sizeof(want) and \
                    _signed(ctype._type_) == _signed(want)
            return True  # a pointer to a pointer or an opaque struct
        return False
    want = _SCALAR_CTYPES.get(c)
    if want is None:
        return False
    return ctype is not None and ctype not in (ctypes.c_void_p, ctypes.c_char_p) and \
        ctypes.sizeof(ctype) == ctypes.sizeof(want) and _signed(ctype) == _signed(want)


def _signed(t):
    try:
        return t(-1).value < 0
    except Exception:
        return None


def test_header_parses_every_declared_function():
    protos = header_prototypes()
    assert {"cir_init", "cir_scan_v1_write", "cir_hash_blocks_dev_bounded",
            "cir_verify_blocks_dev_bounded", "cir_indexes_new"} <= set(protos)
    assert protos["cir_blake2b256"] == ("int", ["const uint8_t*", "size_t", "uint8_t*"])
    assert protos["cir_indexes_new"] == ("cir_indexes*", [])


def test_ctypes_table_matches_header_types():
    protos = header_prototypes()
    problems = []
    for name, (restype, argtypes) in _native._SIGS.items():
        assert name in protos, "bound but not declared: %s" % name
        ret, params = protos[name]
        if len(params) != len(argtypes):
            problems.append("%s: %d parameters in the header, %d in ctypes"
                            % (name, len(params), len(argtypes)))
            continue
        for i, (cdecl, ct) in enumerate(zip(params, argtypes)):
            if not _compatible(cdecl, ct):
                problems.append("%s arg %d: header %s, ctypes %r" % (name, i, cdecl, ct))
        if not _compatible(ret, restype):
            problems.append("%s return: header %s, ctypes %r" % (name, ret, restype))
    assert problems == [], "\n".join(problems)


def test_ctypes_checker_rejects_a_drift():
    assert not _compatible("uint64_t", ctypes.c_uint32)
    assert not _compatible("int", ctypes.c_uint32)
    assert not _compatible("uint32_t", ctypes.c_void_p)
    assert not _compatible("uint64_t*", ctypes.POINTER(ctypes.c_uint32))
    assert _compatible("const uint8_t*", ctypes.c_void_p)
    assert _compatible("void", None)
    assert not _compatible("int", None)
