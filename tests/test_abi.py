"""C ABI and host logic without a GPU (CPU-only).

* the library loads and exports every symbol include/*.h declares;
* error behaviour without a device (no silent CPU fallback);
* index parsing / ImageId / registries (pure host bookkeeping) against the
  reference's fixture (src/cluster/download.rs:357-366).
"""
import glob
import os
import re
import subprocess

import pytest

from conftest import ROOT

import ciruela_amd as ca
from ciruela_amd import _native


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(cir_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    return syms


def test_exports_every_declared_symbol():
    decl = declared_symbols()
    assert len(decl) >= 25
    out = subprocess.check_output(["nm", "-D", "--defined-only", _native.LIB_PATH]).decode()
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = decl - exported
    assert not missing, missing
    # and the Python binding covers all of them
    assert decl <= set(_native.EXPORTED) | {"cir_init"}


def test_integration_binds_every_entry_point():
    """INTEGRATION.md's Rust extern block declares every product entry point
    of the header (test-data and cir_debug_* exports aside)."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    bound = set(re.findall(r"pub fn (cir_[a-z0-9_]+)\(", block))
    product = {s for s in declared_symbols()
               if not s.startswith("cir_debug_") and s != "cir_fill_splitmix64_dev"}
    assert product - bound == set()
    assert bound - declared_symbols() == set()


def test_library_is_gfx950_code():
    """The embedded fat binary carries gfx950 code objects (and only those)."""
    blob = open(_native.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_strerror_codes():
    for code in range(-10, 1):
        assert _native.lib.cir_strerror(code)
    assert _native.lib.cir_strerror(_native.CIR_ENOTFOUND) == b"not found"
    assert _native.lib.cir_strerror(_native.CIR_EAGAIN) == b"try again"


def test_device_count_policy():
    """cir_devices_for_bytes (the CLI's and cir_init_n's device-count hint,
    no HIP call): ceil(bytes / (2 x staging)) devices, capped at the visible
    count, at least one; unknown work (0) opens every visible device."""
    f = _native.lib.cir_devices_for_bytes
    MiB, GiB = 1 << 20, 1 << 30
    assert f(10 * MiB, 10 * MiB, 8) == 1          # the config-1 CLI: one slot, one GPU
    assert f(300 * MiB, 0, 8) == 1                # default staging 256 MiB: 2 x 256 per GPU
    assert f(512 * MiB, 0, 8) == 1
    assert f(512 * MiB + 1, 0, 8) == 2
    assert f(520 * MiB, _native.CIR_STAGING_LAZY, 8) == 2
    assert f(3 * GiB, 0, 8) == 6
    assert f(50 * GiB, 0, 8) == 8                 # config 5 on a node: every GPU
    assert f(50 * GiB, 0, 1) == 1
    assert f(1, 0, 8) == 1
    assert f(0, 0, 8) == 8 and f(0, 0, 3) == 3
    assert f(5 * GiB, 0, 0) == 0
    assert f(100 * MiB, 16 * MiB, 32) == 4        # small slots: more devices per byte
    assert f((1 << 64) - 1, (1 << 63), 4) == 1    # no overflow in 2 x staging
    assert ca.Context.devices_for_bytes(3 * GiB, visible=4) == 4


def test_no_device_is_loud():
    import torch
    if torch.cuda.is_available():
        pytest.skip("this container has no GPU; only meaningful without one")
    with pytest.raises(ca.NoDevice):
        ca.Context()
    with pytest.raises(ca.NoDevice):
        ca.BlockHash.hash_bytes(b"abc")


def test_get_hash_and_image_id(dirsig_example):
    idx = dirsig_example["index"].encode()
    raw = ca.get_hash(idx)
    assert raw.hex() == "552ca5730ee95727e890a2155c88609d244624034ff70de264cf88220d11d6df"
    iid = ca.ImageId(raw)
    assert str(iid) == raw.hex()
    assert ca.ImageId.from_str(raw.hex()) == iid
    with pytest.raises(ca.CiruelaError):
        ca.get_hash(b"DIRSIGNATURE.v1 blake2b/256 block_size=32768\n/\nnot-hex\n")


def test_in_memory_indexes(dirsig_example):
    idx = dirsig_example["index"].encode()
    reg = ca.InMemoryIndexes()
    iid = reg.register_index(idx)
    assert reg.read_index(iid) == idx
    with pytest.raises(ca.ReadError) as e:
        reg.read_index(ca.ImageId(bytes(32)))
    assert e.value.status == _native.CIR_ENOTFOUND
    with pytest.raises(ca.IndexError_):
        reg.register_index(b"garbage")


def test_register_dir_and_read_block(tmp_path, dirsig_example):
    """ThreadedBlockReader::register_dir (src/blocks.rs:145-183) on the
    reference fixture: one block per non-empty file, Disk{path, 0, size}."""
    idx = dirsig_example["index"].encode()
    (tmp_path / "subdir").mkdir()
    (tmp_path / "subdir" / ".hidden").write_bytes(b"Hidden\n")
    r = ca.ThreadedBlockReader()
    r.register_dir(str(tmp_path), idx)
    assert len(r) == 3  # hello.txt, .hidden, file.txt (test.txt is empty)
    h = bytes.fromhex("6d7f5f9804ee4dbc1ff7e12c7665387e0119e8ea629996c52d38b75c12ad0acf")
    assert r.read_block(ca.BlockHash(h)) == b"Hidden\n"
    with pytest.raises(ca.ReadError):  # hello.txt is not on disk
        r.read_block(bytes.fromhex(
            "a79eef66019bfb9a41f798f2cff2d2d36ed294cc3f96bf53bbfc5192ebe60192"))
    with pytest.raises(ca.ReadError) as e:
        r.read_block(bytes(32))
    assert e.value.status == _native.CIR_ENOTFOUND


def test_register_dir_multiblock(tmp_path):
    """Block pointers: offset = idx * bs, size = min(left, bs)."""
    data = bytes(range(256)) * 40  # 10240 bytes, bs 4096 -> 3 blocks
    (tmp_path / "f.bin").write_bytes(data)
    hs = [bytes([i]) * 32 for i in range(3)]
    idx = (b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  f.bin f 10240 " +
           b" ".join(h.hex().encode() for h in hs) + b"\n" + b"ab" * 32 + b"\n")
    r = ca.ThreadedBlockReader()
    r.register_dir(str(tmp_path), idx)
    assert r.read_block(hs[0]) == data[:4096]
    assert r.read_block(hs[1]) == data[4096:8192]
    assert r.read_block(hs[2]) == data[8192:]


def test_register_dir_errors(tmp_path):
    r = ca.ThreadedBlockReader()
    with pytest.raises(ca.DirError) as e:
        r.register_dir(str(tmp_path), b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n"
                                      b"  f f 10 zz\n" + b"ab" * 32 + b"\n")
    assert e.value.status == _native.CIR_EPARSE
    with pytest.raises(ca.DirError):  # wrong number of hashes for the size
        r.register_dir(str(tmp_path), b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n"
                                      b"  f f 5000 " + b"ab" * 32 + b"\n" + b"ab" * 32 + b"\n")


def test_register_dir_hash_size_and_huge_size(tmp_path):
    """A block hash that is not 32 bytes is DirError::HashSize
    (BlockHash::from_bytes, src/blocks.rs:168-170), not a silently
    mis-split hash list; the rewrite reports it as a parse error.  A size
    near 2^64 needs its full hash count (no wrap in ceil(size / bs))."""
    import ctypes
    r = ca.ThreadedBlockReader()
    short = (b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  f f 10 " + b"ab" * 16 +
             b"\n" + b"ab" * 32 + b"\n")
    with pytest.raises(ca.DirError) as e:
        r.register_dir(str(tmp_path), short)
    assert e.value.status == _native.CIR_EHASHSIZE
    out, ln = ctypes.c_void_p(), ctypes.c_size_t()
    rc = _native.lib.cir_index_rewrite(None, short, len(short), ctypes.byref(out),
                                       ctypes.byref(ln))
    assert rc == _native.CIR_EPARSE
    huge = (b"DIRSIGNATURE.v1 blake2b/256 block_size=32768\n/\n  f f 18446744073709551615\n" +
            b"ab" * 32 + b"\n")
    with pytest.raises(ca.DirError) as e:
        r.register_dir(str(tmp_path), huge)
    assert e.value.status == _native.CIR_EPARSE
    assert b"wrong number of hashes" in _native.lib.cir_last_error()
    assert len(r) == 0


def test_block_hash_type():
    h = ca.BlockHash(bytes(range(32)))
    assert str(h) == bytes(range(32)).hex()
    assert repr(h).startswith("BlockHash(")
    assert ca.BlockHash.from_bytes(b"x" * 31) is None
    assert ca.BlockHash.from_bytes(b"x" * 32) == ca.BlockHash(b"x" * 32)
    assert len({ca.BlockHash(b"x" * 32), ca.BlockHash(b"x" * 32)}) == 1


def test_cli_usage():
    cli = os.path.join(ROOT, "bin", "ciruela-index")
    p = subprocess.run([cli], capture_output=True)
    assert p.returncode == 2 and b"usage" in p.stderr


def _cli_staging(args, tmp_path):
    """The staging size the CLI picks for its inputs (printed under
    CIR_TRACE before cir_init, which then fails: no device here)."""
    cli = os.path.join(ROOT, "bin", "ciruela-index")
    env = dict(os.environ, CIR_TRACE="1")
    p = subprocess.run([cli] + args, capture_output=True, env=env, cwd=str(tmp_path))
    m = re.search(rb"staging (\d+) bytes per slot", p.stderr)
    assert m, p.stderr
    return int(m.group(1))


def test_cli_staging_follows_top_level_symlinks(tmp_path):
    """The one-shot CLI sizes its staging slots from the input's bytes; a
    symlinked SRC directory or FILE counts its target (the scan and the hash
    path follow it), a pipe gets the default (0); entries inside a tree are
    not followed, as the scan does not follow them."""
    tree = tmp_path / "tree"
    tree.mkdir()
    (tree / "a.bin").write_bytes(os.urandom(3 << 20))
    os.symlink(str(tree), tmp_path / "link")
    os.symlink(str(tree / "a.bin"), tmp_path / "flink")
    (tree / "inner").symlink_to(tmp_path / "tree" / "a.bin")  # not followed
    mib = 1 << 20
    assert _cli_staging(["sync", "--append", str(tree) + ":/x"], tmp_path) == 3 * mib
    assert _cli_staging(["sync", "--append", str(tmp_path / "link") + ":/x"], tmp_path) == 3 * mib
    assert _cli_staging(["hash", str(tmp_path / "flink")], tmp_path) == 3 * mib
    assert _cli_staging(["hash", "/dev/stdin"], tmp_path) == 0


BAD_PATH_INDEXES = [
    # fill_dirs accepts only RootDir / Normal components (src/cluster/download.rs:120-145)
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n/../etc\n  passwd f 0\n",
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n/a/./b\n  f f 0\n",
    # an entry needs a file_name() (:148-162)
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  .. f 0\n",
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  . f 0\n",
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  a\\x2fb f 0\n",
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  .. s /etc\n",
]


@pytest.mark.parametrize("bad", BAD_PATH_INDEXES)
def test_invalid_paths_rejected(tmp_path, bad):
    """IndexParseEnum::InvalidPath: `..`, `.` and names with a slash are
    rejected by register_dir and by the rewrite (RawIndex::into_mut), so a
    registered block never maps outside its directory."""
    import ctypes
    idx = bad + b"ab" * 32 + b"\n"
    r = ca.ThreadedBlockReader()
    with pytest.raises(ca.DirError) as e:
        r.register_dir(str(tmp_path), idx)
    assert e.value.status == _native.CIR_EPARSE
    assert b"Invalid path" in _native.lib.cir_last_error()
    out, ln = ctypes.c_void_p(), ctypes.c_size_t()
    rc = _native.lib.cir_index_rewrite(None, idx, len(idx), ctypes.byref(out), ctypes.byref(ln))
    assert rc == _native.CIR_EPARSE
    assert len(r) == 0


PATH_CONFLICT_INDEXES = [
    # a file, then a directory line through the same name (download.rs:138-140)
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  a f 0\n/a\n  b f 0\n",
    # a deeper directory line crossing a file of an earlier directory
    b"DIRSIGNATURE.v1 sha512/256 block_size=4096\n/\n/d\n  x f 0\n/d/x/y\n  z f 0\n",
    # a symlink is not a directory either
    b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  l s /tmp\n/l\n  f f 0\n",
]


@pytest.mark.parametrize("bad", PATH_CONFLICT_INDEXES)
def test_rewrite_path_conflict(bad):
    """IndexParseEnum::PathConflict (fill_dirs, src/cluster/download.rs:
    126-140): a directory line whose path runs through a file or a symlink
    of an earlier line.  RawIndex::into_mut fails with it, so the rewrite
    (cir_index_rewrite) returns CIR_EPARSE naming the path -- detected while
    the tree is rebuilt on the host, before any device is needed."""
    import ctypes
    idx = bad + b"ab" * 32 + b"\n"
    out, ln = ctypes.c_void_p(), ctypes.c_size_t()
    rc = _native.lib.cir_index_rewrite(None, idx, len(idx), ctypes.byref(out), ctypes.byref(ln))
    assert rc == _native.CIR_EPARSE
    assert b"conflicts with others" in _native.lib.cir_last_error()
    # the same tree without the conflicting line passes fill_dirs and stops
    # only at the missing context (the footer is hashed on the GPU)
    ok = b"\n".join(ln_ for ln_ in bad.split(b"\n")
                    if not (ln_.startswith(b"/") and ln_ != b"/" and (
                        ln_ in (b"/a", b"/l", b"/d/x/y")))) + b"ab" * 32 + b"\n"
    rc = _native.lib.cir_index_rewrite(None, ok, len(ok), ctypes.byref(out), ctypes.byref(ln))
    assert rc == _native.CIR_EINVAL and b"null ctx" in _native.lib.cir_last_error()


def test_valid_odd_names_still_parse(tmp_path):
    """Names that merely look like paths stay valid: `...`, `.x`, escaped bytes."""
    idx = (b"DIRSIGNATURE.v1 blake2b/256 block_size=4096\n/\n  ... f 0\n  .x f 0\n"
           b"  a\\x20b f 0\n/sub..dir\n  f f 0\n" + b"ab" * 32 + b"\n")
    ca.ThreadedBlockReader().register_dir(str(tmp_path), idx)


def test_descriptor_count_limit():
    """cir_hash_blocks_dev_ht takes at most 2^31-1 descriptors (32-bit block
    indices in the kernels and in the ordering's permutation): larger
    batches are rejected before anything touches a device."""
    lib = _native.lib
    for n in (1 << 31, (1 << 32) + 5):
        rc = lib.cir_hash_blocks_dev_ht(None, _native.CIR_HASH_BLAKE2B_256, 16, 16, 16, n, 32, None)
        assert rc == _native.CIR_EINVAL
        assert b"2^31-1" in lib.cir_last_error()


def test_product_never_loads_the_oracle():
    """The oracle is test infrastructure: the library exports and imports
    nothing of it, and no product source names its library or modules (the
    footer's host BLAKE2b is the product's own, blake2b_host.cpp)."""
    out = subprocess.check_output(["nm", "-D", _native.LIB_PATH]).decode()
    assert "oracle_" not in out
    libs = subprocess.check_output(["readelf", "-d", _native.LIB_PATH]).decode()
    assert "oracle" not in libs
    srcs = glob.glob(os.path.join(ROOT, "ciruela_amd", "**", "*.*"), recursive=True)
    for p in srcs:
        if not p.endswith((".py", ".cpp", ".hpp", ".hip", ".h")):
            continue
        text = open(p, errors="replace").read()
        for bad in ("liboracle", "blake2b_oracle", "import cpu_indexer", "import dirsig_oracle",
                    "oracle/"):
            assert bad not in text, (p, bad)


def test_cli_rejects_bad_numbers(tmp_path):
    """--disk-threads / --block-size take a decimal count; anything else is a
    usage error (exit 2), not an uncaught exception out of main."""
    cli = os.path.join(ROOT, "bin", "ciruela-index")
    for flag, v in [("--disk-threads", "abc"), ("--block-size", "-5"), ("--block-size", "12x"),
                    ("--disk-threads", "99999999999"), ("--block-size", "")]:
        p = subprocess.run([cli, "sync", flag, v, "--append", "%s:/d" % tmp_path],
                           capture_output=True)
        assert p.returncode == 2, (flag, v, p.stderr)
        assert b"invalid value for " + flag.encode() in p.stderr


_ENOMEM_CHILD = r"""
import ctypes, resource, sys
sys.path.insert(0, sys.argv[1])
from ciruela_amd import _native
lib = _native.lib
lines = ["DIRSIGNATURE.v1 blake2b/256 block_size=32768", "/"]
lines += ["  f%07d f 100 %s" % (i, "ab" * 32) for i in range(1000000)]
index = ("\n".join(lines) + "\n" + "00" * 32 + "\n").encode()
h = lib.cir_indexes_new()
assert h
vm = [int(l.split()[1]) for l in open("/proc/self/status") if l.startswith("VmSize:")][0] * 1024
resource.setrlimit(resource.RLIMIT_AS, (vm + (32 << 20), resource.RLIM_INFINITY))
out = ctypes.create_string_buffer(64)
n = ctypes.c_size_t()
rc = lib.cir_indexes_register(h, index, len(index), out, ctypes.byref(n))
print(rc, lib.cir_last_error().decode())
"""


def test_no_exception_crosses_the_abi():
    """A host allocation that fails inside the library comes back as
    CIR_ENOMEM with its text in cir_last_error -- not std::terminate (and
    never an unwind into a Rust caller).  A child process parses a 1M-file
    index with 32 MiB of address space to spare."""
    p = subprocess.run(["python3", "-c", _ENOMEM_CHILD, ROOT], capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    rc, _, msg = p.stdout.decode().strip().partition(" ")
    assert int(rc) == _native.CIR_ENOMEM, p.stdout
    assert "C++ exception" in msg
