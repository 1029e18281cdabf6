"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by ciruela_amd/).

Pure-Python restatement of the parts of dir-signature 0.2.9 (external crate,
Cargo.toml:35, not vendored in the reference) that ciruela's indexing path
uses, for small trees:

* `emit(header, tree)` — the DIRSIGNATURE.v1 text as the reference's own
  re-emitter writes it (MutableIndex::to_raw_data, src/cluster/download.rs:
  266-319): header line, then per directory a "/path" line, its files and
  symlinks sorted by name ("  name f|x size hash..." / "  name s target"),
  then its subdirectories; footer line = hex(H(every byte after the header
  line)).  Pinned by the reference fixture src/cluster/download.rs:357-366
  (tests/golden/dirsig_v1_example.json, checked in tests/test_dirsig.py).
* `scan(path, block_size)` — the v1::scan of `ciruela sync`
  (src/client/sync/uploads.rs:49-59) with blake2b/256 per-block hashes
  (BlockHash::hash_bytes, src/block_id.rs:37-43 = RFC 7693 BLAKE2b, nn=32,
  computed with hashlib, pinned in tests/test_oracle.py).  Unlike the
  re-emitter, the scanner keeps empty directories (unverified against the
  crate: DESIGN.md "Index format").
* escaping of names outside printable ASCII as \\xNN (unverified).
"""
import hashlib
import os
import stat


def h_blake2b256(data):
    return hashlib.blake2b(data, digest_size=32).digest()


def h_sha512_256(data):
    return hashlib.new("sha512_256", data).digest()


HASHES = {"blake2b/256": h_blake2b256, "sha512/256": h_sha512_256}


def escape(raw):
    out = []
    for c in raw:
        if c <= 0x20 or c >= 0x7F or c == 0x5C:
            out.append(b"\\x%02x" % c)
        else:
            out.append(bytes([c]))
    return b"".join(out)


def block_hashes(data, block_size, hash_name="blake2b/256"):
    """Hashes::hash_file: one digest per block_size chunk, none for b''."""
    h = HASHES[hash_name]
    return [h(data[i:i + block_size]) for i in range(0, len(data), block_size)]


def emit(hash_name, block_size, dirs, keep_empty=False):
    """dirs: list of (vpath bytes, [entries]) in emission order, entry =
    ('f', name, exe, size, [digests]) or ('s', name, target)."""
    header = b"DIRSIGNATURE.v1 %s block_size=%d\n" % (hash_name.encode(), block_size)
    body = []
    for vpath, entries in dirs:
        if not entries and not keep_empty:
            continue
        body.append(escape(vpath) + b"\n")
        for e in entries:
            if e[0] == "f":
                _, name, exe, size, digests = e
                line = b"  " + escape(name) + (b" x " if exe else b" f ") + str(size).encode()
                for d in digests:
                    line += b" " + d.hex().encode()
                body.append(line + b"\n")
            else:
                _, name, target = e
                body.append(b"  " + escape(name) + b" s " + escape(target) + b"\n")
    body = b"".join(body)
    footer = HASHES[hash_name](body).hex().encode() + b"\n"
    return header + body + footer


_DIR_FLAGS = os.O_RDONLY | os.O_DIRECTORY | getattr(os, "O_CLOEXEC", 0)


def open_rel(root, parts, flags=os.O_RDONLY):
    """fd of root/parts[0]/.../parts[-1] opened one component at a time
    relative to its parent's fd (openat), so a path of any length opens;
    directories below the root are not followed through symlinks."""
    fd = os.open(root, _DIR_FLAGS)
    try:
        for c in parts[:-1]:
            nfd = os.open(c, _DIR_FLAGS | os.O_NOFOLLOW, dir_fd=fd)
            os.close(fd)
            fd = nfd
        return os.open(parts[-1], flags | getattr(os, "O_CLOEXEC", 0), dir_fd=fd)
    finally:
        os.close(fd)


def walk(root):
    """The tree at `root` mounted at '/': [(vpath, [entries])] in emission
    order, file entries ('f', name, exe, size, real_path, parts) not yet
    hashed (parts: the path's components below root, for open_rel).

    Every directory is listed, lstat'ed and read-linked through its own fd
    (os.listdir(fd), os.stat(.., dir_fd=, follow_symlinks=False),
    os.readlink(.., dir_fd=)), each opened relative to its parent's, as
    dir-signature 0.2.9 walks with openat (Cargo.lock:323): a tree whose
    paths pass PATH_MAX indexes like any other."""
    dirs = []

    def rec(fd, parts, vpath):
        # os.listdir(fd) gives str names (surrogate-escaped): back to raw bytes
        names = sorted(os.fsencode(n) for n in os.listdir(fd))
        entries, subdirs = [], []
        base = os.path.join(os.fsencode(root), *parts) if parts else os.fsencode(root)
        for n in names:
            st = os.stat(n, dir_fd=fd, follow_symlinks=False)
            if stat.S_ISDIR(st.st_mode):
                subdirs.append(n)
            elif stat.S_ISREG(st.st_mode):
                entries.append(("f", n, bool(st.st_mode & 0o111), st.st_size,
                                os.path.join(base, n), parts + (n,)))
            elif stat.S_ISLNK(st.st_mode):
                entries.append(("s", n, os.readlink(n, dir_fd=fd)))
        dirs.append((vpath, entries))
        for n in subdirs:
            cfd = os.open(n, _DIR_FLAGS | os.O_NOFOLLOW, dir_fd=fd)
            try:
                rec(cfd, parts + (n,), (b"/" + n) if vpath == b"/" else vpath + b"/" + n)
            finally:
                os.close(cfd)

    top = os.open(root, _DIR_FLAGS)
    try:
        rec(top, (), b"/")
    finally:
        os.close(top)
    return dirs


def scan(root, block_size=32768, hash_name="blake2b/256", block_hasher=None, files_hasher=None):
    """Index bytes of the tree at `root` (mounted at '/').

    block_hasher(data, block_size) -> [digest, ...] replaces block_hashes
    per file; files_hasher(paths, sizes, block_size) -> [[digest, ...], ...]
    hashes every file at once (the threaded C restatement of the CPU
    indexer's file-level pool, oracle/blake2b_oracle.c oracle_hash_files).
    The footer is always hashlib's."""
    dirs = walk(root)
    files = [e for _, entries in dirs for e in entries if e[0] == "f"]
    if files_hasher is not None:
        digests = files_hasher([e[4] for e in files], [e[3] for e in files], block_size)
    else:
        hasher = block_hasher or (lambda data, bs: block_hashes(data, bs, hash_name))
        digests = []
        for e in files:
            with os.fdopen(open_rel(root, e[5]), "rb") as f:
                data = f.read()
            assert len(data) == e[3], "file changed during the scan"
            digests.append(hasher(data, block_size))
    it = iter(digests)
    out = [(vpath, [(e[0], e[1], e[2], e[3], next(it)) if e[0] == "f" else e for e in entries])
           for vpath, entries in dirs]
    return emit(hash_name, block_size, out, keep_empty=True)


def parse(index):
    """(hash_name, block_size, dirs, footer) of an index (test helper)."""
    lines = index.split(b"\n")
    assert lines[-1] == b""
    head = lines[0].split(b" ")
    assert head[0] == b"DIRSIGNATURE.v1"
    hash_name = head[1].decode()
    bs = int(head[2].split(b"=")[1])
    dirs = []
    for ln in lines[1:-2]:
        if ln.startswith(b"/"):
            dirs.append((ln, []))
        else:
            parts = ln[2:].split(b" ")
            if parts[1] in (b"f", b"x"):
                dirs[-1][1].append(("f", parts[0], parts[1] == b"x", int(parts[2]),
                                    [bytes.fromhex(x.decode()) for x in parts[3:]]))
            else:
                dirs[-1][1].append(("s", parts[0], parts[2]))
    return hash_name, bs, dirs, bytes.fromhex(lines[-2].decode())
