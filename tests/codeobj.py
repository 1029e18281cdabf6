"""Code objects of the built library (test helper, CPU only): the gfx950
ELF objects inside libciruela_amd.so's .hip_fatbin section (one clang
offload bundle per HIP translation unit), their disassembly and the
per-kernel resource metadata (registers, spills, LDS)."""
import os
import re
import struct
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ciruela_amd", "libciruela_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def available():
    return os.path.exists(LIB) and os.path.exists(os.path.join(LLVM, "llvm-objdump"))


def gfx950_objects(tmpdir, lib=LIB):
    fat = os.path.join(tmpdir, "fatbin.bin")
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section",
                           ".hip_fatbin=%s" % fat, lib, os.path.join(tmpdir, "lib_copy.so")])
    with open(fat, "rb") as f:
        data = f.read()
    objs, pos = [], 0
    while True:
        p = data.find(MAGIC, pos)
        if p < 0:
            break
        off = p + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, off)
        off += 8
        for _ in range(n):
            o, size, tlen = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tlen].decode()
            off += tlen
            if "gfx950" in triple and size:
                path = os.path.join(tmpdir, "co%d.elf" % len(objs))
                with open(path, "wb") as f:
                    f.write(data[p + o:p + o + size])
                objs.append(path)
        pos = p + len(MAGIC)
    return objs


def disassembly(tmpdir, with_addr=False):
    """{mangled kernel name: [instruction text without comments]}, or
    [(address, text)] with with_addr."""
    out = {}
    for obj in gfx950_objects(tmpdir):
        asm = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d",
                                       "--mcpu=gfx950", obj], text=True)
        name, body = None, []
        for line in asm.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
            if m:
                if name:
                    out[name] = body
                name, body = m.group(1), []
                continue
            ins = line.split("//")[0].strip()
            if name and ins:
                if with_addr:
                    m = re.search(r"//\s*([0-9A-Fa-f]+):", line)
                    body.append((int(m.group(1), 16) if m else None, ins))
                else:
                    body.append(ins)
        if name:
            out[name] = body
    return out


def resources(tmpdir):
    """{mangled kernel name: {vgpr_count, agpr_count, sgpr_count,
    vgpr_spill_count, sgpr_spill_count, group_segment_fixed_size, ...}}."""
    res = {}
    for obj in gfx950_objects(tmpdir):
        notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", obj],
                                        text=True)
        for entry in notes.split("  - .agpr_count:")[1:]:
            entry = ".agpr_count:" + entry
            fields = dict(re.findall(r"\.([a-z_]+):\s+(\S+)", entry))
            name = fields.get("name")
            if name and name.startswith("_Z"):
                res[name] = {k: int(v) for k, v in fields.items() if v.isdigit()}
    return res


def find(table, short):
    """Entries of a {mangled: ...} table whose name is cir::dev::<short>."""
    return {k: v for k, v in table.items() if re.search(r"\d%s[EI]" % re.escape(short), k)}
