"""Generate the golden vectors under tests/golden/ (run once, output committed).

The reference pins nothing about BLAKE2b-256 itself: its block
ids are `Blake2b::VariableOutput::new(32)` of the `blake2 0.7.1` crate
(src/block_id.rs:37-43), an RFC 7693 implementation that is not vendored.
The vectors here are computed with Python's stdlib `hashlib.blake2b(...,
digest_size=32)` (RFC 7693, digest length in the parameter block), which
this script first checks against RFC 7693 Appendix A.

Inputs are described by small generator specs (see `gen_bytes`) so the
fixture stays tiny; tests regenerate the bytes the same way.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

RFC7693_ABC_512 = (
    "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
    "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923")


def splitmix64_words(seed, nwords, first=0):
    out = []
    mask = (1 << 64) - 1
    for k in range(first, first + nwords):
        z = (seed + (k + 1) * 0x9E3779B97F4A7C15) & mask
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & mask
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & mask
        out.append(z ^ (z >> 31))
    return out


def gen_bytes(spec):
    """Regenerate the input bytes of one vector."""
    kind, n = spec["gen"], spec["n"]
    if kind == "zeros":
        return bytes(n)
    if kind == "range":  # bytes(range(256)) repeated
        return bytes(i & 255 for i in range(n))
    if kind == "ascii":
        return spec["text"].encode()
    if kind == "splitmix64":  # little-endian words of splitmix64(seed)
        words = splitmix64_words(spec["seed"], (n + 7) // 8)
        return struct.pack("<%dQ" % len(words), *words)[:n]
    raise ValueError(kind)


def b2(data):
    return hashlib.blake2b(data, digest_size=32).hexdigest()


def main():
    assert hashlib.blake2b(b"abc").hexdigest() == RFC7693_ABC_512, "hashlib is not RFC 7693"
    specs = []
    specs.append({"gen": "ascii", "n": 0, "text": ""})
    specs.append({"gen": "ascii", "n": 3, "text": "abc"})
    specs.append({"gen": "ascii", "n": 7, "text": "Hidden\n"})
    # every length around the 128-byte compression boundary, and tails
    for n in list(range(0, 260)) + [383, 384, 385, 1000, 4095, 4096, 4097, 8191, 8192,
                                     32767, 32768, 32769, 65536, 100000]:
        specs.append({"gen": "range", "n": n})
    for n in [1, 127, 128, 129, 4096, 32768, 32768 + 1, 1 << 20]:
        specs.append({"gen": "zeros", "n": n})
    for i, n in enumerate([1, 8, 100, 128, 4096, 12345, 32768, 1 << 20]):
        specs.append({"gen": "splitmix64", "n": n, "seed": 0x5EED0000 + i})
    vectors = []
    for s in specs:
        v = dict(s)
        v["blake2b256"] = b2(gen_bytes(s))
        vectors.append(v)
    # Config 2: blocks 0-15 all-zero, 16-31 bytes(range(256))*128
    config2 = {
        "block_size": 32768,
        "zero_block": b2(bytes(32768)),
        "range_block": b2(bytes(range(256)) * 128),
    }
    out = {
        "about": "BLAKE2b-256 (RFC 7693, nn=32, unkeyed) vectors from hashlib; "
                 "see tests/golden/make_golden.py",
        "rfc7693_appendix_a_blake2b512_abc": RFC7693_ABC_512,
        "vectors": vectors,
        "config2": config2,
    }
    with open(os.path.join(HERE, "blake2b256_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(vectors), "vectors")


if __name__ == "__main__":
    main()
