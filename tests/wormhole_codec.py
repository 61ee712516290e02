"""Wormhole felt/byte codecs restated for test vectors.

Follows common/src/utils.rs:137-215 (u64_to_felts, injective_string_to_felt,
injective_bytes_to_felts, digest_bytes_to_felts, digest_felts_to_bytes) and
common/src/utils.rs:104-113 (u128_to_felts).
"""
import struct


def injective_bytes_to_felts(b):
    out = []
    for i in range(0, len(b), 4):
        c = b[i:i + 4]
        c = c + b"\0" * (4 - len(c))
        out.append(struct.unpack("<I", c)[0])
    return out


def injective_string_to_felt(s):
    b = s.encode()
    assert len(b) == 8
    return injective_bytes_to_felts(b)


def u64_to_felts(x):
    return [(x >> 32) & 0xFFFFFFFF, x & 0xFFFFFFFF]


def u128_to_felts(x):
    return [(x >> (96 - 32 * i)) & 0xFFFFFFFF for i in range(4)]


def digest_bytes_to_felts(b):
    return [struct.unpack("<Q", b[8 * i:8 * i + 8])[0] for i in range(4)]


def digest_felts_to_bytes(d):
    return b"".join(struct.pack("<Q", x) for x in d)
