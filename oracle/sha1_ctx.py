"""SHA-1 context oracle -- TEST INFRASTRUCTURE ONLY.

A pure-Python restatement of the SHA_CTX that chunkio's cio_sha1 carries
(src/cio_sha1.c:26-57 over OpenSSL's API, include/chunkio/cio_sha1.h:25-27):
FIPS 180-4 SHA-1, with the context evolving as OpenSSL's md32_common.h
update/final leave it --

  h0..h4    chaining value
  Nl, Nh    message length in bits, low / high 32-bit words (mod 2^64)
  data      pending bytes of the partial block, raw, zero after `num`
  num       number of pending bytes (0..63)
  Final     pads (0x80, zeros, 64-bit big-endian bit count), then leaves the
            final chaining value and Nl/Nh, zeroes data and num

-- serialised as the 96 bytes of OpenSSL's struct SHAstate_st on LP64
(5 + 2 + 16 + 1 little-endian u32).  It is pinned against OpenSSL itself
(libcrypto through ctypes) and hashlib by tests/test_sha1_host.py, and lets
the SHA-1 state tests run where libcrypto cannot be loaded.  Pure Python:
for messages of up to a few hundred KB.
"""
import struct

_H0 = (0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0)
_M32 = 0xFFFFFFFF


def _rol(x, n):
    return ((x << n) | (x >> (32 - n))) & _M32


def _compress(h, block):
    """FIPS 180-4 §6.1.2 on one 64-byte block."""
    w = list(struct.unpack(">16I", block))
    for t in range(16, 80):
        w.append(_rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1))
    a, b, c, d, e = h
    for t in range(80):
        if t < 20:
            f, k = (b & c) | (~b & d), 0x5A827999
        elif t < 40:
            f, k = b ^ c ^ d, 0x6ED9EBA1
        elif t < 60:
            f, k = (b & c) | (b & d) | (c & d), 0x8F1BBCDC
        else:
            f, k = b ^ c ^ d, 0xCA62C1D6
        a, b, c, d, e = (_rol(a, 5) + (f & _M32) + e + k + w[t]) & _M32, a, _rol(b, 30), c, d
    return tuple((x + y) & _M32 for x, y in zip(h, (a, b, c, d, e)))


class Sha1Ctx:
    """SHA1_Init / SHA1_Update / SHA1_Final on an OpenSSL-layout context."""

    def __init__(self, raw=None):
        if raw is None:                          # SHA1_Init: all zero, then H0..H4
            self.h, self.nl, self.nh, self.data, self.num = _H0, 0, 0, bytes(64), 0
        else:
            v = struct.unpack("<5I2I64sI", bytes(raw))
            self.h, self.nl, self.nh, self.data, self.num = tuple(v[:5]), v[5], v[6], v[7], v[8]

    def update(self, msg):
        msg = bytes(msg)
        if not msg:
            return self
        bits = ((self.nh << 32) | self.nl) + 8 * len(msg)
        self.nl, self.nh = bits & _M32, (bits >> 32) & _M32
        pend = self.data[:self.num] + msg
        whole = len(pend) // 64 * 64
        for i in range(0, whole, 64):
            self.h = _compress(self.h, pend[i:i + 64])
        rest = pend[whole:]
        self.num = len(rest)
        self.data = rest + bytes(64 - len(rest))
        return self

    def final(self):
        bits = (self.nh << 32) | self.nl
        pad = self.data[:self.num] + b"\x80"
        pad += bytes((56 - len(pad)) % 64) + struct.pack(">Q", bits)
        for i in range(0, len(pad), 64):
            self.h = _compress(self.h, pad[i:i + 64])
        self.data, self.num = bytes(64), 0
        return struct.pack(">5I", *self.h)

    def raw(self):
        return struct.pack("<5I2I64sI", *self.h, self.nl, self.nh, self.data, self.num)
