"""Keccak-256 in Python ints, independent of the C oracle (TEST INFRASTRUCTURE ONLY).

Keccak256Write / Keccak256Read (halo2_backend/src/transcript.rs:109-463) hash with the
`sha3` crate's Keccak256: Keccak-f[1600], rate 136 bytes, output 32 bytes and the
original Keccak padding (0x01 ... 0x80), not SHA3's 0x06.  The permutation is pinned
by running this sponge with pad 0x06 against hashlib.sha3_256; the padding by the
public constant Keccak-256("") = c5d24601...5d85a470 (tests/test_keccak_transcript.py).
"""

_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_M = (1 << 64) - 1


def _rot(v, r):
    return ((v << r) | (v >> (64 - r))) & _M if r else v


def _rho_offsets():
    """r[x][y] from the (x, y) -> (y, 2x + 3y) walk of FIPS 202 3.2.2"""
    r = [[0] * 5 for _ in range(5)]
    x, y = 1, 0
    for t in range(24):
        r[x][y] = ((t + 1) * (t + 2) // 2) % 64
        x, y = y, (2 * x + 3 * y) % 5
    return r


_R = _rho_offsets()


def keccak_f(a):
    """a: 25 lanes, a[x + 5 y]"""
    for rc in _RC:
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rot(c[(x + 1) % 5], 1) for x in range(5)]
        a = [a[i] ^ d[i % 5] for i in range(25)]
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = _rot(a[x + 5 * y], _R[x][y])
        a = [b[i] ^ (~b[(i % 5 + 1) % 5 + 5 * (i // 5)] & b[(i % 5 + 2) % 5 + 5 * (i // 5)]) & _M
             for i in range(25)]
        a[0] ^= rc
    return a


class Keccak:
    RATE = 136

    def __init__(self, pad=0x01):
        self.pad = pad
        self.a = [0] * 25
        self.buf = b""

    def copy(self):
        k = Keccak(self.pad)
        k.a = list(self.a)
        k.buf = self.buf
        return k

    def _absorb(self, blk):
        for i in range(17):
            self.a[i] ^= int.from_bytes(blk[8 * i:8 * i + 8], "little")
        self.a = keccak_f(self.a)

    def update(self, data):
        self.buf += bytes(data)
        while len(self.buf) >= self.RATE:
            self._absorb(self.buf[:self.RATE])
            self.buf = self.buf[self.RATE:]
        return self

    def digest(self):
        k = self.copy()
        blk = bytearray(k.buf + bytes(self.RATE - len(k.buf)))
        blk[len(k.buf)] ^= k.pad
        blk[-1] ^= 0x80
        k._absorb(bytes(blk))
        return b"".join(v.to_bytes(8, "little") for v in k.a[:4])


def keccak256(data):
    return Keccak(0x01).update(data).digest()
