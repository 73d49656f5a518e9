"""RSA signatures for DHT records (hivemind.dht.crypto.RSASignatureValidator replacement).

``cryptography`` is not available in this image, so RSA is implemented over Python integers:
keygen with Miller-Rabin primes, e = 65537, EMSA-PKCS1-v1_5 with a SHA-256 DigestInfo.  Signing
uses the CRT form (two half-size exponentiations), verification one exponentiation with e = 65537;
keygen runs once per process.
"""
from __future__ import annotations

import base64
import hashlib
import os
import secrets
import threading

_SHA256_PREFIX = bytes.fromhex("3031300d060960864801650304020105000420")
_SMALL_PRIMES = [p for p in range(3, 2000, 2) if all(p % q for q in range(3, int(p ** 0.5) + 1, 2))]


def _is_probable_prime(n: int, rounds: int = 24) -> bool:
    if n < 2:
        return False
    for p in _SMALL_PRIMES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = secrets.randbelow(n - 3) + 2
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = pow(x, 2, n)
            if x == n - 1:
                break
        else:
            return False
    return True


def _gen_prime(bits: int) -> int:
    while True:
        c = secrets.randbits(bits) | (1 << (bits - 1)) | (1 << (bits - 2)) | 1
        if _is_probable_prime(c):
            return c


class RSAPrivateKey:
    _process_wide = None
    _lock = threading.Lock()

    def __init__(self, bits: int | None = None):
        bits = bits or int(os.environ.get("DEDLOC_RSA_BITS", "1024"))
        e = 65537
        while True:
            p, q = _gen_prime(bits // 2), _gen_prime(bits // 2)
            if p == q:
                continue
            phi = (p - 1) * (q - 1)
            if phi % e:
                break
        self.n, self.e = p * q, e
        self.d = pow(e, -1, phi)
        self.k = (self.n.bit_length() + 7) // 8
        # CRT form of the private exponent (PKCS#1 RSAPrivateKey's dP, dQ, qInv): a signature is two
        # half-size exponentiations, ~3x faster than m^d mod n; the result is the same integer
        self.p, self.q = p, q
        self.dp, self.dq, self.qinv = self.d % (p - 1), self.d % (q - 1), pow(q, -1, p)

    @classmethod
    def process_wide(cls) -> "RSAPrivateKey":
        with cls._lock:
            if cls._process_wide is None:
                cls._process_wide = cls()
            return cls._process_wide

    def public_key(self) -> "RSAPublicKey":
        return RSAPublicKey(self.n, self.e)

    def sign(self, data: bytes) -> bytes:
        m = int.from_bytes(_emsa(data, self.k), "big")
        s1, s2 = pow(m, self.dp, self.p), pow(m, self.dq, self.q)
        return (s2 + self.q * ((s1 - s2) * self.qinv % self.p)).to_bytes(self.k, "big")


class RSAPublicKey:
    def __init__(self, n: int, e: int = 65537):
        self.n, self.e = n, e
        self.k = (n.bit_length() + 7) // 8

    def to_bytes(self) -> bytes:
        return b"rsa:" + base64.b64encode(self.n.to_bytes(self.k, "big"))

    @classmethod
    def from_bytes(cls, b: bytes) -> "RSAPublicKey":
        if not b.startswith(b"rsa:"):
            raise ValueError("not an RSA public key")
        return cls(int.from_bytes(base64.b64decode(b[4:]), "big"))

    def verify(self, data: bytes, sig: bytes) -> bool:
        if len(sig) != self.k:
            return False
        m = pow(int.from_bytes(sig, "big"), self.e, self.n)
        return m.to_bytes(self.k, "big") == _emsa(data, self.k)


def _emsa(data: bytes, k: int) -> bytes:
    t = _SHA256_PREFIX + hashlib.sha256(data).digest()
    if k < len(t) + 11:
        raise ValueError("key too small")
    return b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
