"""DHT record validators (hivemind.dht.validation / schema / crypto equivalents).

* ``RSASignatureValidator`` — a record whose key or subkey carries ``[owner:<public key>]`` must be
  signed by that key; the signature travels appended to the serialized value
  (``...[signature:<b64>]``) and covers (key, subkey, value, expiration).  Only the owner can write
  its own entry (used for ``{prefix}_metrics`` / ``{prefix}_progress``, metrics_utils.py:21-24).
* ``SchemaValidator(Model, prefix)`` — records under ``f"{prefix}_{field}"`` must match the pydantic
  field type (``Dict[BytesWithPublicKey, LocalMetrics]`` -> subkey must carry an owner marker and
  the value must parse as ``LocalMetrics``).
* validators compose in order (``CompositeValidator``): signing happens on store, validation on
  store and on every read (a record that fails validation is invisible to the reader).
"""
from __future__ import annotations

import base64
import re
import struct
import typing
from typing import Any, Dict, Iterable, List, Optional

import msgpack

from .crypto import RSAPrivateKey, RSAPublicKey

_SIG_RE = re.compile(rb"\[signature:([A-Za-z0-9+/=]+)\]$")
_TOKEN_RE = re.compile(rb"\[token:([A-Za-z0-9+/=]+)\]")  # access-token marker (dht/auth.py)


def strip_token(value: bytes) -> bytes:
    """Remove the last ``[token:...]`` marker (appended by AuthorizedRecordValidator)."""
    m = None
    for m in _TOKEN_RE.finditer(value):
        pass
    return value if m is None else value[:m.start()] + value[m.end():]
_OWNER_RE = re.compile(rb"\[owner:(rsa:[A-Za-z0-9+/=]+)\]")


class BytesWithPublicKey(bytes):
    """Marker type: a subkey that must embed an ``[owner:...]`` public key."""

    @classmethod
    def __get_pydantic_core_schema__(cls, source, handler):
        from pydantic_core import core_schema

        def check(v):
            if not isinstance(v, (bytes, bytearray)) or _OWNER_RE.search(bytes(v)) is None:
                raise ValueError("subkey must contain [owner:<public key>]")
            return bytes(v)

        return core_schema.no_info_plain_validator_function(check)


class RecordValidatorBase:
    priority = 0

    def validate(self, key: bytes, subkey: Optional[bytes], value: bytes, expiration: float) -> bool:
        return True

    def sign_value(self, key: bytes, subkey: Optional[bytes], value: bytes, expiration: float | None = None) -> bytes:
        return value

    def strip_value(self, key: bytes, subkey: Optional[bytes], value: bytes) -> bytes:
        return value


def _split_sig(value: bytes):
    m = _SIG_RE.search(value)
    if m is None:
        return value, None
    return value[:m.start()], base64.b64decode(m.group(1))


class RSASignatureValidator(RecordValidatorBase):
    priority = 10  # signs last, validates first

    def __init__(self, private_key: Optional[RSAPrivateKey] = None):
        self._key = private_key or RSAPrivateKey.process_wide()
        self._pub = self._key.public_key().to_bytes()
        self.local_public_key = b"[owner:" + self._pub + b"]"

    @staticmethod
    def _owner(key: bytes, subkey: Optional[bytes]) -> Optional[bytes]:
        for part in (key, subkey or b""):
            m = _OWNER_RE.search(part)
            if m:
                return m.group(1)
        return None

    @staticmethod
    def _payload(key, subkey, value, expiration):
        # the expiration is signed in its exact wire form (the float64 the server stores), so a
        # replayed record cannot be given a later expiration to pin a stale owner's state
        return b"|".join((key, subkey or b"", value, struct.pack("<d", float(expiration))))

    def sign_value(self, key, subkey, value, expiration=None):
        owner = self._owner(key, subkey)
        if owner is None or owner != self._pub:
            return value
        if expiration is None:
            raise ValueError("signing an owned record needs its expiration time")
        sig = self._key.sign(self._payload(key, subkey, value, expiration))
        return value + b"[signature:" + base64.b64encode(sig) + b"]"

    def strip_value(self, key, subkey, value):
        return _split_sig(value)[0]

    def validate(self, key, subkey, value, expiration):
        owner = self._owner(key, subkey)
        if owner is None:
            return True
        body, sig = _split_sig(value)
        if sig is None:
            return False
        try:
            return RSAPublicKey.from_bytes(owner).verify(self._payload(key, subkey, body, expiration), sig)
        except Exception:  # noqa: BLE001
            return False


class SchemaValidator(RecordValidatorBase):
    priority = 0

    def __init__(self, schema, prefix: Optional[str] = None, allow_extra_keys: bool = True):
        self.schema = schema
        self.prefix = prefix
        self.allow_extra_keys = allow_extra_keys
        self.fields: Dict[bytes, Any] = {}
        for name, f in schema.model_fields.items():
            key = f"{prefix}_{name}" if prefix else name
            self.fields[key.encode()] = f.annotation

    def validate(self, key, subkey, value, expiration):
        ftype = self.fields.get(key)
        if ftype is None:
            return self.allow_extra_keys
        body = strip_token(_split_sig(value)[0])
        try:
            obj = msgpack.unpackb(body, raw=False)
        except Exception:  # noqa: BLE001
            return False
        origin = typing.get_origin(ftype)
        try:
            if origin in (dict, Dict):
                kt, vt = typing.get_args(ftype)
                if subkey is None:
                    return False
                if kt is BytesWithPublicKey and _OWNER_RE.search(subkey) is None:
                    return False
                if obj is None:  # tombstone
                    return True
                return _check(vt, obj)
            if subkey is not None:
                return False
            return _check(ftype, obj)
        except Exception:  # noqa: BLE001
            return False


def _check(tp, obj) -> bool:
    if hasattr(tp, "model_validate"):
        tp.model_validate(obj, strict=False)
        return True
    from pydantic import TypeAdapter

    TypeAdapter(tp).validate_python(obj)
    return True


class CompositeValidator(RecordValidatorBase):
    def __init__(self, validators: Iterable[RecordValidatorBase] = ()):
        self.validators: List[RecordValidatorBase] = sorted(validators, key=lambda v: v.priority)

    def sign_value(self, key, subkey, value, expiration=None):
        for v in self.validators:  # ascending priority: the signature is appended last
            value = v.sign_value(key, subkey, value, expiration)
        return value

    def strip_value(self, key, subkey, value):
        for v in reversed(self.validators):
            value = v.strip_value(key, subkey, value)
        return value

    def validate(self, key, subkey, value, expiration):
        return all(v.validate(key, subkey, value, expiration) for v in reversed(self.validators))
