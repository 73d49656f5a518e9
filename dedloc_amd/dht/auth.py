"""Token-based access control for the collaboration.

The reference's sahajBERT volunteers obtain a signed access token from the Hugging Face auth server
(``sahajbert/huggingface_auth.py:46-171``: login -> PUT /api/experiments/join/{id} with the peer's
public key -> ``AccessToken{username, public_key, expiration_time, signature}`` signed by the
authority, verified by every peer, refreshed one minute before expiry) and hivemind's
``TokenAuthorizerBase`` interface wires it into the network layer.

There is no network here, so the authority is local (``LocalAuthority``: an RSA key, an allowlist,
coordinator address, token lifetime); ``LocalTokenAuthorizer`` is the client side with the same
behaviour as the reference authorizer (join with retries, validate signature + expiry, refresh
before expiry).  Tokens enter the control plane through ``AuthorizedRecordValidator``: every record a
peer writes carries its access token, and readers drop records whose token is missing, forged,
expired, or issued for a different public key than the record's ``[owner:...]`` marker.
"""
from __future__ import annotations

import base64
import time
from dataclasses import dataclass
from datetime import datetime, timedelta
from typing import Callable, Dict, Iterable, Optional

import msgpack

from .crypto import RSAPrivateKey, RSAPublicKey
from .validation import _OWNER_RE, _TOKEN_RE, RecordValidatorBase, strip_token


@dataclass
class AccessToken:
    username: str
    public_key: bytes
    expiration_time: str  # ISO-8601, naive UTC (reference: str(datetime))
    signature: bytes = b""

    def payload(self) -> bytes:
        return f"{self.username} {self.public_key.decode()} {self.expiration_time}".encode()

    def to_bytes(self) -> bytes:
        return msgpack.packb([self.username, self.public_key, self.expiration_time, self.signature])

    @classmethod
    def from_bytes(cls, b: bytes) -> "AccessToken":
        u, pk, exp, sig = msgpack.unpackb(b)
        return cls(u, pk, exp, sig)


class NonRetriableError(Exception):
    pass


class InvalidCredentialsError(NonRetriableError):
    pass


class NotInAllowlistError(NonRetriableError):
    pass


def call_with_retries(func, n_retries: int = 10, initial_delay: float = 1.0):
    """Exponential backoff; authorization failures are not retried (huggingface_auth.py:23-35)."""
    for i in range(n_retries):
        try:
            return func()
        except NonRetriableError:
            raise
        except Exception:  # noqa: BLE001
            if i == n_retries - 1:
                raise
            time.sleep(initial_delay * (2 ** i))


class LocalAuthority:
    """Offline stand-in for the experiment's auth server: checks credentials + allowlist, signs tokens."""

    def __init__(self, allowlist: Dict[str, str], coordinator: str = "127.0.0.1:0", ttl: float = 3600.0,
                 key: Optional[RSAPrivateKey] = None):
        self.allowlist = dict(allowlist)  # username -> password
        self.coordinator = coordinator
        self.ttl = ttl
        self.key = key or RSAPrivateKey(bits=1024)
        self.public_key = self.key.public_key()

    def join_experiment(self, username: str, password: str, peer_public_key: bytes) -> Dict:
        if username not in self.allowlist:
            raise NotInAllowlistError(username)
        if self.allowlist[username] != password:
            raise InvalidCredentialsError(username)
        exp = (datetime.utcnow() + timedelta(seconds=self.ttl)).isoformat()
        token = AccessToken(username, peer_public_key, exp)
        token.signature = base64.b64encode(self.key.sign(token.payload()))
        ip, _, port = self.coordinator.partition(":")
        return {"auth_server_public_key": self.public_key.to_bytes(), "coordinator_ip": ip,
                "coordinator_port": int(port or 0), "hivemind_access": token}


class TokenAuthorizerBase:
    """hivemind.utils.auth.TokenAuthorizerBase interface: get_token / is_token_valid / refresh."""

    def __init__(self, local_private_key: Optional[RSAPrivateKey] = None):
        self._local_private_key = local_private_key or RSAPrivateKey.process_wide()
        self.local_public_key = self._local_private_key.public_key()
        self._local_access_token: Optional[AccessToken] = None

    def get_token(self) -> AccessToken:
        raise NotImplementedError

    def is_token_valid(self, access_token: AccessToken) -> bool:
        raise NotImplementedError

    def does_token_need_refreshing(self, access_token: AccessToken) -> bool:
        raise NotImplementedError

    def local_access_token(self) -> AccessToken:
        tok = self._local_access_token
        if tok is None or self.does_token_need_refreshing(tok):
            tok = self._local_access_token = self.get_token()
        return tok


class LocalTokenAuthorizer(TokenAuthorizerBase):
    _MAX_LATENCY = timedelta(minutes=1)

    def __init__(self, authority: LocalAuthority, username: str, password: str,
                 local_private_key: Optional[RSAPrivateKey] = None):
        super().__init__(local_private_key)
        self.authority, self.username, self.password = authority, username, password
        self._authority_public_key: Optional[RSAPublicKey] = None
        self.coordinator_ip = self.coordinator_port = None

    def join_experiment(self):
        call_with_retries(self._join_experiment)

    def _join_experiment(self):
        resp = self.authority.join_experiment(self.username, self.password, self.local_public_key.to_bytes())
        self._authority_public_key = RSAPublicKey.from_bytes(resp["auth_server_public_key"])
        self.coordinator_ip, self.coordinator_port = resp["coordinator_ip"], resp["coordinator_port"]
        self._local_access_token = resp["hivemind_access"]

    def get_token(self) -> AccessToken:
        self.join_experiment()
        return self._local_access_token

    def is_token_valid(self, access_token: AccessToken) -> bool:
        if self._authority_public_key is None:
            self.join_experiment()
        try:
            sig = base64.b64decode(access_token.signature)
        except Exception:  # noqa: BLE001
            return False
        if not self._authority_public_key.verify(access_token.payload(), sig):
            return False
        try:
            exp = datetime.fromisoformat(access_token.expiration_time)
        except ValueError:
            return False
        if exp.tzinfo is not None:
            return False
        return exp >= datetime.utcnow()

    def does_token_need_refreshing(self, access_token: AccessToken) -> bool:
        return datetime.fromisoformat(access_token.expiration_time) < datetime.utcnow() + self._MAX_LATENCY


class AuthorizedRecordValidator(RecordValidatorBase):
    """Every written record carries the writer's access token; invalid / foreign tokens are dropped."""

    priority = 5  # after the schema check, before the RSA signature (which then also covers the token)

    def __init__(self, authorizer: TokenAuthorizerBase):
        self.authorizer = authorizer

    def sign_value(self, key, subkey, value, expiration=None):
        tok = self.authorizer.local_access_token()
        return value + b"[token:" + base64.b64encode(tok.to_bytes()) + b"]"

    def strip_value(self, key, subkey, value):
        return strip_token(value)

    def validate(self, key, subkey, value, expiration):
        m = None
        for m in _TOKEN_RE.finditer(value):
            pass
        if m is None:
            return False
        try:
            tok = AccessToken.from_bytes(base64.b64decode(m.group(1)))
        except Exception:  # noqa: BLE001
            return False
        if not self.authorizer.is_token_valid(tok):
            return False
        for part in (key, subkey or b""):
            own = _OWNER_RE.search(part)
            if own is not None and own.group(1) != tok.public_key:
                return False  # a token issued to someone else cannot authorize this owner's record
        return True


def authorized_validators(authorizer: TokenAuthorizerBase, validators: Iterable[RecordValidatorBase] = ()):
    return list(validators) + [AuthorizedRecordValidator(authorizer)]
