"""Control plane: replicated native DHT + record validators (hivemind.DHT equivalent)."""
from .node import DHT, DHTClient, NativeServer, ValueWithExpiration, get_dht_time, parse_endpoint  # noqa: F401
from .validation import (  # noqa: F401
    BytesWithPublicKey, CompositeValidator, RecordValidatorBase, RSASignatureValidator, SchemaValidator,
)
