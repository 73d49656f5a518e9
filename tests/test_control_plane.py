"""Control-plane unit tests (CPU): DHT semantics, record validators, RSA, LP load balancing vs brute force,
Hagenbach-Bischoff rounding, PerformanceEMA, argument surface (SURVEY.md §4 "Unit tests (CPU)")."""
import itertools
import time

import numpy as np
import pytest

from dedloc_amd.averaging.load_balancing import hagenbach_bischoff, load_balance_peers, optimize_parts_lp
from dedloc_amd.dht import DHT, get_dht_time
from dedloc_amd.dht.crypto import RSAPrivateKey, RSAPublicKey
from dedloc_amd.dht.validation import RSASignatureValidator, SchemaValidator
from dedloc_amd.metrics import LocalMetrics, MetricSchema, make_validators
from dedloc_amd.optim.performance_ema import PerformanceEMA


@pytest.fixture
def dht():
    d = DHT(start=True)
    yield d
    d.shutdown()


# ----------------------------------------------------------------------------- DHT
def test_dht_store_get_plain_and_expiration(dht):
    now = get_dht_time()
    assert dht.store("k", {"a": 1}, now + 30)
    v = dht.get("k", latest=True)
    assert v.value == {"a": 1} and abs(v.expiration_time - (now + 30)) < 1e-6
    # an older record does not replace a newer one; a newer one does
    assert not dht.store("k", "older", now + 10) or dht.get("k").value == {"a": 1}
    assert dht.get("k").value == {"a": 1}
    dht.store("k", "newer", now + 60)
    assert dht.get("k").value == "newer"
    # already-expired records are never returned
    dht.store("gone", 1, now - 1)
    assert dht.get("gone") is None
    dht.store("short", 1, get_dht_time() + 0.3)
    assert dht.get("short").value == 1
    time.sleep(0.5)
    assert dht.get("short") is None


def test_dht_subkeys_merge_and_expire(dht):
    now = get_dht_time()
    dht.store("progress", {"step": 1}, now + 30, subkey=b"peer-a")
    dht.store("progress", {"step": 2}, now + 0.3, subkey=b"peer-b")
    v = dht.get("progress", latest=True)
    assert set(v.value) == {b"peer-a", b"peer-b"}
    assert v.value[b"peer-a"].value == {"step": 1}
    time.sleep(0.5)
    v = dht.get("progress", latest=True)
    assert set(v.value) == {b"peer-a"}
    # per-subkey freshness: a newer value for the same subkey wins
    dht.store("progress", {"step": 5}, now + 40, subkey=b"peer-a")
    assert dht.get("progress").value[b"peer-a"].value == {"step": 5}


def test_dht_replication_between_nodes():
    a = DHT(start=True)
    b = DHT(initial_peers=[a.endpoint], start=True)
    c = DHT(initial_peers=[b.endpoint], client_mode=True, start=True)  # client: no server of its own
    try:
        now = get_dht_time()
        b.store("x", 42, now + 30)
        assert a.get("x").value == 42
        c.store("y", "from-client", now + 30)
        assert a.get("y").value == "from-client" and b.get("y").value == "from-client"
        assert c.endpoint is None and c.port == b.port
        assert b.primary().endpoint == a.endpoint  # the oldest replica coordinates matchmaking
    finally:
        for n in (c, b, a):
            n.shutdown()


def test_dht_needs_listen_or_peers():
    with pytest.raises(ValueError):
        DHT(client_mode=True, start=True)


def test_dht_matchmaking_forms_one_group(dht):
    import threading

    out = {}

    def join(i):
        out[i] = dht.join_group(b"grp", f"p{i}".encode(), {"rank": i}, target_size=3, min_size=2, expected_size=3,
                                window=5.0, timeout=10.0)

    ts = [threading.Thread(target=join, args=(i,)) for i in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    gids = {out[i][1] for i in range(3)}
    assert all(out[i][0] for i in range(3)) and len(gids) == 1
    assert sorted(m[1]["rank"] for m in out[0][2]) == [0, 1, 2]


def test_dht_matchmaking_small_groups_alternate_partitions(dht):
    """target_group_size < peers (SwAV: groups of 4 out of 8): every round gathers all expected peers
    and splits them; even rounds take contiguous blocks of the peer-id order, odd rounds stride
    classes, so two rounds of equal-weight averaging mix the whole collaboration (Moshpit), and an
    always-early subset can no longer average only among itself."""
    import threading

    def one_round():
        out = {}

        def join(i):
            time.sleep(0.01 * (7 - i))  # arrival order is the reverse of the peer-id order
            out[i] = dht.join_group(b"moshpit", f"p{i}".encode(), {"rank": i}, target_size=4, min_size=2,
                                    expected_size=8, window=5.0, timeout=10.0)

        ts = [threading.Thread(target=join, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert all(out[i][0] for i in range(8))
        groups = {}
        for i in range(8):
            ranks = tuple(sorted(m[1]["rank"] for m in out[i][2]))
            assert i in ranks and len(ranks) == 4
            groups.setdefault(out[i][1], set()).add(ranks)
        assert len(groups) == 2 and all(len(v) == 1 for v in groups.values())  # one member list per group id
        return sorted(next(iter(v)) for v in groups.values())

    r0, r1, r2 = one_round(), one_round(), one_round()
    assert r0 == [(0, 1, 2, 3), (4, 5, 6, 7)]
    assert r1 == [(0, 2, 4, 6), (1, 3, 5, 7)]
    assert r2 == r0
    # two rounds of plain averaging in these groups give every peer the global mean
    x = np.arange(8, dtype=np.float64)
    for part in (r0, r1):
        for grp in part:
            x[list(grp)] = x[list(grp)].mean()
    assert np.allclose(x, 3.5)


def test_dht_matchmaking_duplicate_join_fails_the_open_round(dht):
    """A peer that re-joins a round it already waits in (it gave up on it client-side) fails that round
    for everybody in it instead of leaving them blocked, and starts a fresh one."""
    import threading

    out = {}

    def join(tag, peer, timeout):
        try:
            out[tag] = dht.join_group(b"dup", peer, {}, target_size=4, min_size=2, expected_size=3, window=30.0,
                                      timeout=timeout)
        except OSError as e:  # the re-joined peer waits alone in the fresh round until its own timeout
            out[tag] = e

    t1 = threading.Thread(target=join, args=("a", b"p0", 20.0))
    t1.start()
    time.sleep(0.3)
    t2 = threading.Thread(target=join, args=("b", b"p0", 2.0))  # the same peer again: round 1 fails
    t2.start()
    t1.join(timeout=15)
    assert not t1.is_alive() and out["a"][0] is False
    t2.join(timeout=15)


# ----------------------------------------------------------------------------- crypto + validators
def test_rsa_sign_verify_roundtrip():
    k = RSAPrivateKey(bits=1024)
    pub = RSAPublicKey.from_bytes(k.public_key().to_bytes())
    sig = k.sign(b"hello")
    assert pub.verify(b"hello", sig)
    assert not pub.verify(b"hellO", sig)
    other = RSAPrivateKey(bits=1024)
    assert not RSAPublicKey.from_bytes(other.public_key().to_bytes()).verify(b"hello", sig)


def test_rsa_crt_signature_equals_plain_exponentiation():
    """CRT signing (two half-size exponentiations, dht/crypto.py) yields the PKCS#1 v1.5 signature
    m^d mod n byte for byte."""
    from dedloc_amd.dht.crypto import _emsa

    k = RSAPrivateKey(bits=1024)
    for msg in (b"", b"x" * 200, bytes(range(256))):
        m = int.from_bytes(_emsa(msg, k.k), "big")
        assert k.sign(msg) == pow(m, k.d, k.n).to_bytes(k.k, "big")


def test_signature_validator_owner_only():
    owner = RSASignatureValidator(RSAPrivateKey(bits=1024))
    intruder = RSASignatureValidator(RSAPrivateKey(bits=1024))
    key, sub, val, exp = b"exp_metrics", owner.local_public_key, b"payload", 1234.5
    signed = owner.sign_value(key, sub, val, exp)
    assert owner.validate(key, sub, signed, exp) and intruder.validate(key, sub, signed, exp)
    forged = intruder.sign_value(key, sub, val, exp)  # intruder cannot sign for someone else's subkey
    assert forged == val and not owner.validate(key, sub, forged, exp)
    tampered = signed.replace(b"payload", b"paylaod")
    assert not owner.validate(key, sub, tampered, exp)
    assert owner.strip_value(key, sub, signed) == val
    assert owner.validate(b"public_key", None, b"anything", 0)  # unowned records are not signature-checked
    # the signature covers the expiration: a replayed record with a later expiration is rejected
    assert not owner.validate(key, sub, signed, exp + 1e6)
    assert not owner.validate(key, sub, signed, exp + 1e-9 * exp)


def test_replayed_record_with_extended_expiration_is_rejected_by_dht():
    """replaying an owner's signed record with a far-future expiration must not pin it."""
    from dedloc_amd.dht import DHT, get_dht_time
    from dedloc_amd.dht.node import _b

    owner_v = RSASignatureValidator(RSAPrivateKey(bits=1024))
    root = DHT(listen_on="127.0.0.1:*", record_validators=[owner_v])
    try:
        sub = owner_v.local_public_key
        exp = get_dht_time() + 30
        assert root.store("exp_progress", {"step": 1}, exp, subkey=sub)
        got = root.get("exp_progress", latest=True)
        assert got is not None and got.value[sub].value == {"step": 1}
        # an attacker copies the signed bytes and re-stores them directly with a later expiration
        kb, sb = _b("exp_progress"), _b(sub)
        import msgpack

        body = owner_v.sign_value(kb, sb, msgpack.packb({"step": 0}, use_bin_type=True), exp - 10)
        root._raw_store_all(kb, sb, body, get_dht_time() + 1e6)  # replay of an older record, expiration bumped
        got = root.get("exp_progress", latest=True)
        # the replay wins the latest-expiration merge on the server but fails validation on read
        assert got is None or sub not in got.value or got.value[sub].value != {"step": 0}
    finally:
        root.shutdown()


def test_schema_validator_metrics_records():
    import msgpack

    v = SchemaValidator(MetricSchema, prefix="exp")
    sub = b"[owner:rsa:QUJD]"
    good = LocalMetrics(step=1, samples_per_second=2.0, samples_accumulated=3, loss=0.5, mini_steps=1).model_dump()
    assert v.validate(b"exp_metrics", sub, msgpack.packb(good), 0)
    bad = dict(good, step=-1)
    assert not v.validate(b"exp_metrics", sub, msgpack.packb(bad), 0)
    assert not v.validate(b"exp_metrics", b"no-owner-marker", msgpack.packb(good), 0)
    assert not v.validate(b"exp_metrics", None, msgpack.packb(good), 0)  # dict field requires a subkey
    assert v.validate(b"unrelated_key", None, msgpack.packb("x"), 0)


def test_metrics_end_to_end_through_dht():
    validators, pub = make_validators("exp")
    d = DHT(start=True, record_validators=validators)
    try:
        m = LocalMetrics(step=3, samples_per_second=10.0, samples_accumulated=7, loss=1.5, mini_steps=2)
        assert d.store("exp_metrics", m.model_dump(), get_dht_time() + 30, subkey=pub)
        assert not d.store("exp_metrics", {"step": "x"}, get_dht_time() + 30, subkey=pub)
        rec = d.get("exp_metrics", latest=True)
        assert LocalMetrics(**rec.value[pub].value) == m
    finally:
        d.shutdown()


# ----------------------------------------------------------------------------- load balancing
def _cost(w, b):
    n = len(b)
    return max((1 + (n - 2) * wi) / bi for wi, bi in zip(w, b) if bi > 0)


@pytest.mark.parametrize("seed", range(6))
def test_lp_matches_brute_force(seed):
    rng = np.random.default_rng(seed)
    n = 3 + seed % 2
    b = rng.uniform(10, 1000, size=n)
    parts = optimize_parts_lp(10_000, list(b))
    assert parts.sum() == 10_000 and (parts >= 0).all()
    lp_cost = _cost(parts / 10_000, b)
    grid = np.linspace(0, 1, 41)
    best = min(_cost(w + (1 - sum(w),), b) for w in itertools.product(grid, repeat=n - 1) if sum(w) <= 1 + 1e-12)
    assert lp_cost <= best + 1e-3 * best


def test_lp_client_mode_gets_zero_share_and_uniform_when_equal():
    parts = load_balance_peers(1000, [100.0, 0.0, 100.0, 100.0])
    assert parts[1] == 0 and sum(parts) == 1000
    assert load_balance_peers(999, [5.0, 5.0, 5.0]) == (333, 333, 333)
    assert sum(load_balance_peers(7, [None, 10.0])) == 7


def test_hagenbach_bischoff():
    parts = hagenbach_bischoff(10, np.array([0.333, 0.333, 0.334]))
    assert parts.sum() == 10 and sorted(parts.tolist()) == [3, 3, 4]
    rng = np.random.default_rng(0)
    for _ in range(20):
        f = rng.dirichlet(np.ones(5))
        total = int(rng.integers(1, 10_000))
        p = hagenbach_bischoff(total, f)
        assert p.sum() == total and np.all(np.abs(p - f * total) < 1.0 + 1e-9)


# ----------------------------------------------------------------------------- PerformanceEMA
class FakeClock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def test_performance_ema_constant_rate_and_pause():
    clk = FakeClock()
    ema = PerformanceEMA(alpha=0.1, clock=clk)
    for _ in range(10):
        clk.t += 2.0
        sps = ema.update(8)
    assert sps == pytest.approx(4.0)  # bias-corrected: exact from the first update on
    with ema.pause():
        clk.t += 100.0  # averaging time is excluded
    clk.t += 2.0
    assert ema.update(8) == pytest.approx(4.0)
    with pytest.raises(AssertionError):
        with ema.pause():
            ema.update(1)


def test_performance_ema_tracks_rate_change():
    clk = FakeClock()
    ema = PerformanceEMA(alpha=0.5, clock=clk)
    for _ in range(30):
        clk.t += 1.0
        ema.update(10)
    for _ in range(30):
        clk.t += 1.0
        ema.update(20)
    assert ema.samples_per_second == pytest.approx(20.0, rel=1e-3)


# ----------------------------------------------------------------------------- argument surface
def test_reference_flag_surface_parses():
    from transformers import HfArgumentParser

    from dedloc_amd.cli.arguments import (AlbertTrainingArguments, CollaborationArguments, CoordinatorArguments,
                                          DatasetArguments)

    # albert/README.md-style trainer command line
    argv = ["--experiment_prefix", "albert", "--initial_peers", "1.2.3.4:1337", "5.6.7.8:1337",
            "--per_device_train_batch_size", "4", "--gradient_accumulation_steps", "2", "--target_batch_size", "4096",
            "--averaging_timeout", "120", "--bandwidth", "200", "--client_mode", "--batch_size_lead", "400",
            "--compression", "FLOAT16", "--statistics_expiration", "120", "--averaging_expiration", "10"]
    t, d, c = HfArgumentParser((AlbertTrainingArguments, DatasetArguments, CollaborationArguments)) \
        .parse_args_into_dataclasses(argv)
    assert c.initial_peers == ["1.2.3.4:1337", "5.6.7.8:1337"] and c.client_mode and c.bandwidth == 200.0
    assert c.target_group_size == 256 and c.metadata_expiration == 30 and c.performance_ema_alpha == 0.1
    assert t.learning_rate == 0.00176 and t.warmup_steps == 5000 and t.max_steps == 1_000_000
    assert t.clamp_value == 10000.0 and t.weight_decay == 0.01 and t.max_grad_norm == 1.0
    assert t.save_steps == 500 and t.save_total_limit == 2 and t.seed == 42
    (co,) = HfArgumentParser((CoordinatorArguments,)).parse_args_into_dataclasses(
        ["--experiment_prefix", "albert", "--refresh_period", "5"])
    assert co.refresh_period == 5 and co.save_checkpoint_step_interval == 5


# ----------------------------------------------------------------------------- access tokens (D14/H10)
def test_token_authorizer_and_authorized_records():
    from datetime import datetime, timedelta

    from dedloc_amd.dht.auth import (AccessToken, InvalidCredentialsError, LocalAuthority, LocalTokenAuthorizer,
                                     NotInAllowlistError)

    authority = LocalAuthority({"alice": "pw", "bob": "pw2"}, coordinator="127.0.0.1:4242", ttl=600)
    alice = LocalTokenAuthorizer(authority, "alice", "pw", RSAPrivateKey(bits=1024))
    tok = alice.get_token()
    assert tok.username == "alice" and alice.is_token_valid(tok) and alice.coordinator_port == 4242
    assert not alice.does_token_need_refreshing(tok)
    forged = AccessToken("mallory", tok.public_key, tok.expiration_time, tok.signature)
    assert not alice.is_token_valid(forged)
    old = (datetime.utcnow() - timedelta(seconds=5)).isoformat()
    expired = AccessToken("alice", tok.public_key, old)
    import base64
    expired.signature = base64.b64encode(authority.key.sign(expired.payload()))
    assert not alice.is_token_valid(expired)
    with pytest.raises(NotInAllowlistError):
        LocalTokenAuthorizer(authority, "eve", "x").join_experiment()
    with pytest.raises(InvalidCredentialsError):
        LocalTokenAuthorizer(authority, "bob", "wrong").join_experiment()

    # records written through an authorized DHT are visible to authorized readers; unauthorized
    # writers (no token) are invisible to them
    validators, pub = make_validators("auth")
    d_alice = DHT(start=True, record_validators=validators,
                  authorizer=LocalTokenAuthorizer(authority, "alice", "pw"))
    d_anon = DHT(initial_peers=[d_alice.endpoint], start=True)
    try:
        m = LocalMetrics(step=1, samples_per_second=1.0, samples_accumulated=1, loss=1.0, mini_steps=1)
        assert d_alice.store("auth_metrics", m.model_dump(), get_dht_time() + 30, subkey=pub)
        assert d_alice.get("auth_metrics", latest=True).value[pub].value["step"] == 1
        d_anon.store("plain_key", 7, get_dht_time() + 30)
        assert d_anon.get("plain_key").value == 7          # no validators on the anonymous node
        assert d_alice.get("plain_key") is None            # ... but the authorized node rejects it
    finally:
        d_anon.shutdown()
        d_alice.shutdown()
