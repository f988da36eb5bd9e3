"""Uniqueness providers of the notary commit step (f4), CPU only.

Restates node/src/test/kotlin/net/corda/node/services/UniquenessProviderTests.kt and
PersistentUniquenessProviderTests.kt (commit of unused inputs; conflict on reuse reporting the
consuming tx id, input index and requesting party), then checks what the batched commit adds:
`commit_batch` decides exactly as the same sequence of `commit` calls (random batches with
intra-batch and cross-batch reuse, repeated inputs), the persistent store survives a reopen, and a
conflicting request commits nothing.
"""
import os
import random
import threading

import pytest

from corda_amd.transactions import SecureHash
from corda_amd.uniqueness import (ConsumingTx, InMemoryUniquenessProvider, PersistentUniquenessProvider,
                                  UniquenessConflict, UniquenessException)

MEGA_CORP = "MegaCorp"


def random_sha256(rng=random) -> SecureHash:
    return SecureHash(bytes(rng.getrandbits(8) for _ in range(32)))


def generate_state_ref(rng=random):
    """CoreTestUtils.kt:74: StateRef(SecureHash.randomSHA256(), 0)."""
    return (random_sha256(rng), 0)


@pytest.fixture(params=["memory", "persistent"])
def provider(request, tmp_path):
    if request.param == "memory":
        yield InMemoryUniquenessProvider()
    else:
        p = PersistentUniquenessProvider(str(tmp_path / "commit_log.db"))
        yield p
        p.close()


def test_should_commit_a_transaction_with_unused_inputs_without_exception(provider):
    provider.commit([generate_state_ref()], random_sha256(), MEGA_CORP)


def test_should_report_a_conflict_for_a_transaction_with_previously_used_inputs(provider):
    tx_id = random_sha256()
    input_state = generate_state_ref()
    inputs = [input_state]
    provider.commit(inputs, tx_id, MEGA_CORP)
    with pytest.raises(UniquenessException) as ei:
        provider.commit(inputs, tx_id, MEGA_CORP)
    consuming = ei.value.error.state_history[input_state]
    assert consuming.id == tx_id
    assert consuming.input_index == inputs.index(input_state)
    assert consuming.requesting_party == MEGA_CORP


def test_conflicting_commit_is_all_or_nothing(provider):
    a, b, c = (generate_state_ref() for _ in range(3))
    provider.commit([a], random_sha256(), "P1")
    with pytest.raises(UniquenessException) as ei:
        provider.commit([b, a, c], random_sha256(), "P2")
    assert list(ei.value.error.state_history) == [a]
    provider.commit([b, c], random_sha256(), "P3")       # b and c were not consumed by the failed call


def _sequential(reqs):
    ref = InMemoryUniquenessProvider()
    out = []
    for s, t, c in reqs:
        try:
            ref.commit(s, t, c)
            out.append(None)
        except UniquenessException as e:
            out.append(e.error)
    return ref, out


def test_batch_matches_sequential_commits(provider):
    rng = random.Random(20261017)
    pool = [generate_state_ref(rng) for _ in range(400)]
    reqs_all = []
    for _ in range(12):                                       # 12 batches of up to 120 requests
        batch = []
        for _ in range(rng.randint(1, 120)):
            k = rng.randint(1, 4)
            states = [rng.choice(pool) for _ in range(k)]     # may repeat a state inside one request
            batch.append((states, random_sha256(rng), f"party{rng.randint(0, 3)}"))
        reqs_all.append(batch)
    ref, want = _sequential([r for b in reqs_all for r in b])
    got = [c for b in reqs_all for c in provider.commit_batch(b)]
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert (g is None) == (w is None)
        if w is not None:
            assert g.state_history == w.state_history
    assert sum(c is None for c in got) > 10 and sum(c is not None for c in got) > 10
    # the stored consumer of every state equals the sequential provider's
    if isinstance(provider, PersistentUniquenessProvider):
        assert len(provider) == len(ref.committed)
        for s, c in ref.committed.items():
            assert provider.get(s) == c
    else:
        assert provider.committed == ref.committed


def test_repeated_input_last_index_wins(provider):
    s = generate_state_ref()
    t = random_sha256()
    provider.commit([s, generate_state_ref(), s], t, MEGA_CORP)
    with pytest.raises(UniquenessException) as ei:
        provider.commit([s], random_sha256(), MEGA_CORP)
    assert ei.value.error.state_history[s] == ConsumingTx(t, 2, MEGA_CORP)


def test_persistent_store_survives_reopen(tmp_path):
    path = str(tmp_path / "durable.db")
    p = PersistentUniquenessProvider(path)
    states = [generate_state_ref() for _ in range(50)]
    t = random_sha256()
    assert p.commit_batch([([s], t, "N") for s in states[:25]] + [(states[25:], t, "N")]) == [None] * 26
    p.close()
    q = PersistentUniquenessProvider(path)
    assert len(q) == 50
    res = q.commit_batch([([states[3]], random_sha256(), "X"), ([generate_state_ref()], random_sha256(), "Y")])
    assert res[0] is not None and res[0].state_history[states[3]] == ConsumingTx(t, 0, "N")
    assert res[1] is None
    q.close()


def test_conflict_report_round_trip():
    s1, s2 = generate_state_ref(), (b"leaf-bytes", 7)
    c = UniquenessConflict({s1: ConsumingTx(random_sha256(), 1, "A"), s2: ConsumingTx(random_sha256(), 0, "B")})
    assert UniquenessConflict.deserialize(c.serialize()) == c


def test_persistent_concurrent_batches_never_double_spend(tmp_path):
    p = PersistentUniquenessProvider(str(tmp_path / "race.db"))
    pool = [generate_state_ref() for _ in range(64)]
    wins = []
    lock = threading.Lock()

    def worker(seed):
        rng = random.Random(seed)
        got = p.commit_batch([([rng.choice(pool)], random_sha256(rng), f"w{seed}") for _ in range(40)])
        with lock:
            wins.extend(c is None for c in got)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert sum(wins) == len(p) <= len(pool)        # every state consumed at most once
    p.close()


def test_failed_commit_reports_its_own_error(tmp_path):
    """when COMMIT itself fails (a disk / fsync error) SQLite has already rolled the
    transaction back; commit_batch must re-raise THAT error (not "no transaction is active" from a
    second ROLLBACK), and nothing of the batch is stored."""
    import sqlite3
    p = PersistentUniquenessProvider(str(tmp_path / "failing.db"))
    real = p._db

    class FailingCommit:
        def __getattr__(self, name):
            return getattr(real, name)

        def execute(self, sql, *a):
            if sql == "COMMIT":
                real.execute("ROLLBACK")
                raise sqlite3.OperationalError("disk I/O error")
            return real.execute(sql, *a)

    p._db = FailingCommit()
    with pytest.raises(sqlite3.OperationalError, match="disk I/O error"):
        p.commit_batch([([generate_state_ref()], random_sha256(), "N")])
    p._db = real
    assert len(p) == 0
    assert p.commit_batch([([generate_state_ref()], random_sha256(), "N")]) == [None]
    p.close()
