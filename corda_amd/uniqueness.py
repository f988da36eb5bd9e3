"""Uniqueness providers of the notary commit step.

The reference commits the inputs of ONE transaction per notary flow:
  UniquenessProvider.commit(states, txId, callerIdentity)   core/.../node/services/UniquenessProvider.kt:15
  InMemoryUniquenessProvider                                node/.../transactions/InMemoryUniquenessProvider.kt
  PersistentUniquenessProvider (RDBMS, ThreadBox-locked)    node/.../transactions/PersistentUniquenessProvider.kt:19-81
    committedStates: StateRef -> ConsumingTx(id, inputIndex, requestingParty), table
    "node_notary_commit_log"; commit: under the lock, collect every input already in the map (in
    input order) -> UniquenessException(Conflict(those)); otherwise put(state, ConsumingTx(txId, i,
    caller)) for every input (a repeated input is re-put: the last index wins).

`commit_batch(requests)` is the batched commit of a verified notary batch: the requests are decided
in request order, exactly as that many sequential `commit` calls would decide them (a request
conflicts with states committed by an EARLIER request of the same batch, never a later one, and a
conflicting request commits nothing), but the persistent provider does it in ONE database
transaction — one lock acquisition and one durable commit (fsync) per batch instead of per
transaction.  Each result is None (committed) or the UniquenessConflict the sequential call would
have raised.

The node's JDBC/H2 store is out of scope; the persistent provider keeps the
reference's table and columns on SQLite (Python's sqlite3, synchronous=FULL, WAL journal), keyed by
the canonical encoding of the state reference.
"""
from __future__ import annotations

import sqlite3
import struct
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from .crypto import IllegalArgumentException
from .transactions import SecureHash


@dataclass(frozen=True)
class ConsumingTx:
    """UniquenessProvider.ConsumingTx(id, inputIndex, requestingParty) (UniquenessProvider.kt:31)."""
    id: SecureHash
    input_index: int
    requesting_party: str


def _enc(x) -> bytes:
    """Canonical tagged encoding of the state references and parties a conflict report carries and
    the persistent provider keys its rows by (the reference's Kryo serialization is out of scope)."""
    if isinstance(x, SecureHash):
        return b"H" + x.bytes
    if isinstance(x, (bytes, bytearray)):
        return b"B" + struct.pack("<I", len(x)) + bytes(x)
    if isinstance(x, str):
        b = x.encode()
        return b"S" + struct.pack("<I", len(b)) + b
    if isinstance(x, bool) or not isinstance(x, (int, tuple, list)):
        raise IllegalArgumentException(f"cannot serialize {type(x).__name__}")
    if isinstance(x, int):
        return b"I" + struct.pack("<q", x)
    return b"T" + struct.pack("<I", len(x)) + b"".join(_enc(v) for v in x)


def _dec(b: bytes, p: int):
    t = b[p:p + 1]
    p += 1
    if t == b"H":
        return SecureHash(b[p:p + 32]), p + 32
    if t in (b"B", b"S"):
        (m,) = struct.unpack_from("<I", b, p)
        v = b[p + 4:p + 4 + m]
        return (bytes(v) if t == b"B" else v.decode()), p + 4 + m
    if t == b"I":
        return struct.unpack_from("<q", b, p)[0], p + 8
    if t == b"T":
        (m,) = struct.unpack_from("<I", b, p)
        p += 4
        out = []
        for _ in range(m):
            v, p = _dec(b, p)
            out.append(v)
        return tuple(out), p
    raise IllegalArgumentException("malformed conflict encoding")


@dataclass
class UniquenessConflict:
    """UniquenessProvider.Conflict(stateHistory): the consuming transaction of every conflicting state."""
    state_history: Dict[object, ConsumingTx]

    def serialize(self) -> bytes:
        rows = sorted((_enc(s), c) for s, c in self.state_history.items())
        return b"CONFLICT" + _enc(tuple((s_enc, c.id, c.input_index, c.requesting_party) for s_enc, c in rows))

    @staticmethod
    def deserialize(raw: bytes) -> "UniquenessConflict":
        if not raw.startswith(b"CONFLICT"):
            raise IllegalArgumentException("not a conflict report")
        rows, _ = _dec(raw, 8)
        return UniquenessConflict({_dec(s_enc, 0)[0]: ConsumingTx(h, i, party) for s_enc, h, i, party in rows})


class UniquenessException(Exception):
    """UniquenessException(error: Conflict) (UniquenessProvider.kt:34)."""

    def __init__(self, conflict: UniquenessConflict):
        super().__init__("conflict")
        self.error = conflict


CommitRequest = Tuple[Sequence[object], SecureHash, str]     # (input states, tx id, caller identity)


class InMemoryUniquenessProvider:
    """InMemoryUniquenessProvider.kt semantics: all-or-nothing commit under one lock."""

    def __init__(self):
        self.committed: Dict[object, ConsumingTx] = {}
        self._lock = threading.Lock()

    def _commit_locked(self, states, tx_id, caller) -> Optional[UniquenessConflict]:
        conflict = {s: self.committed[s] for s in states if s in self.committed}
        if conflict:
            return UniquenessConflict(conflict)
        for i, s in enumerate(states):
            self.committed[s] = ConsumingTx(tx_id, i, caller)
        return None

    def commit(self, states: Sequence[object], tx_id: SecureHash, caller: str) -> None:
        with self._lock:
            c = self._commit_locked(states, tx_id, caller)
        if c is not None:
            raise UniquenessException(c)

    def commit_batch(self, requests: Sequence[CommitRequest]) -> List[Optional[UniquenessConflict]]:
        with self._lock:
            return [self._commit_locked(s, t, c) for s, t, c in requests]


class PersistentUniquenessProvider:
    """PersistentUniquenessProvider.kt:19-81 on SQLite: table node_notary_commit_log, one row per
    consumed state (state reference -> consuming transaction id, input index, requesting party).
    Thread-safe (one connection behind a lock, as the reference's ThreadBox); every commit or batch
    is one IMMEDIATE transaction, durable when it returns (synchronous=FULL)."""

    TABLE = "node_notary_commit_log"

    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()
        self._db = sqlite3.connect(path, isolation_level=None, check_same_thread=False)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("PRAGMA synchronous=FULL")
        self._db.execute(f"CREATE TABLE IF NOT EXISTS {self.TABLE} ("
                         "output BLOB PRIMARY KEY, consuming_transaction_id BLOB NOT NULL, "
                         "consuming_input_index INTEGER NOT NULL, requesting_party_name TEXT NOT NULL)")

    def close(self) -> None:
        with self._lock:
            self._db.close()

    def __len__(self) -> int:
        with self._lock:
            return self._db.execute(f"SELECT COUNT(*) FROM {self.TABLE}").fetchone()[0]

    def get(self, state) -> Optional[ConsumingTx]:
        with self._lock:
            r = self._db.execute(f"SELECT consuming_transaction_id, consuming_input_index, requesting_party_name "
                                 f"FROM {self.TABLE} WHERE output = ?", (_enc(state),)).fetchone()
        return None if r is None else ConsumingTx(SecureHash(bytes(r[0])), int(r[1]), r[2])

    def _lookup(self, keys: List[bytes]) -> Dict[bytes, ConsumingTx]:
        found: Dict[bytes, ConsumingTx] = {}
        for j in range(0, len(keys), 500):                  # SQLite's bound-parameter limit
            part = keys[j:j + 500]
            q = (f"SELECT output, consuming_transaction_id, consuming_input_index, requesting_party_name "
                 f"FROM {self.TABLE} WHERE output IN ({','.join('?' * len(part))})")
            for out, h, i, party in self._db.execute(q, part):
                found[bytes(out)] = ConsumingTx(SecureHash(bytes(h)), int(i), party)
        return found

    def _decide(self, requests: Sequence[CommitRequest]) -> Tuple[List[Optional[UniquenessConflict]], list]:
        """Sequential decisions of the batch against the store plus the batch's own earlier commits."""
        keyed = [[_enc(s) for s in states] for states, _, _ in requests]
        stored = self._lookup(sorted({k for ks in keyed for k in ks}))
        pending: Dict[bytes, ConsumingTx] = {}
        out: List[Optional[UniquenessConflict]] = []
        rows = []
        for (states, tx_id, caller), ks in zip(requests, keyed):
            conflict = {}
            for s, k in zip(states, ks):
                c = pending.get(k) or stored.get(k)
                if c is not None:
                    conflict[s] = c
            if conflict:
                out.append(UniquenessConflict(conflict))
                continue
            for i, k in enumerate(ks):                      # put(): a repeated input is re-put, last index wins
                pending[k] = ConsumingTx(tx_id, i, caller)
            rows.extend((k, tx_id.bytes, i, caller) for i, k in enumerate(ks))
            out.append(None)
        return out, rows

    def commit_batch(self, requests: Sequence[CommitRequest]) -> List[Optional[UniquenessConflict]]:
        with self._lock:
            self._db.execute("BEGIN IMMEDIATE")
            try:
                out, rows = self._decide(requests)
                self._db.executemany(f"INSERT OR REPLACE INTO {self.TABLE} VALUES (?, ?, ?, ?)", rows)
                self._db.execute("COMMIT")
            except BaseException:
                # a failed COMMIT (disk / fsync error) may already have rolled back: a second ROLLBACK
                # would raise "no transaction is active" and replace the error the notary must report
                if self._db.in_transaction:
                    try:
                        self._db.execute("ROLLBACK")
                    except Exception:  # noqa: BLE001 - the original exception is the one to report
                        pass
                raise
        return out

    def commit(self, states: Sequence[object], tx_id: SecureHash, caller: str) -> None:
        (c,) = self.commit_batch([(states, tx_id, caller)])
        if c is not None:
            raise UniquenessException(c)
