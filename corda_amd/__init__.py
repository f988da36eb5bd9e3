"""corda_amd — MI355X-native batched Ed25519 verification + SHA-256 Merkle tx-id engine for Corda's
transaction-validation hot path (drop-in behind SignedTransaction.verifySignatures /
PublicKey.verifyWithECDSA / WireTransaction.id).  See DESIGN.md and include/cordaverify.h."""

from . import native  # noqa: F401

__all__ = ["native", "crypto", "transactions", "notary", "workload"]
