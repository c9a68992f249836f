"""Checkpoint stores: protocol, in-memory, CQL (Scylla / Astra)."""
from .base import CheckpointStore, StoreError
from .memory import MemoryStore

__all__ = ["CheckpointStore", "StoreError", "MemoryStore"]
